"""Optional NER detector (BASELINE.json configs[4]): BERT-base token classification in
bf16 on the MI355X matrix cores (csrc/ner.hip -> libner.so), a PERSON_NAME detector beside the rule
engine.  The reference has no such detector; its hotword rule "full name|your name"
(main_service/dlp_config.yaml:170) asks for one.

The model is ``transformers.BertConfig()`` (bert-base shapes) with seeded random weights built locally
(nothing is fetched), so the parity target is the HF model itself run in fp32 on
the CPU: same token ids in, logits compared within a bf16 tolerance (tests/test_ner.py).  With no
vocabulary file available offline, ``HashTokenizer`` maps lower-cased word / punctuation tokens onto
the vocabulary by a 64-bit FNV-1a hash; token character offsets map labels back to spans.

GPU forward (one call per op, all on the current torch stream; torch only allocates):
    embed+LN -> 12 x [QKV GEMM -> attention -> out GEMM(+residual) -> LN -> FFN1 GEMM(+GELU)
    -> FFN2 GEMM(+residual) -> LN] -> classifier
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NER_LIB = os.environ.get("PII_NER_LIB") or os.path.join(HERE, "libner.so")
LABELS = ["O", "B-PERSON_NAME", "I-PERSON_NAME"]
EPI_BIAS, EPI_GELU, EPI_RESID = 0, 1, 2
LIKELY = 4                  # likelihood of a PERSON_NAME finding (DLP scale)
CLS, SEP, PAD = 101, 102, 0

_LIB = None


def load_library(path: str = NER_LIB) -> ctypes.CDLL:
    """the process-wide libner.so (loaded once; PII_NER_LIB selects another build)"""
    global _LIB
    if _LIB is None:
        _LIB = open_library(path)
    return _LIB


def open_library(path: str) -> ctypes.CDLL:
    """a libner.so build with its signatures declared, not cached (A/B timing of several builds)"""
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run __graft_entry__.build() (no CPU fallback exists)")
    import torch  # noqa: F401  (one HIP runtime for torch and the library)
    lib = ctypes.CDLL(path)
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.ner_gemm.argtypes = [P, P, P, P, P, I, I, I, I, P]
    lib.ner_layernorm.argtypes = [P, P, P, P, I, I, F, P]
    lib.ner_embed.argtypes = [P, P, P, P, P, P, P, I, I, I, F, P]
    lib.ner_attention.argtypes = [P, P, P, I, I, I, I, P]
    lib.ner_classify.argtypes = [P, P, P, P, I, I, I, P]
    lib.ner_tokenize.argtypes = [P, P, I, I, I, P, P, P, P, P, P]
    lib.ner_spans.argtypes = [P, I, P, P, P, I, I, I, I, P, P, P]
    for n in ("ner_gemm", "ner_layernorm", "ner_embed", "ner_attention", "ner_classify", "ner_tokenize", "ner_spans"):
        getattr(lib, n).restype = ctypes.c_int
    return lib


# ------------------------------------------------------------------------------------ tokenizer
_TOKEN = re.compile(rb"[A-Za-z0-9_]+|[^\sA-Za-z0-9_]")


def _fnv1a64(b: bytes) -> int:
    h = 0xcbf29ce484222325
    for c in b:
        h = ((h ^ c) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


class HashTokenizer:
    """Lower-cased word / punctuation tokens, id = 1000 + fnv1a64(token) mod (vocab - 1000);
    [CLS] text [SEP] [PAD]..., with each token's byte span in the text."""

    def __init__(self, vocab_size: int = 30522, max_len: int = 128):
        self.vocab_size, self.max_len = vocab_size, max_len

    def encode(self, text: bytes) -> Tuple[List[int], List[Tuple[int, int]]]:
        ids, spans = [CLS], [(0, 0)]
        for m in _TOKEN.finditer(text):
            if len(ids) >= self.max_len - 1:
                break
            ids.append(1000 + _fnv1a64(m.group().lower()) % (self.vocab_size - 1000))
            spans.append((m.start(), m.end()))
        ids.append(SEP)
        spans.append((0, 0))
        return ids, spans

    def batch(self, texts: Sequence[bytes]):
        """(ids int32 [B, max_len], mask int32 [B, max_len], spans per text)"""
        B, S = len(texts), self.max_len
        ids = np.full((B, S), PAD, dtype=np.int32)
        mask = np.zeros((B, S), dtype=np.int32)
        spans = []
        for i, t in enumerate(texts):
            x, sp = self.encode(t)
            ids[i, :len(x)] = x
            mask[i, :len(x)] = 1
            spans.append(sp)
        return ids, mask, spans


def decode_spans(labels: Sequence[int], spans: Sequence[Tuple[int, int]]) -> List[Tuple[int, int]]:
    """BIO labels (LABELS order) over tokens -> merged PERSON_NAME byte spans ([CLS]/[SEP] skipped)"""
    out: List[Tuple[int, int]] = []
    cur = None
    for lab, (s, e) in zip(labels, spans):
        if e <= s:                       # special token
            if cur:
                out.append(cur)
            cur = None
            continue
        if lab == 1 or (lab == 2 and cur is None):
            if cur:
                out.append(cur)
            cur = (s, e)
        elif lab == 2:
            cur = (cur[0], e)
        else:
            if cur:
                out.append(cur)
            cur = None
    if cur:
        out.append(cur)
    return out


# ------------------------------------------------------------------------------------ model
def reference_model(seed: int = 0, num_labels: int = 3):
    """The HF BertForTokenClassification the GPU model is built from (fp32, CPU, eval mode)."""
    import torch
    from transformers import BertConfig, BertForTokenClassification
    cfg = BertConfig()
    cfg.num_labels = num_labels
    torch.manual_seed(seed)
    return BertForTokenClassification(cfg).eval()


class BertNer:
    """bf16 BERT-base token classifier on one GPU (weights copied from an HF model)."""

    def __init__(self, model=None, device: int = 0, seed: int = 0, num_labels: int = 3):
        import torch
        self.torch = torch
        self.lib = load_library()
        model = model if model is not None else reference_model(seed, num_labels)
        cfg = model.config
        if cfg.hidden_size // cfg.num_attention_heads != 64 or cfg.hidden_act != "gelu":
            raise ValueError("the GPU kernels implement head size 64 and exact GELU (BertConfig defaults)")
        self.H, self.heads, self.L = cfg.hidden_size, cfg.num_attention_heads, cfg.num_labels
        self.vocab = cfg.vocab_size
        self.eps = float(cfg.layer_norm_eps)
        self.dev = torch.device("cuda", device)
        sd = {k: v.detach().float() for k, v in model.state_dict().items()}
        bf = lambda t: t.to(self.dev, dtype=torch.bfloat16).contiguous()        # noqa: E731
        f32 = lambda t: t.to(self.dev, dtype=torch.float32).contiguous()        # noqa: E731
        p = "bert.embeddings."
        self.wemb, self.pemb = bf(sd[p + "word_embeddings.weight"]), bf(sd[p + "position_embeddings.weight"])
        self.temb = bf(sd[p + "token_type_embeddings.weight"][0])
        self.eg, self.eb = f32(sd[p + "LayerNorm.weight"]), f32(sd[p + "LayerNorm.bias"])
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            q = f"bert.encoder.layer.{i}."
            a = q + "attention."
            self.layers.append(dict(
                wqkv=bf(torch.cat([sd[a + "self.query.weight"], sd[a + "self.key.weight"], sd[a + "self.value.weight"]])),
                bqkv=f32(torch.cat([sd[a + "self.query.bias"], sd[a + "self.key.bias"], sd[a + "self.value.bias"]])),
                wo=bf(sd[a + "output.dense.weight"]), bo=f32(sd[a + "output.dense.bias"]),
                g1=f32(sd[a + "output.LayerNorm.weight"]), b1=f32(sd[a + "output.LayerNorm.bias"]),
                wi=bf(sd[q + "intermediate.dense.weight"]), bi=f32(sd[q + "intermediate.dense.bias"]),
                wf=bf(sd[q + "output.dense.weight"]), bf=f32(sd[q + "output.dense.bias"]),
                g2=f32(sd[q + "output.LayerNorm.weight"]), b2=f32(sd[q + "output.LayerNorm.bias"])))
        self.wc, self.bc = bf(sd["classifier.weight"]), f32(sd["classifier.bias"])
        self.inter = self.layers[0]["wi"].shape[0]
        self._bufs = {}

    # -------------------------------------------------------------- ops (device pointers, current stream)
    def _st(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc})")

    def gemm(self, a, w, bias, out, epi=EPI_BIAS, resid=None):
        M, K = a.shape
        N = w.shape[0]
        self._check(self.lib.ner_gemm(a.data_ptr(), w.data_ptr(), bias.data_ptr() if bias is not None else None,
                                      resid.data_ptr() if resid is not None else None, out.data_ptr(), M, N, K, epi,
                                      self._st()), "ner_gemm")
        return out

    def layernorm(self, x, g, b, out):
        M, H = x.shape
        self._check(self.lib.ner_layernorm(x.data_ptr(), g.data_ptr(), b.data_ptr(), out.data_ptr(), M, H, self.eps,
                                           self._st()), "ner_layernorm")
        return out

    def _buffers(self, Mp):
        if Mp not in self._bufs:
            t, bf = self.torch, self.torch.bfloat16
            z = lambda n: t.zeros((Mp, n), dtype=bf, device=self.dev)          # noqa: E731
            self._bufs[Mp] = dict(h=z(self.H), h1=z(self.H), a=z(self.H), ctx=z(self.H), qkv=z(3 * self.H),
                                  f=z(self.inter), ids=t.zeros(Mp, dtype=t.int32, device=self.dev),
                                  logits=t.zeros((Mp, self.L), dtype=t.float32, device=self.dev))
        return self._bufs[Mp]

    def forward(self, ids, mask):
        """ids, mask: int32 [B, S] (host numpy or device tensors) -> logits f32 [B, S, L] (device)"""
        t = self.torch
        ids = t.as_tensor(ids, dtype=t.int32).to(self.dev)
        mask = t.as_tensor(mask, dtype=t.int32).to(self.dev).contiguous()
        B, S = ids.shape
        M = B * S
        Mp = (M + 127) // 128 * 128
        bu = self._buffers(Mp)
        bu["ids"][:M] = ids.reshape(-1)
        # a copy: the buffer is reused by the next forward of the same padded size
        return self._forward_ids(bu, mask, B, S).reshape(B, S, self.L).clone()

    def _forward_ids(self, bu, mask, B, S):
        """the 12-layer forward over bu["ids"][:B*S] -> logits [B*S, L] (a view of the buffer)"""
        M = B * S
        Mp = bu["h"].shape[0]
        st = self._st()
        h, h1, a, ctx, qkv, f = bu["h"], bu["h1"], bu["a"], bu["ctx"], bu["qkv"], bu["f"]
        self._check(self.lib.ner_embed(bu["ids"].data_ptr(), self.wemb.data_ptr(), self.pemb.data_ptr(),
                                       self.temb.data_ptr(), self.eg.data_ptr(), self.eb.data_ptr(), h.data_ptr(),
                                       Mp, S, self.H, self.eps, st), "ner_embed")
        for Ly in self.layers:
            self.gemm(h, Ly["wqkv"], Ly["bqkv"], qkv)
            self._check(self.lib.ner_attention(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), B, S, self.heads, 64,
                                               st), "ner_attention")
            self.gemm(ctx, Ly["wo"], Ly["bo"], a, EPI_RESID, resid=h)
            self.layernorm(a, Ly["g1"], Ly["b1"], h1)
            self.gemm(h1, Ly["wi"], Ly["bi"], f, EPI_GELU)
            self.gemm(f, Ly["wf"], Ly["bf"], a, EPI_RESID, resid=h1)
            self.layernorm(a, Ly["g2"], Ly["b2"], h)
        self._check(self.lib.ner_classify(h.data_ptr(), self.wc.data_ptr(), self.bc.data_ptr(),
                                          bu["logits"].data_ptr(), Mp, self.H, self.L, st), "ner_classify")
        return bu["logits"][:M]

    def flops_per_token(self, S: int) -> float:
        H, I = self.H, self.inter
        gemm = 2 * (H * 3 * H + H * H + 2 * H * I)
        attn = 4 * S * H
        return len(self.layers) * (gemm + attn) + 2 * H * self.L

    # -------------------------------------------------------------- detector
    def detect(self, texts: Sequence[bytes], tokenizer: Optional[HashTokenizer] = None):
        """PERSON_NAME byte spans per text (argmax labels, BIO-merged)"""
        tok = tokenizer or HashTokenizer()
        ids, mask, spans = tok.batch(texts)
        lab = self.forward(ids, mask).argmax(-1).cpu().numpy()
        return [decode_spans(lab[i], spans[i]) for i in range(len(texts))]

    def detect_device(self, d_text, d_offs, n_rows: int, S: int = 64, info_type: int = 0,
                      likelihood: int = LIKELY):
        """The whole detector on the GPU, for rows already in HBM (d_text / d_offs: device pointers of
        the engine's batch layout, offsets relative to d_text): tokenize (k_tokenize = HashTokenizer
        with max_len S) -> bf16 BERT forward -> argmax + BIO decode (k_ner_spans = decode_spans) ->
        the engine's external candidates.  Returns (ext, ext_n, stride) device tensors for
        Engine.scan_redact_device_ext; nothing is copied to the host.  Rows past S - 2 tokens are
        truncated, as HashTokenizer does."""
        t = self.torch
        if S % 32 or S > 128:
            raise ValueError("S must be a multiple of 32, at most 128 (the matrix-core attention)")
        st = self._st()
        M = n_rows * S
        Mp = (M + 127) // 128 * 128
        bu = self._buffers(Mp)
        i32 = dict(dtype=t.int32, device=self.dev)
        mask = t.empty(M, **i32)
        lo = t.empty(M, dtype=t.int32, device=self.dev)
        hi = t.empty(M, dtype=t.int32, device=self.dev)
        ntok = t.empty(n_rows, **i32)
        self._check(self.lib.ner_tokenize(d_text, d_offs, n_rows, S, self.vocab, bu["ids"].data_ptr(),
                                          mask.data_ptr(), lo.data_ptr(), hi.data_ptr(), ntok.data_ptr(), st),
                    "ner_tokenize")
        logits = self._forward_ids(bu, mask.view(n_rows, S), n_rows, S)
        ext = t.empty((n_rows * S, 4), dtype=t.int32, device=self.dev)      # pii_span rows (16 B)
        ext_n = t.empty(n_rows, **i32)
        self._check(self.lib.ner_spans(logits.data_ptr(), self.L, lo.data_ptr(), hi.data_ptr(), ntok.data_ptr(),
                                       n_rows, S, info_type, likelihood, ext.data_ptr(), ext_n.data_ptr(), st),
                    "ner_spans")
        return ext, ext_n, S

    def ext_candidates(self, texts: Sequence[bytes], info_type: int, likelihood: int = LIKELY,
                       max_len: int = 64):
        """Host form for Engine.scan_redact(..., ext=): per text [(start, end, info_type, likelihood)]"""
        return [[(s, e, info_type, likelihood) for s, e in sp]
                for sp in self.detect(texts, HashTokenizer(self.vocab, max_len))]
