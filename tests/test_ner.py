"""Optional NER detector: bf16 BERT-base token classification on MFMA
(csrc/ner.hip) vs the same HF model in fp32 on the CPU (transformers.BertConfig(), seeded random
weights, nothing fetched).  Tolerances are bf16's: per op against a torch fp32 computation on the
bf16-rounded inputs, and for the whole 12-layer model on the logits (relative L2 error and argmax
agreement)."""
import numpy as np
import pytest

from conftest import pkg


def test_tokenizer_and_span_decoding():
    N = pkg("ner")
    tok = N.HashTokenizer(max_len=16)
    ids, spans = tok.encode(b"My name is John Smith, ok?")
    assert ids[0] == N.CLS and ids[-1] == N.SEP and len(ids) == len(spans)
    assert [b"My name is John Smith, ok?"[s:e] for s, e in spans[1:-1]] == [b"My", b"name", b"is", b"John", b"Smith",
                                                                           b",", b"ok", b"?"]
    assert tok.encode(b"JOHN")[0][1] == tok.encode(b"john")[0][1]               # case-folded
    assert all(1000 <= i < 30522 for i in ids[1:-1])
    B, M, S = tok.batch([b"a b", b"x" * 3 + b" y" * 40])
    assert B.shape == (2, 16) and M[0].sum() == 4 and M[1].sum() == 16         # truncated to max_len
    # BIO: [CLS] My name is John Smith , ok ? [SEP]
    lab = [0, 0, 0, 0, 1, 2, 0, 0, 0, 0]
    assert N.decode_spans(lab, spans) == [(11, 21)]
    assert N.decode_spans([0, 2, 2, 0, 1, 1, 0, 0, 0, 0], spans) == [(0, 7), (11, 15), (16, 21)]


@pytest.fixture(scope="module")
def ner_model():
    N = pkg("ner")
    ref = N.reference_model(seed=3)
    return ref, N.BertNer(ref, device=0)


def _bf(x):
    import torch
    return x.to(torch.bfloat16).float()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 192), (1024, 2304, 768), (512, 768, 3072)])
def test_gemm_vs_torch(ner_model, M, N, K):
    import torch
    Nm = pkg("ner")
    _, m = ner_model
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    dev = m.dev
    Ab, Wb, Rb = (x.to(dev, torch.bfloat16) for x in (A, W, R))
    ref = _bf(A) @ _bf(W).T + bias
    for epi in (Nm.EPI_BIAS, Nm.EPI_GELU, Nm.EPI_RESID):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        m.gemm(Ab, Wb, bias.to(dev), out, epi, resid=Rb if epi == Nm.EPI_RESID else None)
        want = ref if epi == Nm.EPI_BIAS else (torch.nn.functional.gelu(ref) if epi == Nm.EPI_GELU else ref + _bf(R))
        got = out.float().cpu()
        err = (got - want).abs().max().item()
        assert err <= 0.02 * want.abs().max().item() + 1e-2, (epi, err)       # bf16 output rounding


@pytest.mark.gpu
def test_layernorm_and_attention_vs_torch(ner_model):
    import torch
    _, m = ner_model
    dev = m.dev
    g = torch.Generator().manual_seed(5)
    x = torch.randn(256, 768, generator=g) * 3 + 1
    gam, bet = torch.randn(768, generator=g), torch.randn(768, generator=g)
    out = torch.empty(256, 768, dtype=torch.bfloat16, device=dev)
    m.layernorm(x.to(dev, torch.bfloat16), gam.to(dev), bet.to(dev), out)
    want = torch.nn.functional.layer_norm(_bf(x), (768,), gam, bet, eps=m.eps)
    assert (out.float().cpu() - want).abs().max().item() < 0.05
    # attention over the fused QKV rows, with padded keys masked: the matrix-core kernel (S % 32 == 0,
    # S <= 128) and the general one
    for B, S in ((2, 64), (3, 128), (2, 48), (1, 160)):
        Hh = 12
        qkv = torch.randn(B * S, 3 * 768, generator=g)
        mask = torch.ones(B, S, dtype=torch.int32)
        mask[-1, S * 5 // 8:] = 0
        ctx = torch.zeros(B * S, 768, dtype=torch.bfloat16, device=dev)
        rc = m.lib.ner_attention(qkv.to(dev, torch.bfloat16).data_ptr(), mask.to(dev).data_ptr(), ctx.data_ptr(), B, S,
                                 Hh, 64, m._st())
        assert rc == 0
        q, k, v = (_bf(qkv).reshape(B, S, 3, Hh, 64)[:, :, i].transpose(1, 2) for i in range(3))
        sc = q @ k.transpose(-1, -2) / 8.0 + (1 - mask[:, None, None, :].float()) * -1e30
        want = (sc.softmax(-1) @ v).transpose(1, 2).reshape(B * S, 768)
        assert (ctx.float().cpu() - want).abs().max().item() < 0.03, S


@pytest.mark.gpu
def test_bert_logits_vs_hf_cpu(ner_model):
    """the whole 12-layer model vs HF fp32 on the CPU, same ids and mask (ragged lengths)"""
    import torch
    Nm = pkg("ner")
    ref, m = ner_model
    tok = Nm.HashTokenizer(max_len=64)
    texts = [b"my name is john smith and i live on main street", b"ok", b"please call jane doe at home " * 3,
             b"the account holder is Maria Garcia-Lopez, date of birth 01/02/1980"]
    ids, mask, _ = tok.batch(texts)
    got = m.forward(ids, mask).float().cpu()
    with torch.no_grad():
        want = ref(input_ids=torch.as_tensor(ids, dtype=torch.long),
                   attention_mask=torch.as_tensor(mask, dtype=torch.long)).logits
    sel = torch.as_tensor(mask, dtype=torch.bool)
    g, w = got[sel], want[sel]
    rel = ((g - w).norm() / w.norm()).item()
    agree = (g.argmax(-1) == w.argmax(-1)).float().mean().item()
    assert rel < 0.05 and agree > 0.9, (rel, agree)
