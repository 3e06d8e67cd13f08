"""The optional NER on the redaction path: PERSON_NAME spans enter the engine as
EXTERNAL candidates (include/pii_engine.h pii_scan_redact_ext / pii_scan_redact_device_ext) and take
part in overlap resolution (A.6) with the rule findings, so they reach the span list, the redacted
bytes ("[PERSON_NAME]") and the histogram.

Checkers:
* the merge: engine with external candidates vs ``oracle.process_rows(rows, extra=...)`` with the
  SAME candidates -- bit-exact (bytes, spans, context), including long rows cut over many lanes;
* the detector front / back end on the GPU (k_tokenize, k_ner_spans) vs ner.py's HashTokenizer and
  decode_spans -- exact;
* the whole device detector (tokenize -> bf16 BERT on MFMA -> decode -> engine) vs oracle + the same
  seeded HF model in fp32 on the CPU.  bf16 and fp32 logits differ by rounding, so a token whose fp32
  top-two logit margin is below NER_MARGIN may take the other label (test_ner.py's logit tolerance);
  every other token's label must agree, and every row whose tokens all clear the margin must be
  redacted exactly as oracle + HF redacts it.  The engine output is always bit-exact against the
  oracle fed the GPU's own spans.
The seeded random weights make the labels meaningless as names (nothing is fetched); the point is the
pipeline and its parity."""
import random

import numpy as np
import pytest

from conftest import pkg

NER_MARGIN = 0.1          # |fp32 top1 - top2| below which bf16 may pick the other label


def _spans_of(res, i):
    m = res.spans["utt"] == i
    return [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]


def _random_ext(r, text, person, types, n_max=4):
    """sorted-by-start candidates: mostly PERSON_NAME, some of other types; some below min_likelihood,
    some 1 byte, some overlapping each other and the rule findings"""
    out = []
    L = len(text)
    if L == 0:
        return out
    for _ in range(r.randrange(0, n_max + 1)):
        s = r.randrange(0, L)
        e = min(L, s + r.choice([1, 2, 5, 9, 14, 30]))
        t = person if r.random() < 0.8 else r.choice(types)
        out.append((s, e, t, r.choice([2, 3, 4, 4, 5])))
    out.sort(key=lambda x: x[0])
    return out


def test_oracle_extra_candidates_follow_overlap_resolution(oracle_cfg):
    from oracle import pii_oracle as O
    P = oracle_cfg.type_id["PERSON_NAME"]
    assert oracle_cfg.type_names[-1] == "PERSON_NAME"
    t = b"I am John Smith, email jsmith@example.com thanks"
    # a name candidate overlapping the email: the longer candidate at the same start wins; a
    # candidate starting inside a kept finding is dropped; below min_likelihood (POSSIBLE) is dropped
    assert len(t) == 48 and t[23:41] == b"jsmith@example.com"
    red, fs = O.redact(t, oracle_cfg, None, [(5, 15, P, 4), (23, 29, P, 5), (30, 35, P, 5), (42, 48, P, 2)])
    assert red == b"I am [PERSON_NAME], email [EMAIL_ADDRESS] thanks"
    red, _ = O.redact(t, oracle_cfg, None, [(23, 48, P, 4)])            # covers the email: longer wins
    assert red == b"I am John Smith, email [PERSON_NAME]"


def test_ext_arrays_layout():
    E = pkg("engine")
    spans, counts, stride = E.ext_arrays([[(0, 3, 22, 4)], [], [(1, 2, 22, 5), (4, 9, 22, 4)]], 3)
    assert stride == 2 and list(counts) == [1, 0, 2]
    assert spans["start"][4] == 1 and spans["end"][5] == 9 and spans["likelihood"][5] == 4


@pytest.fixture(scope="module")
def eng(compiled):
    E = pkg("engine")
    e = E.Engine(compiled.blob, device=0, n_conv_slots=1 << 14)
    yield e
    e.close()


def _rows(seed, n_conv, per_conv, long_every=0):
    """synthetic conversations (the config-2 generator) with names spliced in; every `long_every`-th
    row is a whole-transcript-sized row (cut over several scan lanes)"""
    synth = pkg("synth")
    from oracle import pii_oracle as O
    r = random.Random(seed)
    bank = synth.build_bank(400, 400, seed=seed)
    rows = []
    k = 0
    for c in range(n_conv):
        for j in range(per_conv):
            role = O.ROLE_AGENT if j % 2 == 0 else O.ROLE_CUSTOMER
            base = r.choice(bank.texts[:400] if role == O.ROLE_AGENT else bank.texts[400:])
            name = f"{r.choice(synth.NAMES).capitalize()} {r.choice(synth.NAMES).capitalize()}"
            text = (f"my name is {name}. ".encode() + base) if r.random() < 0.5 else base
            if long_every and k % long_every == long_every - 1:
                text = b" ".join(r.choice(bank.texts) for _ in range(r.randrange(30, 120)))
            rows.append((c, role, text, 1_760_000_000_000_000 + j * 5_000_000))
            k += 1
    return rows


@pytest.mark.gpu
def test_ext_candidates_vs_oracle(eng, oracle_cfg):
    """host API: random external candidates (names, other types, 1-byte, overlapping, below
    min_likelihood) over conversations with context and long rows -> bit-exact vs the oracle"""
    from oracle import pii_oracle as O
    P = oracle_cfg.type_id["PERSON_NAME"]
    r = random.Random(5)
    rows = _rows(11, 60, 12, long_every=37)
    others = [oracle_cfg.type_id[x] for x in ("EMAIL_ADDRESS", "PHONE_NUMBER", "SOCIAL_HANDLE", "US_PASSPORT")]
    ext = [_random_ext(r, t, P, others) for _, _, t, _ in rows]
    eng.histogram_reset()
    res = eng.scan_redact([t for _, _, t, _ in rows], [c + 1 for c, _, _, _ in rows], [x for _, x, _, _ in rows],
                          [s for _, _, _, s in rows], ext=ext)
    exp = O.process_rows(rows, oracle_cfg, extra=ext)
    n_person = 0
    for i, (red, fs, _, _) in enumerate(exp):
        assert res.text(i) == red, (i, rows[i][2][:80], ext[i])
        assert _spans_of(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
        n_person += sum(f.type_id == P for f in fs)
    assert n_person > 100
    assert int(eng.histogram()[P]) == n_person
    assert max(len(t) for _, _, t, _ in rows) > 4096                 # long rows were cut over lanes


@pytest.mark.gpu
def test_ext_long_row_candidates_across_lane_cuts(eng, oracle_cfg):
    """one 200 KB row with candidates every few bytes, many crossing the 1 KiB lane cuts, mixed
    with rule findings"""
    from oracle import pii_oracle as O
    P = oracle_cfg.type_id["PERSON_NAME"]
    r = random.Random(9)
    text = b" ".join(t for _, _, t, _ in _rows(3, 40, 10))[:200_000]
    cands, s = [], 0
    while True:
        s += r.randrange(1, 60)
        if s >= len(text):
            break
        cands.append((s, min(len(text), s + r.randrange(1, 40)), P, r.choice([3, 4, 5])))
    res = eng.scan_redact([text], [2], [O.ROLE_CUSTOMER], [0], ext=[cands])
    (red, fs, _, _), = O.process_rows([(0, O.ROLE_CUSTOMER, text, 0)], oracle_cfg, extra=[cands])
    assert res.text(0) == red
    assert _spans_of(res, 0) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs]


@pytest.mark.gpu
def test_malformed_ext_is_an_argument_error_and_commits_nothing(eng, oracle_cfg):
    from oracle import pii_oracle as O
    E = pkg("engine")
    P = oracle_cfg.type_id["PERSON_NAME"]
    eng.context_set(9, -1, 0)
    texts = [b"What is your email address?", b"jane@example.com"]
    for bad in ([(5, 3, P, 4)], [(0, 99, P, 4)], [(4, 6, P, 4), (1, 2, P, 4)], [(0, 2, 999, 4)], [(0, 2, P, 0)]):
        with pytest.raises(E.PiiError) as ei:
            eng.scan_redact(texts, [9, 9], [O.ROLE_AGENT, O.ROLE_CUSTOMER], [1, 2], ext=[[], bad])
        assert ei.value.code == E.PII_E_ARG
        assert eng.context_get(9)[0] == -1                            # the agent row's context: not stored
    res = eng.scan_redact(texts, [9, 9], [O.ROLE_AGENT, O.ROLE_CUSTOMER], [1, 2], ext=[[], [(0, 4, P, 4)]])
    assert res.text(1) == b"[EMAIL_ADDRESS]"                         # the longer email wins at start 0
    assert eng.group_types[eng.context_get(9)[0]] == "EMAIL_ADDRESS"


# ------------------------------------------------------------------------------ the device detector
@pytest.fixture(scope="module")
def ner_model():
    N = pkg("ner")
    ref = N.reference_model(seed=3)
    return ref, N.BertNer(ref, device=0)


def _device_rows(texts):
    import torch
    E = pkg("engine")
    data, offs = E.pack(texts)
    dev = torch.device("cuda:0")
    d_text = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    return data, offs, d_text, d_offs


@pytest.mark.gpu
def test_device_tokenizer_matches_hash_tokenizer(ner_model):
    import torch
    N = pkg("ner")
    _, m = ner_model
    r = random.Random(1)
    alphabet = b"abcXYZ019_ \t\n.,!?'@-" + bytes([0xc3, 0xa9, 0xff])
    texts = [b"", b"My name is John Smith, ok?", b"x" * 3 + b" y" * 70]
    texts += [bytes(r.choice(alphabet) for _ in range(r.randrange(0, 300))) for _ in range(300)]
    S = 64
    _, offs, d_text, d_offs = _device_rows(texts)
    n = len(texts)
    dev = m.dev
    ids = torch.empty(n * S, dtype=torch.int32, device=dev)
    mask, lo, hi = (torch.empty(n * S, dtype=torch.int32, device=dev) for _ in range(3))
    nt = torch.empty(n, dtype=torch.int32, device=dev)
    assert m.lib.ner_tokenize(d_text.data_ptr(), d_offs.data_ptr(), n, S, m.vocab, ids.data_ptr(), mask.data_ptr(),
                              lo.data_ptr(), hi.data_ptr(), nt.data_ptr(), m._st()) == 0
    want_ids, want_mask, want_spans = N.HashTokenizer(m.vocab, S).batch(texts)
    assert (ids.view(n, S).cpu().numpy() == want_ids).all()
    assert (mask.view(n, S).cpu().numpy() == want_mask).all()
    lo, hi, nt = lo.view(n, S).cpu().numpy(), hi.view(n, S).cpu().numpy(), nt.cpu().numpy()
    for i in range(n):
        assert nt[i] == len(want_spans[i])
        assert [(int(a), int(b)) for a, b in zip(lo[i, :nt[i]], hi[i, :nt[i]])] == want_spans[i], i


@pytest.mark.gpu
def test_span_decoder_matches_decode_spans(ner_model):
    import torch
    N = pkg("ner")
    _, m = ner_model
    g = torch.Generator().manual_seed(4)
    texts = [b"alpha beta gamma, delta epsilon zeta eta theta iota kappa lambda mu" * (1 + i % 3) for i in range(200)]
    S = 32
    tok = N.HashTokenizer(m.vocab, S)
    _, _, spans = tok.batch(texts)
    n = len(texts)
    logits = torch.randn(n * S, 3, generator=g)
    logits[::7] = 0.0                                                  # ties: the first maximum wins
    lo = np.zeros((n, S), np.int32)
    hi = np.zeros((n, S), np.int32)
    nt = np.array([len(s) for s in spans], np.int32)
    for i, sp in enumerate(spans):
        for j, (a, b) in enumerate(sp):
            lo[i, j], hi[i, j] = a, b
    dev = m.dev
    ext = torch.empty((n * S, 4), dtype=torch.int32, device=dev)
    ext_n = torch.empty(n, dtype=torch.int32, device=dev)
    T = lambda a: torch.from_numpy(a.reshape(-1)).to(dev)              # noqa: E731
    d_lo, d_hi, d_nt, d_lg = T(lo), T(hi), T(nt), logits.to(dev)
    assert m.lib.ner_spans(d_lg.data_ptr(), 3, d_lo.data_ptr(), d_hi.data_ptr(), d_nt.data_ptr(), n, S, 22, 4,
                           ext.data_ptr(), ext_n.data_ptr(), m._st()) == 0
    E = pkg("engine")
    got = ext.cpu().numpy().view(E.SPAN_DTYPE).reshape(n, S)
    cnt = ext_n.cpu().numpy()
    lab = logits.argmax(-1).view(n, S).numpy()
    for i in range(n):
        want = N.decode_spans(lab[i][:nt[i]], spans[i])
        assert [(int(x["start"]), int(x["end"])) for x in got[i][:cnt[i]]] == want, i
        assert all(int(x["info_type"]) == 22 and int(x["likelihood"]) == 4 for x in got[i][:cnt[i]])


@pytest.mark.gpu
def test_device_ner_on_the_redaction_path(eng, oracle_cfg, ner_model):
    """rows in HBM -> k_tokenize -> BERT -> k_ner_spans -> pii_scan_redact_device_ext, no host round
    trip; vs oracle + the GPU's spans (exact) and vs oracle + HF fp32 (exact on rows that clear the
    bf16 margin, token labels agreeing wherever fp32 is decisive)"""
    import torch
    from oracle import pii_oracle as O
    N = pkg("ner")
    ref, m = ner_model
    P = oracle_cfg.type_id["PERSON_NAME"]
    rows = _rows(21, 40, 8)
    texts = [t for _, _, t, _ in rows]
    n = len(texts)
    S = 64
    data, offs, d_text, d_offs = _device_rows(texts)
    dev = m.dev
    # one explicit stream for the detector and the engine (a NULL stream handle would select the
    # engine's own stream, which is not ordered after the detector's kernels)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        ext, ext_n, stride = m.detect_device(d_text.data_ptr(), d_offs.data_ptr(), n, S=S, info_type=P)
    d_slot = torch.tensor([c + 100 for c, _, _, _ in rows], dtype=torch.int32, device=dev)
    d_role = torch.tensor([x for _, x, _, _ in rows], dtype=torch.uint8, device=dev)
    d_ts = torch.tensor([s for _, _, _, s in rows], dtype=torch.int64, device=dev)
    out_cap = int(offs[-1]) * 4 + 64 * n
    span_cap = int(offs[-1]) + n
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, device=dev)
    d_ctx = torch.empty(n, dtype=torch.int16, device=dev)
    eng.scan_redact_device_ext(d_text.data_ptr(), d_offs.data_ptr(), n, 0, int(offs[-1]), d_slot.data_ptr(),
                               d_role.data_ptr(), d_ts.data_ptr(), d_out.data_ptr(), out_cap, d_oo.data_ptr(),
                               d_sp.data_ptr(), span_cap, d_ctx.data_ptr(), ext.data_ptr(), ext_n.data_ptr(), stride,
                               st.cuda_stream)
    assert st.cuda_stream != 0
    ob, ns, fl = eng.sync()
    st.synchronize()
    assert fl == 0
    out = d_out[:ob].cpu().numpy().tobytes()
    oo = d_oo.cpu().numpy()
    E = pkg("engine")
    spans = d_sp[:ns * 16].cpu().numpy().view(E.SPAN_DTYPE)
    gx = ext.cpu().numpy().view(E.SPAN_DTYPE).reshape(n, stride)
    gn = ext_n.cpu().numpy()
    gpu_ext = [[(int(x["start"]), int(x["end"]), P, int(x["likelihood"])) for x in gx[i][:gn[i]]] for i in range(n)]
    # (1) the merge: bit-exact vs the oracle fed the GPU's spans
    exp = O.process_rows(rows, oracle_cfg, extra=gpu_ext)
    for i, (red, fs, _, _) in enumerate(exp):
        assert out[int(oo[i]):int(oo[i + 1])] == red, i
        sel = spans[spans["utt"] == i]
        assert [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in sel] == \
            [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
    assert sum(len(x) for x in gpu_ext) > n                            # names did reach the engine
    # (2) the detector vs HF fp32 (same ids)
    tok = N.HashTokenizer(m.vocab, S)
    ids, mask, tspans = tok.batch(texts)
    with torch.no_grad():
        lg = ref(input_ids=torch.as_tensor(ids, dtype=torch.long),
                 attention_mask=torch.as_tensor(mask, dtype=torch.long)).logits.numpy()
    top2 = np.sort(lg, -1)
    margin = top2[..., -1] - top2[..., -2]
    hf_lab = lg.argmax(-1)
    gpu_lab = m.forward(ids, mask).argmax(-1).cpu().numpy()
    real = mask.astype(bool)
    decisive = real & (margin >= NER_MARGIN)
    assert (gpu_lab[decisive] == hf_lab[decisive]).all()
    assert decisive.sum() > 0.5 * real.sum()
    hf_ext = [[(s, e, P, N.LIKELY) for s, e in N.decode_spans(hf_lab[i], tspans[i])] for i in range(n)]
    exp_hf = O.process_rows(rows, oracle_cfg, extra=hf_ext)
    clean = [i for i in range(n) if decisive[i][1:len(tspans[i]) - 1].all()]
    for i in clean:
        assert out[int(oo[i]):int(oo[i + 1])] == exp_hf[i][0], i
    assert len(clean) > 0
    # rows on which the bf16 detector labels every token as the fp32 model does redact exactly as
    # oracle + HF; with seeded random weights many tokens sit near a tie (only 10 of 320 rows clear the
    # 0.1 margin on every token), so the bar is that most rows agree token for token (not
    # just "> 0 rows")
    agree = [i for i in range(n) if (gpu_lab[i][real[i]] == hf_lab[i][real[i]]).all()]
    for i in agree:
        assert out[int(oo[i]):int(oo[i + 1])] == exp_hf[i][0], i
    assert len(agree) >= 0.75 * n, (len(agree), n)
