"""HIP engine vs the CPU oracle, through the C ABI (libpii.so).  Needs an MI355X: pytest -m gpu.

Bar: bit-exact redacted bytes, spans (start, end, infoType, likelihood) and context decisions.
"""
import json
import os
import random

import numpy as np
import pytest

from conftest import ROOT, pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(compiled):
    E = pkg("engine")
    e = E.Engine(compiled.blob, device=0, n_conv_slots=1 << 18)
    yield e
    e.close()


def _spans_of(res, i):
    m = res.spans["utt"] == i
    return [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]


def _check_rows(eng, oracle_cfg, rows, slot_base=0):
    """rows: list of (conv, role, text, ts); every conversation must be contiguous."""
    from oracle import pii_oracle as O
    convs = {}
    slots = [slot_base + convs.setdefault(c, len(convs)) for c, _, _, _ in rows]
    res = eng.scan_redact([t for _, _, t, _ in rows], slots, [r for _, r, _, _ in rows], [s for _, _, _, s in rows])
    exp = O.process_rows(rows, oracle_cfg)
    groups = list(oracle_cfg.context_keywords.keys())
    for i, ((red, fs, used, stored), row) in enumerate(zip(exp, rows)):
        assert res.text(i) == red, (i, row[2], res.text(i), red)
        assert _spans_of(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], (i, row[2])
        info = int(res.ctx_info[i])
        if row[1] == O.ROLE_AGENT:
            assert (groups[info] if info >= 0 else None) == stored, (i, row[2])
        elif row[1] == O.ROLE_CUSTOMER:
            assert (groups[info] if info >= 0 else None) == used, (i, row[2])
    return res


def test_transcripts_replay(eng, oracle_cfg):
    """BASELINE config 1: final_transcript/*.json replayed through context + redaction."""
    from oracle import pii_oracle as O
    with open(os.path.join(ROOT, "tests", "golden", "transcripts.json")) as f:
        ts = json.load(f)
    rows = []
    for name, t in ts.items():
        for e in t["entries"]:
            rows.append((name, O.ROLE_AGENT if e["role"] == "AGENT" else O.ROLE_CUSTOMER, e["text"].encode(), e["ts"]))
    _check_rows(eng, oracle_cfg, rows, slot_base=100)
    with open(os.path.join(ROOT, "tests", "golden", "oracle_transcripts.json")) as f:
        gold = json.load(f)
    # the committed golden redactions (oracle regression pin) agree with the engine too
    res = _check_rows(eng, oracle_cfg, rows, slot_base=200)
    flat = [r for name in ts for r in gold[name]]
    for i, g in enumerate(flat):
        assert res.text(i).decode() == g["redacted"]


def test_synthetic_conversations(eng, oracle_cfg):
    synth = pkg("synth")
    bank = synth.build_bank(600, 1400, seed=11)
    corp = synth.make_corpus(120, 24, bank, seed=5)
    rows = []
    for i in range(corp.n):
        a, b = int(corp.offsets[i]), int(corp.offsets[i + 1])
        rows.append((int(corp.conv_slot[i]), int(corp.role[i]), corp.data[a:b].tobytes(), int(corp.ts_us[i])))
    _check_rows(eng, oracle_cfg, rows, slot_base=2000)


def _mutated(r, synth):
    mut = b"0123456789-. @:/AZaz\n"
    ty = r.choice(synth.PII_TYPES)
    v = bytearray(synth.pii_value(r, ty, r.random() < 0.5).encode())
    for _ in range(r.randrange(0, 3)):
        k = r.randrange(len(v))
        op = r.randrange(3)
        if op == 0:
            v[k] = r.choice(mut)
        elif op == 1:
            del v[k]
        else:
            v.insert(k, r.choice(mut))
    hw = r.choice(synth.HOTWORDS[ty]).encode()
    pre = r.choice([b"", hw + b" is ", b"my " + hw + b" " + b"x" * r.randrange(0, 70) + b" ", b"(", b"a"])
    return pre + bytes(v) + r.choice([b"", b".", b" ok", b"1", b"-2", b"@x.io"])


def test_random_and_mutated_with_context(eng, oracle_cfg):
    """Single-row conversations whose context is preset with pii_context_set (every group)."""
    from oracle import pii_oracle as O
    synth = pkg("synth")
    r = random.Random(7)
    alpha = b"0123456789 -./@:()abcXYZAEI_%+,\n'\xc3\xa9\x80\xff"
    texts = []
    for i in range(4000):
        if i % 2:
            texts.append(bytes(r.choice(alpha) for _ in range(r.randrange(0, 80))))
        else:
            texts.append(_mutated(r, synth))
    groups = list(oracle_cfg.context_keywords.keys())
    slot0 = 10000
    ctxs = [r.randrange(-1, len(groups)) for _ in texts]
    for i, g in enumerate(ctxs):
        eng.context_set(slot0 + i, g, 1_000_000)
    res = eng.scan_redact(texts, [slot0 + i for i in range(len(texts))], [O.ROLE_CUSTOMER] * len(texts),
                          [1_000_000 + 1000] * len(texts))
    for i, (t, g) in enumerate(zip(texts, ctxs)):
        red, fs = O.redact(t, oracle_cfg, groups[g] if g >= 0 else None)
        assert res.text(i) == red, (t, g, res.text(i), red)
        assert _spans_of(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], (t, g)


def test_edge_cases(eng, oracle_cfg):
    from oracle import pii_oracle as O
    long_row = b" ".join([b"card number 4141-1212-2323-5009 and jane.doe@example.com, ip address 10.0.0.1;"] * 700)
    texts = [b"", b"x", b"\n", b"1", "café ü 4141-1212-2323-5009 中".encode(), b"@", b"@a",
             b"a" * 5000, b"9" * 4000, long_row, b"", b"SSN 123-45-6789\nCVV 123"]
    res = eng.scan_redact(texts, list(range(20000, 20000 + len(texts))), [O.ROLE_CUSTOMER] * len(texts))
    for i, t in enumerate(texts):
        red, fs = O.redact(t, oracle_cfg, None)
        assert res.text(i) == red, (i, t[:60])
        assert _spans_of(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs]
    empty = eng.scan_redact([], [], [])
    assert len(empty.out) == 0 and len(empty.spans) == 0
    allempty = eng.scan_redact([b""] * 5, [1, 1, 2, 3, 3], [1, 0, 1, 0, 2])
    assert list(allempty.out_offsets) == [0] * 6


def test_dense_findings_per_lane(eng, oracle_cfg):
    """more than 64 findings in one scan lane and in one utterance (k_spans / k_select carry their
    running state across 64-finding chunks), beside rows with none"""
    from oracle import pii_oracle as O
    r = random.Random(41)
    texts = []
    for k in range(60):
        n = r.randrange(40, 400)
        items = [f"u{r.randrange(10 ** 6)}@x{r.randrange(9)}.io" if r.random() < 0.7 else
                 f"10.{r.randrange(256)}.{r.randrange(256)}.{r.randrange(256)}" for _ in range(n)]
        texts.append(" ".join(items).encode())
        texts.append(b"ok thanks" if k % 3 else b"")
    res = eng.scan_redact(texts, list(range(30000, 30000 + len(texts))), [O.ROLE_CUSTOMER] * len(texts))
    assert max(len(_spans_of(res, i)) for i in range(len(texts))) > 128
    for i, t in enumerate(texts):
        red, fs = O.redact(t, oracle_cfg, None)
        assert res.text(i) == red, (i, t[:60])
        assert _spans_of(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i


def test_context_ttl_and_persistence(eng, oracle_cfg):
    from oracle import pii_oracle as O
    E = pkg("engine")
    slot = 30000
    ask = b"Can you confirm the CVV on the card?"
    ans = b"Sure, it is 123."
    t0 = 1_760_000_000_000_000
    r1 = eng.scan_redact([ask], [slot], [O.ROLE_AGENT], [t0])
    g = int(r1.ctx_info[0])
    assert oracle_cfg.context_keywords and list(oracle_cfg.context_keywords)[g] == O.extract_expected_pii(ask, oracle_cfg)
    assert eng.context_get(slot) == (g, t0)
    r2 = eng.scan_redact([ans], [slot], [O.ROLE_CUSTOMER], [t0 + 89_000_000])
    assert int(r2.ctx_info[0]) == g
    r3 = eng.scan_redact([ans], [slot], [O.ROLE_CUSTOMER], [t0 + 90_000_000])
    assert int(r3.ctx_info[0]) == -1                     # SETEX 90 s expired
    # a miss does not clear the context (main.py:381-382)
    eng.scan_redact([b"Thanks!"], [slot], [O.ROLE_AGENT], [t0 + 1])
    assert eng.context_get(slot)[0] == g
    # ORDER: one slot in two runs of one batch is rejected and leaves state untouched
    with pytest.raises(E.PiiError) as ei:
        eng.scan_redact([ask, ans, ask], [slot, slot + 1, slot], [1, 0, 1], [t0] * 3)
    assert ei.value.code == E.PII_E_ORDER


def test_histogram_matches_spans(eng, oracle_cfg):
    """counts accumulate over calls until pii_histogram_reset; the reset is deferred to the next call's
    first kernel, and the counts read as zero until then"""
    synth = pkg("synth")
    bank = synth.build_bank(100, 400, seed=3)
    eng.histogram_reset()
    assert not eng.histogram().any()
    res = eng.scan_redact(bank.texts, list(range(40000, 40000 + len(bank.texts))), list(bank.roles))
    h = eng.histogram()
    want = np.bincount(res.spans["info_type"].astype(np.int64), minlength=len(h))
    assert want.any() and (h == want).all()
    res2 = eng.scan_redact(bank.texts[:50], list(range(41000, 41050)), list(bank.roles[:50]))
    want2 = np.bincount(res2.spans["info_type"].astype(np.int64), minlength=len(h))
    assert (eng.histogram() == want + want2).all()
    eng.histogram_reset()
    assert not eng.histogram().any()
    res3 = eng.scan_redact(bank.texts[:50], list(range(42000, 42050)), list(bank.roles[:50]))
    assert (eng.histogram() == np.bincount(res3.spans["info_type"].astype(np.int64), minlength=len(h))).all()


def test_device_api_large_batch_properties(eng, oracle_cfg):
    """Config-2-shaped batch through the device API: invariants at full size + sampled oracle rows."""
    import torch
    from oracle import pii_oracle as O
    synth = pkg("synth")
    bank = synth.build_bank(2000, 2000, seed=99)
    corp = synth.make_corpus(20000, 50, bank, seed=1, conv_base=100000)   # 1M utterances
    dev = torch.device("cuda:0")
    d_text = torch.from_numpy(corp.data).to(dev)
    d_offs = torch.from_numpy(corp.offsets.view(np.int64)).to(dev)
    d_slot = torch.from_numpy(corp.conv_slot.view(np.int32)).to(dev)
    d_role = torch.from_numpy(corp.role).to(dev)
    d_ts = torch.from_numpy(corp.ts_us).to(dev)
    n = corp.n
    out_cap = int(corp.offsets[-1]) * 2 + 64 * n
    span_cap = n * 4
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, device=dev)
    d_ctx = torch.empty(n, dtype=torch.int16, device=dev)
    eng.scan_redact_device(d_text.data_ptr(), d_offs.data_ptr(), n, d_slot.data_ptr(), d_role.data_ptr(),
                           d_ts.data_ptr(), d_out.data_ptr(), out_cap, d_oo.data_ptr(), d_sp.data_ptr(), span_cap,
                           d_ctx.data_ptr())
    ob, ns, flags = eng.sync()
    assert flags == 0
    oo = d_oo.cpu().numpy().astype(np.uint64)
    assert oo[-1] == ob and (np.diff(oo.astype(np.int64)) >= 0).all()
    out = d_out[:ob].cpu().numpy()
    ctx = d_ctx.cpu().numpy()
    spans = np.frombuffer(d_sp[:ns * 16].cpu().numpy().tobytes(), dtype=pkg("engine").SPAN_DTYPE)
    assert (np.diff(spans["utt"].astype(np.int64)) >= 0).all()
    groups = list(oracle_cfg.context_keywords.keys())
    kw_cache = {}

    def kw(bid):
        if bid not in kw_cache:
            kw_cache[bid] = O.extract_expected_pii(bank.texts[bid], oracle_cfg)
        return kw_cache[bid]
    r = random.Random(0)
    per_conv = 50
    starts = np.searchsorted(spans["utt"], np.arange(n + 1))
    for i in r.sample(range(n), 3000):
        t = corp.data[int(corp.offsets[i]):int(corp.offsets[i + 1])].tobytes()
        if corp.role[i] == O.ROLE_AGENT:
            et = None
            assert (groups[ctx[i]] if ctx[i] >= 0 else None) == kw(int(corp.bank_id[i]))
        else:
            et = None
            c0 = i - i % per_conv
            for j in range(i - 1, c0 - 1, -1):
                if corp.role[j] == O.ROLE_AGENT and kw(int(corp.bank_id[j])):
                    if corp.ts_us[i] - corp.ts_us[j] < 90_000_000:
                        et = kw(int(corp.bank_id[j]))
                    break
            assert (groups[ctx[i]] if ctx[i] >= 0 else None) == et
        red, fs = O.redact(t, oracle_cfg, et)
        assert out[int(oo[i]):int(oo[i + 1])].tobytes() == red
        got = [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"]))
               for s in spans[starts[i]:starts[i + 1]]]
        assert got == [(f.start, f.end, f.type_id, f.likelihood) for f in fs]


def test_context_update_alone_matches_the_oracle(compiled, oracle_cfg):
    """pii_context_update (the context half alone, run after a failed redaction) commits exactly the
    context records and reports exactly the ctx_info of a full call, vs the oracle replay, on synthetic
    conversations and the golden transcripts; a following full call sees those records."""
    from oracle import pii_oracle as O
    E, synth = pkg("engine"), pkg("synth")
    eng = E.Engine(compiled.blob, device=0, n_conv_slots=4096)
    try:
        bank = synth.build_bank(400, 900, seed=41)
        corp = synth.make_corpus(300, 12, bank, seed=42)
        rows = []
        for i in range(corp.n):
            a, b = int(corp.offsets[i]), int(corp.offsets[i + 1])
            rows.append((int(corp.conv_slot[i]), int(corp.role[i]), corp.data[a:b].tobytes(), int(corp.ts_us[i])))
        ctx = eng.context_update([r[2] for r in rows], [1 + r[0] for r in rows], [r[1] for r in rows],
                                 [r[3] for r in rows])
        store = O.ContextStore()
        exp = O.process_rows(rows, oracle_cfg, store=store)
        groups = list(oracle_cfg.context_keywords.keys())
        for i, ((_, _, used, stored), row) in enumerate(zip(exp, rows)):
            want = stored if row[1] == O.ROLE_AGENT else used if row[1] == O.ROLE_CUSTOMER else None
            assert (groups[ctx[i]] if ctx[i] >= 0 else None) == want, (i, row)
        for c in {r[0] for r in rows}:
            g, ts = eng.context_get(1 + c)
            rec = store.d.get(c)
            if rec is not None:
                assert groups[g] == rec[0] and ts == rec[2]
        # later rows read the records the context-only call stored
        later = [(r[0], O.ROLE_CUSTOMER, b"4141-1212-2323-5009 and 123", r[3] + 1) for r in rows[-30:]]
        res = eng.scan_redact([t for _, _, t, _ in later], [1 + c for c, _, _, _ in later],
                              [O.ROLE_CUSTOMER] * len(later), [s for _, _, _, s in later])
        exp2 = O.process_rows(later, oracle_cfg, store=store)
        assert [res.text(i) for i in range(len(later))] == [x[0] for x in exp2]
    finally:
        eng.close()
