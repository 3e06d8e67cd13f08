"""Long rows (whole transcripts, realtime joins, joined windows: /root/reference/ccai_insights_function/
main.py:47-50, main_service/main.py:457) are cut into 1 KiB lanes, scanned with a halo and stitched by
verification (k_scan_fix), selected per lane with the carried state re-run where a match reaches over
a cut (k_sel_dirty / k_sel_fix / k_rowlen), and redacted by output tiles (k_redact).

* parity vs the oracle on rows of 20-300 KB built to stress the stitching: long unbroken runs (email
  local parts, digits, capitals, one long word) across many cuts, PII straddling cuts, hotwords just
  before a cut, dense PII;
* at full size (64 MB row, 1000 x 1 MB rows), the size-independent split property: utterances joined
  by 128 spaces (no detector consumes two spaces, no hotword window is 128 bytes wide, a space gives
  the same word boundary as a text edge) redact to the join of their own redactions, which the engine
  computes as ordinary short rows (themselves pinned to the oracle by test_gpu_parity.py).
"""
import random

import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu

SEP = b" " * 128


@pytest.fixture(scope="module")
def eng(compiled):
    E = pkg("engine")
    e = E.Engine(compiled.blob, device=0, n_conv_slots=1 << 12)
    yield e
    e.close()


def _spans(res, i):
    m = res.spans["utt"] == i
    return [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]


def _adversarial_row(r, synth, bank, target):
    """~target bytes: synthetic utterances joined by ' ' / '\\n', with long unbroken runs mixed in."""
    parts = []
    n = 0
    while n < target:
        k = r.random()
        if k < 0.55:
            p = r.choice(bank.texts)
        elif k < 0.62:          # an email whose local part spans several lanes
            p = ("".join(r.choice("abcxyz0123._") for _ in range(r.randrange(900, 3500))) + "@example.com").encode()
        elif k < 0.68:          # long digit run (no detector matches it whole)
            p = ("".join(r.choice("0123456789") for _ in range(r.randrange(500, 3000)))).encode()
        elif k < 0.73:          # long capitals (SWIFT / passport / MBI / IBAN shapes inside)
            p = ("".join(r.choice("ABCDEFGHJKLMNPQRTUVWXY0123456789") for _ in range(r.randrange(500, 2500)))).encode()
        elif k < 0.78:          # one long word
            p = ("x" * r.randrange(1000, 4000)).encode()
        elif k < 0.9:           # PII right after a hotword, placed anywhere (also across cuts)
            ty = r.choice(synth.PII_TYPES)
            p = f"my {r.choice(synth.HOTWORDS[ty])} is {synth.pii_value(r, ty, r.random() < 0.6)}".encode()
        else:                   # dense PII
            p = b" ".join(synth.pii_value(r, r.choice(synth.PII_TYPES), True).encode() for _ in range(r.randrange(5, 40)))
        parts.append(p)
        parts.append(r.choice([b" ", b"\n", b", ", b"  "]))
        n += len(p) + 1
    return b"".join(parts)


def test_long_rows_vs_oracle(eng, oracle_cfg):
    from oracle import pii_oracle as O
    synth = pkg("synth")
    bank = synth.build_bank(300, 600, seed=17)
    r = random.Random(23)
    texts, ctx = [], []
    groups = list(oracle_cfg.context_keywords.keys())
    for k in range(14):
        texts.append(_adversarial_row(r, synth, bank, r.choice([20_000, 60_000, 150_000, 300_000])))
        texts.append(r.choice(bank.texts))                      # short rows between the long ones
    slot0 = 300
    for i in range(len(texts)):
        g = r.randrange(-1, len(groups))
        ctx.append(g)
        eng.context_set(slot0 + i, g, 1_000_000)
    res = eng.scan_redact(texts, [slot0 + i for i in range(len(texts))], [O.ROLE_CUSTOMER] * len(texts),
                          [1_000_001] * len(texts))
    for i, (t, g) in enumerate(zip(texts, ctx)):
        red, fs = O.redact(t, oracle_cfg, groups[g] if g >= 0 else None)
        got = res.text(i)
        if got != red:
            k = next(j for j in range(min(len(got), len(red))) if got[j] != red[j])
            raise AssertionError((i, len(t), k, got[max(0, k - 80):k + 80], red[max(0, k - 80):k + 80]))
        assert _spans(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i


def test_long_agent_row_context(eng, oracle_cfg):
    """A long AGENT row (keyword hits in several lanes: the atomic-min keyword group) sets the
    context that the next customer row uses."""
    from oracle import pii_oracle as O
    synth = pkg("synth")
    bank = synth.build_bank(300, 600, seed=19)
    r = random.Random(5)
    agent = _adversarial_row(r, synth, bank, 80_000) + b" what's your date of birth? and the cvv please"
    rows = [(7, O.ROLE_AGENT, agent, 1_000_000), (7, O.ROLE_CUSTOMER, b"sure 01/22/1985 and 123", 2_000_000)]
    res = eng.scan_redact([x[2] for x in rows], [900, 900], [x[1] for x in rows], [x[3] for x in rows])
    exp = O.process_rows([(900, a, b, c) for _, a, b, c in rows], oracle_cfg)
    for i, (red, fs, used, stored) in enumerate(exp):
        assert res.text(i) == red
        assert _spans(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs]
    groups = list(oracle_cfg.context_keywords.keys())
    assert groups[int(res.ctx_info[0])] == exp[0][3]


def _split_property(eng, utts, rows_per):
    """rows = SEP.join(utts[k*rows_per:(k+1)*rows_per]); engine(rows) == SEP.join(engine(utts))."""
    E = pkg("engine")
    n_rows = len(utts) // rows_per
    utts = utts[:n_rows * rows_per]
    short = eng.scan_redact(utts, [1] * len(utts), [E.ROLE_OTHER] * len(utts))
    longs = [SEP.join(utts[k * rows_per:(k + 1) * rows_per]) for k in range(n_rows)]
    res = eng.scan_redact(longs, [2] * n_rows, [E.ROLE_OTHER] * n_rows)
    so = short.out_offsets.astype(np.int64)
    sp_u = short.spans["utt"].astype(np.int64)
    lens = np.array([len(u) for u in utts], dtype=np.int64)
    for k in range(n_rows):
        lo, hi = k * rows_per, (k + 1) * rows_per
        want = SEP.join(short.out[so[i]:so[i + 1]].tobytes() for i in range(lo, hi))
        got = res.text(k)
        assert got == want, (k, len(got), len(want))
        # spans: each utterance's spans shifted by its start inside the long row
        base = np.concatenate([[0], np.cumsum(lens[lo:hi] + len(SEP))[:-1]])
        m = (sp_u >= lo) & (sp_u < hi)
        sub = short.spans[m]
        exp = np.stack([sub["start"].astype(np.int64) + base[sub["utt"].astype(np.int64) - lo],
                        sub["end"].astype(np.int64) + base[sub["utt"].astype(np.int64) - lo],
                        sub["info_type"].astype(np.int64), sub["likelihood"].astype(np.int64)], axis=1)
        g = res.spans[res.spans["utt"] == k]
        gotv = np.stack([g["start"].astype(np.int64), g["end"].astype(np.int64), g["info_type"].astype(np.int64),
                         g["likelihood"].astype(np.int64)], axis=1)
        assert gotv.shape == exp.shape and (gotv == exp).all(), k
    return res


def test_one_64mb_row_split_property(eng):
    synth = pkg("synth")
    bank = synth.build_bank(4096, 4096, seed=29)
    meta = synth.corpus_meta(2600, 100, bank, seed=31)       # 260k utterances: ~31 MB + 33 MB of separators
    data = synth.gather_bytes(meta, bank)
    o = meta.offsets
    utts = [data[int(o[i]):int(o[i + 1])].tobytes() for i in range(meta.n)]
    res = _split_property(eng, utts, len(utts))
    assert len(res.text(0)) > 60_000_000


def test_thousand_1mb_rows_split_property(eng):
    synth = pkg("synth")
    bank = synth.build_bank(4096, 4096, seed=37)
    meta = synth.corpus_meta(40000, 100, bank, seed=41)
    data = synth.gather_bytes(meta, bank)
    o = meta.offsets
    utts = [data[int(o[i]):int(o[i + 1])].tobytes() for i in range(meta.n)]
    # ~1 MB rows: 4000 utterances each (~0.48 MB of text + 0.51 MB of separators); 1000 rows
    rows_per = 4000
    assert len(utts) // rows_per == 1000
    _split_property(eng, utts, rows_per)


def test_whole_rows_before_and_after_a_long_row(eng, oracle_cfg):
    """k_sel_fix re-runs the clean lane that holds a cut row's start (and the dirty lanes after it)
    when a match of the cut row reaches over a cut: the whole rows sharing those lanes must keep
    their output lengths (counted once).  Short rows with findings packed around long rows whose
    matches straddle the first cut, at 128-byte lanes (a small batch) and at 1 KiB lanes."""
    from oracle import pii_oracle as O
    synth = pkg("synth")
    r = random.Random(17)
    bank = synth.build_bank(300, 300, seed=17)
    for n_pad in (0, 700_000):
        rows = []
        for k in range(120):
            rows.append((k, O.ROLE_CUSTOMER, b"mail me at jo@ex.com ok", 0))
            email = ("".join(r.choice("abcxyz0123._") for _ in range(r.randrange(20, 300))) + "@example.com").encode()
            lead = b"y" * r.randrange(0, 200)
            rows.append((k, O.ROLE_CUSTOMER, lead + b" " + email + b" " + r.choice(bank.texts) * r.randrange(3, 30), 0))
            rows.append((k, O.ROLE_CUSTOMER, r.choice(bank.texts[300:]), 0))
        n_head = len(rows)
        if n_pad:                                  # a big batch (> 64 MB): 1 KiB lanes
            rows += [(121 + i % 3000, O.ROLE_CUSTOMER, bank.texts[i % len(bank.texts)], 0) for i in range(n_pad)]
            rows.sort(key=lambda x: x[0])
        res = eng.scan_redact([t for _, _, t, _ in rows], [c + 1 for c, _, _, _ in rows], [x for _, x, _, _ in rows],
                              [0] * len(rows))
        if n_pad:
            assert eng.stats()["lane_bytes"] == 1024
        exp = O.process_rows(rows[:n_head], oracle_cfg)          # the conversations with the long rows
        for i, (red, fs, _, _) in enumerate(exp):
            assert res.text(i) == red, (n_pad, i)
            assert _spans(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], (n_pad, i)


def test_2mb_row_of_joined_utterances_vs_oracle(eng, oracle_cfg):
    """A 2 MB row of synthetic utterances joined by '\\n' / ' ' (the aggregator's joins and the
    realtime join, README.md:131-134, main_service/main.py:457): hotwords of one utterance reach the
    PII of the next across the joins and across 2000 lane cuts; the row is redacted with a context
    (the agent row's SSN request) and without."""
    from oracle import pii_oracle as O
    synth = pkg("synth")
    r = random.Random(23)
    bank = synth.build_bank(2000, 2000, seed=23)
    parts, n = [], 0
    while n < 2_100_000:
        p = r.choice(bank.texts)
        parts += [p, r.choice([b"\n", b" "])]
        n += len(p) + 1
    text = b"".join(parts)
    rows = [(1, O.ROLE_AGENT, b"Could you confirm your social security number please?", 0),
            (1, O.ROLE_CUSTOMER, text, 1), (2, O.ROLE_OTHER, text, 2)]
    res = eng.scan_redact([t for _, _, t, _ in rows], [5, 5, 6], [x for _, x, _, _ in rows], [0, 1, 2])
    exp = O.process_rows(rows, oracle_cfg)
    for i, (red, fs, _, _) in enumerate(exp):
        assert res.text(i) == red, i
        assert _spans(res, i) == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
    assert len(exp[1][1]) > 1000 and exp[1][2] == "US_SOCIAL_SECURITY_NUMBER"     # the context was applied
