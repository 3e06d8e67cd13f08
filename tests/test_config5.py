"""Config 5 (BASELINE.json configs[4], SURVEY §8 ★X1): 500+ seeded custom regex and dictionary
infoTypes (rulegen.Config5) on top of the shipped dlp_config.

The reference runs such a rule set through the same DLP call (main_service/main.py:580) with the
custom types in inspect_config.custom_info_types and the context merge of main.py:614-686; the
oracle restates that (dictionaries as case-insensitive word-boundary alternations).  Parity is
"unpinned" in the SURVEY §8(c) sense (no reference output exists for synthetic types): the oracle is
the checker.

* CPU: the generated rule set, its split over SCAN groups, and the compiled tables (tests/tablesim.py
  executes them the way the kernels do) vs the oracle on generated text, with and without context;
* GPU: the engine (one k_scan pass per SCAN group, merged events, FIRST / rule tables read from
  global memory where they exceed LDS) vs the oracle on conversations whose agent rows set custom and
  built-in contexts."""
import os
import random

import numpy as np
import pytest

from conftest import pkg


@pytest.fixture(scope="module")
def c5(tmp_path_factory):
    G = pkg("rulegen")
    c = G.Config5()
    path = str(tmp_path_factory.mktemp("c5") / "config5.json")
    c.save(path)
    return c, path


@pytest.fixture(scope="module")
def c5_comp(c5):
    C = pkg("compiler")
    return C.compile_rules(C.Rules.load(c5[1]))


@pytest.fixture(scope="module")
def c5_oracle(c5):
    from oracle import pii_oracle as O
    return O.RuleConfig.load(c5[1])


def _builtin_value(r):
    synth = pkg("synth")
    return synth.pii_value(r, r.choice(synth.PII_TYPES), r.random() < 0.7)


def test_config5_rule_set(c5, c5_comp):
    c, _ = c5
    customs = c.cfg["inspect_config"]["custom_info_types"]
    assert len(customs) >= 500
    assert sum("dictionary" in x for x in customs) >= 150 and sum("regex" in x for x in customs) >= 300
    assert len(c5_comp.rules.type_names) >= 520
    groups = c5_comp.scan_groups
    assert len(groups) > 1                         # the rule set does not fit one LDS automaton
    assert sorted(p for g in groups for p in g) == list(range(len(c5_comp.rules.patterns)))
    assert len(c5_comp.sections["pool.trans"]) * 2 > 160 * 1024     # FIRST pool larger than LDS


def test_config5_tables_vs_oracle(c5, c5_comp, c5_oracle):
    from oracle import pii_oracle as O
    from tablesim import TableSim
    c, _ = c5
    sim = TableSim(c5_comp)
    r = random.Random(3)
    groups = list(c5_oracle.context_keywords.keys())
    for i in range(160):
        t = c.utterance(r, _builtin_value).encode()
        g = r.choice([None, None, r.choice(c.context_types), r.choice(groups)])
        ev = sim.scan(t, False)
        v = 0 if g is None else 1 + groups.index(g)
        got = sim.resolve(t, ev, v)
        exp = [(f.start, f.end, f.type_id, f.likelihood) for f in O.find_pii(t, c5_oracle, g)]
        assert got == exp, (t, g)


def _conversations(c, n_conv, per, seed):
    r = random.Random(seed)
    rows = []
    for conv in range(n_conv):
        ts = 1_700_000_000_000_000 + conv * 10**9
        for k in range(per):
            ts += r.randrange(3, 30) * 1_000_000
            if k % 2 == 0:
                rows.append((conv, 1, c.agent_utterance(r).encode(), ts))
            else:
                rows.append((conv, 0, c.utterance(r, _builtin_value).encode(), ts))
    return rows


@pytest.mark.gpu
def test_config5_engine_vs_oracle(c5, c5_comp, c5_oracle):
    """conversations (agent rows name custom and built-in contexts) through scan_redact vs
    oracle.process_rows: redacted bytes, spans and context bit-exact"""
    from oracle import pii_oracle as O
    E = pkg("engine")
    c, _ = c5
    rows = _conversations(c, 300, 12, 7)
    eng = E.Engine(c5_comp.blob, device=0, n_conv_slots=1 << 10)
    res = eng.scan_redact([x[2] for x in rows], [x[0] for x in rows], [x[1] for x in rows], [x[3] for x in rows])
    exp = O.process_rows(rows, c5_oracle)
    groups = list(c5_oracle.context_keywords.keys())
    n_custom = 0
    for i, (red, fs, used, stored) in enumerate(exp):
        assert res.text(i) == red, (i, rows[i][2], res.text(i), red)
        m = res.spans["utt"] == i
        got = [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]
        assert got == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
        want = stored if rows[i][1] == O.ROLE_AGENT else used
        assert int(res.ctx_info[i]) == (groups.index(want) if want is not None else -1), i
        n_custom += sum(c5_oracle.type_names[f.type_id].startswith("CUSTOM_") for f in fs)
    assert n_custom > 500
    # the per-infoType histogram covers all 500+ types
    h = eng.histogram()
    assert len(h) == len(c5_oracle.type_names)
    want = np.zeros(len(h), dtype=np.int64)
    for _, fs, _, _ in exp:
        for f in fs:
            want[f.type_id] += 1
    assert (h.astype(np.int64) == want).all()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["incremental", "full"])
def test_config5_window_rescan(c5, c5_comp, c5_oracle, mode):
    """the aggregator re-scan with 500+ custom types (several SCAN groups) vs
    oracle.process_window_rows, one utterance per conversation per call: incremental (resident
    candidates of every group, VERDICT r3 Missing 1) and the forced full re-scan of the joined windows"""
    from oracle import pii_oracle as O
    E = pkg("engine")
    c, _ = c5
    rows = _conversations(c, 120, 8, 13)
    eng = E.Engine(c5_comp.blob, device=0, n_conv_slots=1 << 9)
    try:
        eng.window_enable(5, 16384, full=mode == "full")
        assert eng.window_mode() == mode
        groups = list(c5_oracle.context_keywords.keys())
        by_conv = {}
        for row in rows:
            by_conv.setdefault(row[0], []).append(row)
        store, hist = O.ContextStore(), {}
        n_custom = 0
        for k in range(8):
            batch = [by_conv[cv][k] for cv in sorted(by_conv) if k < len(by_conv[cv])]
            res = eng.rescan_window([x[2] for x in batch], [x[0] for x in batch], [x[1] for x in batch],
                                    [x[3] for x in batch])
            exp = O.process_window_rows(batch, c5_oracle, n=5, store=store, history=hist)
            for i, (red, fs, et) in enumerate(exp):
                assert res.text(i) == red, (k, i)
                m = res.spans["utt"] == i
                got = [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"]))
                       for s in res.spans[m]]
                assert got == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], (k, i)
                g = int(res.ctx_info[i])
                assert (groups[g] if g >= 0 else None) == et, (k, i)
                n_custom += sum(c5_oracle.type_names[f.type_id].startswith("CUSTOM_") for f in fs)
        assert n_custom > 200
    finally:
        eng.close()


@pytest.mark.gpu
def test_config5_long_rows(c5, c5_comp, c5_oracle):
    """rows of 30-200 KB (cut into lanes, every SCAN group stitched) vs the oracle"""
    from oracle import pii_oracle as O
    E = pkg("engine")
    c, _ = c5
    r = random.Random(11)
    texts = []
    for k in range(6):
        parts, n = [], 0
        target = r.choice([30_000, 80_000, 200_000])
        while n < target:
            p = c.utterance(r, _builtin_value)
            parts.append(p)
            n += len(p) + 1
        texts.append(" ".join(parts).encode())
    eng = E.Engine(c5_comp.blob, device=0, n_conv_slots=64)
    res = eng.scan_redact(texts, [1] * len(texts), [O.ROLE_OTHER] * len(texts))
    for i, t in enumerate(texts):
        red, fs = O.redact(t, c5_oracle, None)
        assert res.text(i) == red, i
        m = res.spans["utt"] == i             # spans too, not only the redacted bytes
        got = [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]
        assert got == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["0", "40"])
def test_config5_merge_walk_fallback(c5, c5_comp, c5_oracle, monkeypatch, cap):
    """k_pairs_merge stages a wavefront's events of every SCAN group and ranks them in LDS; a
    wavefront with more events than PII_MERGE_CAP walks its lanes instead.  cap 0: every wavefront
    walks; cap 40: the two forms side by side in one call.  Bit-exact vs the oracle either way."""
    from oracle import pii_oracle as O
    E = pkg("engine")
    c, _ = c5
    rows = _conversations(c, 120, 8, 19)
    monkeypatch.setenv("PII_MERGE_CAP", cap)
    eng = E.Engine(c5_comp.blob, device=0, n_conv_slots=1 << 8)
    try:
        res = eng.scan_redact([x[2] for x in rows], [x[0] for x in rows], [x[1] for x in rows],
                              [x[3] for x in rows])
        exp = O.process_rows(rows, c5_oracle)
        for i, (red, fs, _, _) in enumerate(exp):
            assert res.text(i) == red, i
            m = res.spans["utt"] == i
            got = [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"])) for s in res.spans[m]]
            assert got == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
    finally:
        eng.close()
