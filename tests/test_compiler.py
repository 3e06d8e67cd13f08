"""Rule compiler (host): DFA construction vs Python `re`, relaxation superset, blob format, and the
whole table-driven algorithm (tests/tablesim.py) vs the CPU oracle.  CPU only."""
import random
import re

import numpy as np
import pytest

from conftest import pkg


@pytest.fixture(scope="module")
def C():
    return pkg("compiler")


@pytest.fixture(scope="module")
def sim(compiled):
    from tablesim import TableSim
    return TableSim(compiled)


def _first_dfa(C, pattern):
    nfa = C.NFA()
    st = C.add_pattern(nfa, pattern, 0, reverse=False)
    return C.build_first_dfa(nfa, st)


def _run_first(d, text: bytes, s: int) -> int:
    W = pkg("compiler").WORD
    st = d.start[0 if s == 0 else (1 if (W >> text[s - 1]) & 1 else 2)]
    last = -1
    for j in range(s, len(text)):
        st = int(d.trans[st, d.cmap[text[j]]])
        if d.flags[st] & 1:
            last = j
        if d.flags[st] & 2:
            return last
    st = int(d.trans[st, -1])
    if d.flags[st] & 1:
        last = len(text)
    return last


DIALECT = [
    r"a{0,1}(?:ab){0,1}b",            # leftmost-first != leftmost-longest
    r"\bfoo\b", r"\Bx+", r"(?i)x[^a]y", r"[a-c]+@\w", r"\Ax\d", r"x\d\Z", r"(?:ab|a)(?:bc|c)?",
    r"\d{2,4}?z", r"(?i)(?:social security|ssn)", r".+", r"[^\s]{3}", r"a|ab|abc",
]


@pytest.mark.parametrize("pat", DIALECT)
def test_first_dfa_matches_re(C, pat):
    d = _first_dfa(C, pat)
    rx = re.compile(pat.encode())
    r = random.Random(hash(pat) & 0xffff)
    alpha = b"abcxyzfo09 _@ABXY\n"
    for _ in range(600):
        t = bytes(r.choice(alpha) for _ in range(r.randrange(0, 12)))
        for s in range(len(t) + 1):
            m = rx.match(t, s)
            want = m.end() if m and m.end() > s else (-1 if not m else m.end())
            if m and m.end() == s:
                continue          # empty matches are rejected by the compiler for real rules
            assert _run_first(d, t, s) == want, (pat, t, s)


def test_rejects_unsupported(C):
    for bad in [r"a*", r"(a)\1", r"a(?=b)", r"x$", r"(?m)^x", r"(?:a*)*b"]:
        with pytest.raises(C.RuleError):
            nfa = C.NFA()
            C.add_pattern(nfa, bad, 0, reverse=False)


def test_relaxed_scan_is_superset_of_true_starts(compiled, sim):
    """Every start where a detector matches (re.match) is reported by SCAN-D with that pattern."""
    r = random.Random(3)
    alpha = b"0123456789 -./@:()abcXYZAEI_%+,\n'"
    pats = [re.compile(p.pattern.encode()) for p in compiled.rules.patterns]
    for _ in range(400):
        t = bytes(r.choice(alpha) for _ in range(r.randrange(1, 50)))
        ev = sim.scan(t, True)
        reported = {}
        for pos, sd, sk in ev:
            cd, _ = sim._classes(t, pos)
            a = int(sim.dacc[sd, cd])
            reported[pos] = {int(sim.d_ids[i]) for i in range(int(sim.d_off[a]), int(sim.d_off[a + 1]))}
        for pid, rx in enumerate(pats):
            for s in range(len(t)):
                m = rx.match(t, s)
                if m and m.end() > s:
                    assert pid in reported.get(s, set()), (compiled.rules.patterns[pid].type_name, t, s)


def test_digit_run_prefixes_stay_supersets(compiled, sim):
    """The exact digit-run prefixes (passport 8-9 digits, 10-digit phone / DOD id: the SCAN automaton
    counts the run and checks its closing boundary) still report every true start: runs of 1-20 digits
    with letter / separator neighbours, where an off-by-one in the count would drop a match."""
    r = random.Random(11)
    pats = [re.compile(p.pattern.encode()) for p in compiled.rules.patterns]
    names = {"US_PASSPORT", "PHONE_NUMBER", "DOD_ID_NUMBER"}
    pids = [i for i, p in enumerate(compiled.rules.patterns) if p.type_name in names]
    assert pids
    for _ in range(600):
        parts = []
        for _ in range(r.randrange(1, 4)):
            parts.append(r.choice([b"", b"A", b"x", b" ", b"-", b"(", b"Z"]))
            parts.append(bytes(r.choice(b"0123456789") for _ in range(r.randrange(1, 21))))
            parts.append(r.choice([b"", b" ", b".", b"a", b"_", b"-"]))
        t = b"".join(parts)
        ev = sim.scan(t, True)
        reported = {}
        for pos, sd, sk in ev:
            cd, _ = sim._classes(t, pos)
            a = int(sim.dacc[sd, cd])
            reported[pos] = {int(sim.d_ids[i]) for i in range(int(sim.d_off[a]), int(sim.d_off[a + 1]))}
        for pid in pids:
            for s in range(len(t)):
                m = pats[pid].match(t, s)
                if m and m.end() > s:
                    assert pid in reported.get(s, set()), (compiled.rules.patterns[pid].type_name, t, s)


def test_blob_roundtrip(C, compiled):
    back = C.blob_sections(compiled.blob)
    assert list(back) == list(compiled.sections)
    for k in back:
        assert np.array_equal(back[k], compiled.sections[k]), k


def test_scan_tables_fit_lds(compiled):
    m = compiled.sections["meta"]
    lds = 512 + int(m[4]) * int(m[5]) * 2 + int(m[7]) * int(m[8]) * 2
    assert lds < 64 * 1024


def _check(sim, oracle_cfg, text, g):
    from oracle import pii_oracle as O
    groups = list(oracle_cfg.context_keywords.keys())
    ev = sim.scan(text, True)
    kg = sim.keyword_group(text, ev)
    assert (groups[kg] if kg >= 0 else None) == O.extract_expected_pii(text, oracle_cfg), text
    got = sim.resolve(text, ev, 0 if g < 0 else 1 + g)
    exp = [(f.start, f.end, f.type_id, f.likelihood) for f in O.find_pii(text, oracle_cfg, groups[g] if g >= 0 else None)]
    assert got == exp, (text, g, got, exp)


def test_tables_vs_oracle_synthetic(sim, oracle_cfg):
    synth = pkg("synth")
    bank = synth.build_bank(300, 700, seed=5)
    r = random.Random(2)
    for t in bank.texts:
        _check(sim, oracle_cfg, t, r.randrange(-1, len(oracle_cfg.context_keywords)))


def test_tables_vs_oracle_random_and_mutated(sim, oracle_cfg):
    from test_gpu_parity import _mutated
    synth = pkg("synth")
    r = random.Random(9)
    alpha = b"0123456789 -./@:()abcXYZAEI_%+,\n'\xc3\xa9"
    for i in range(1500):
        t = _mutated(r, synth) if i % 2 else bytes(r.choice(alpha) for _ in range(r.randrange(0, 60)))
        _check(sim, oracle_cfg, t, r.randrange(-1, len(oracle_cfg.context_keywords)))


def test_context_variants_for_types_without_rule_sets(C):
    """A custom rule set where the context branch appends the '.+' rule (main.py:673-686)."""
    import copy
    import json
    import os
    rules = C.Rules.load()
    raw = copy.deepcopy(rules.raw)
    raw["inspect_config"]["rule_set"] = raw["inspect_config"]["rule_set"][:1]     # keep only rule set 1
    builtin = {"detectors": {"CVV_NUMBER": [{"pattern": r"\b\d{3,4}\b", "likelihood": "UNLIKELY"}]}}
    r2 = C.Rules(raw, builtin)
    comp = C.compile_rules(r2)
    from tablesim import TableSim
    sim = TableSim(comp)
    g = [t for t, _, _ in r2.kw_groups].index("CVV_NUMBER")
    t = b"code 123 ok"
    ev = sim.scan(t, True)
    assert sim.resolve(t, ev, 0) == []                          # UNLIKELY, no hotword rule
    got = sim.resolve(t, ev, 1 + g)                             # expected type CVV: '.+' boost
    assert [(s, e, comp.rules.type_names[ty], lk) for s, e, ty, lk in got] == [(5, 8, "CVV_NUMBER", 5)]
