"""CPU check of the incremental window re-scan algorithm (a12) that the HIP kernels implement.

tests/tablesim.py restates k_win_eval/k_win_cands (per-utterance resident candidates: finditer,
validators, hotword bits with proximity windows clipped to the utterance) and k_win_select (window
variant, hotword halo re-check across "\\n", exclusion, overlap).  Here that composition is checked
against the oracle's FULL re-scan of the joined window (oracle.window_rescan / process_window_rows),
so the decomposition the engine relies on is pinned without a GPU.
"""
import random

import pytest

from conftest import pkg
from tablesim import TableSim


@pytest.fixture(scope="module")
def sim(compiled):
    return TableSim(compiled)


def _windows_equal(sim, oracle_cfg, texts, et, history=()):
    """texts = the window; `history` = utterances before it (they shaped the residents' halo bits)"""
    from oracle import pii_oracle as O
    v = 0 if et is None else 1 + list(oracle_cfg.context_keywords.keys()).index(et)
    conv = list(history) + list(texts)
    n0 = len(history)
    entries = [(conv[i], sim.resident_cands(conv[i], conv[max(0, i - 4):i])) for i in range(n0, len(conv))]
    W, kept = sim.window_select(entries, v)
    red, fs = O.redact(W, oracle_cfg, et)
    assert sim.redact(W, kept) == red, (texts, et)
    assert kept == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], (texts, et)


def test_compiled_rules_allow_incremental_windows(compiled):
    assert int(compiled.sections["meta"][13]) == 1


def test_hotword_halo_across_utterances(sim, oracle_cfg):
    """the SSN's hotword sits in the previous utterance: only the window sees it"""
    groups = list(oracle_cfg.context_keywords.keys())
    for et in [None] + groups[:6]:
        _windows_equal(sim, oracle_cfg, [b"please read me your social security", b"987654321 thanks"], et)
        _windows_equal(sim, oracle_cfg, [b"ok", b"what's your driver's license", b"",
                                         b"G223456789", b"and passport E98765432"], et)
        _windows_equal(sim, oracle_cfg, [b"card number", b"\n", b"4141 1212 2323 5009"], et)
        # the hotword sat in an utterance that has left the window: the resident halo bits must not leak
        _windows_equal(sim, oracle_cfg, [b"x", b"987654321 thanks"], et, history=[b"your social security"])
        _windows_equal(sim, oracle_cfg, [b"987654321 thanks"], et, history=[b"ssn", b"is"])


def test_window_random_synthetic(sim, oracle_cfg):
    synth = pkg("synth")
    bank = synth.build_bank(300, 700, seed=3)
    corp = synth.make_corpus(12, 20, bank, seed=9)
    rng = random.Random(4)
    groups = [None] + list(oracle_cfg.context_keywords.keys())
    texts = [corp.data[int(corp.offsets[i]):int(corp.offsets[i + 1])].tobytes() for i in range(corp.n)]
    for _ in range(200):
        n = rng.randint(1, 5)
        i = rng.randrange(0, len(texts) - n - 4)
        conv = texts[i:i + n + 4]
        if rng.random() < 0.4:                      # short rows: hotword windows span several rows
            conv = [w[-rng.randint(0, 30):] if w else w for w in conv]
        h = rng.randint(0, 4)                        # utterances already dropped from the window
        _windows_equal(sim, oracle_cfg, conv[h:h + n], rng.choice(groups), history=conv[:h])


def test_process_window_rows_context(oracle_cfg):
    """the oracle replay: windows of N, the context a row after would see, any role"""
    from oracle import pii_oracle as O
    rows = [("c", O.ROLE_AGENT, b"Can I get your email address?", 0),
            ("c", O.ROLE_CUSTOMER, b"sure it is", 1_000_000),
            ("c", O.ROLE_CUSTOMER, b"jane.doe@example.com", 2_000_000),
            ("d", O.ROLE_CUSTOMER, b"hello", 0)]
    out = O.process_window_rows(rows, oracle_cfg, n=2)
    assert out[2][0] == b"sure it is\n[EMAIL_ADDRESS]"
    assert out[2][2] == "EMAIL_ADDRESS" and out[3][2] is None
    assert out[0][2] == "EMAIL_ADDRESS"        # an agent row's own hit is the window's context
