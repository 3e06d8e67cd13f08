"""Host-side mirror of main_service (context-based-pii_amd/service.py): handler shapes, the
reference's error strings, slot mapping, context TTL and realtime join/split.

CPU tests drive PiiService with a test double of the engine whose results come from the oracle
(test infrastructure only); the `gpu` tests drive it with the real HIP engine and compare the whole
handler sequence with the oracle's replay of the reference handlers (main.py:344-466)."""
import json
import time
import os

import numpy as np
import pytest

from conftest import ROOT, pkg


class OracleEngine:
    """Engine test double: same Python surface as engine.Engine, results from oracle/pii_oracle.py."""

    def __init__(self, cfg, n_slots=8, fail_code=None):
        from oracle import pii_oracle as O
        self.O, self.cfg = O, cfg
        self.n_slots = n_slots
        self.group_types = list(cfg.context_keywords.keys())
        self.ctx = {}
        self.fail_code = fail_code
        self.calls = []

    def context_get(self, slot):
        return self.ctx.get(slot, (-1, 0))

    def context_set(self, slot, g, ts):
        self.ctx[slot] = (g, ts)

    def context_resize(self, n):
        assert n >= self.n_slots
        self.n_slots = n

    def context_update(self, texts, slots, roles, ts):
        """the context half alone (pii_context_update): commits AGENT rows' keyword hits"""
        E = pkg("engine")
        if self.fail_code is not None and self.fail_code != E.PII_E_NOMEM:
            raise E.PiiError(self.fail_code, "injected")
        out = []
        for t, s, r, now in zip(texts, slots, roles, ts):
            info = -1
            if r == E.ROLE_AGENT:
                hit = self.O.extract_expected_pii(t, self.cfg)
                if hit:
                    info = self.group_types.index(hit)
                    self.context_set(s, info, now)
            elif r == E.ROLE_CUSTOMER:
                g, t0 = self.context_get(s)
                if g >= 0 and now - t0 < 90_000_000:
                    info = g
            out.append(info)
        return np.array(out, np.int16)

    def scan_redact(self, texts, slots, roles, ts):
        E = pkg("engine")
        if self.fail_code is not None:
            raise E.PiiError(self.fail_code, "injected")
        assert all(0 < s < self.n_slots or s == 0 for s in slots)
        self.calls.append(list(zip(slots, roles)))
        outs, ctx_info = [], []
        for t, s, r, now in zip(texts, slots, roles, ts):
            et = None
            if r == E.ROLE_CUSTOMER:
                g, t0 = self.context_get(s)
                if g >= 0 and now - t0 < 90_000_000:
                    et = self.group_types[g]
            red, _ = self.O.redact(t, self.cfg, et)
            info = -1
            if r == E.ROLE_AGENT:
                hit = self.O.extract_expected_pii(t, self.cfg)
                if hit:
                    info = self.group_types.index(hit)
                    self.context_set(s, info, now)
            elif et is not None:
                info = self.group_types.index(et)
            outs.append(red)
            ctx_info.append(info)
        data, offs = E.pack(outs)
        return E.BatchResult(data, offs, np.zeros(0, E.SPAN_DTYPE), np.array(ctx_info, np.int16))


class Clock:
    def __init__(self, t=1_760_000_000.0):
        self.t = t

    def __call__(self):
        return self.t


@pytest.fixture
def svc(oracle_cfg):
    S = pkg("service")
    clock = Clock()
    s = S.PiiService(engine=OracleEngine(oracle_cfg), clock=clock)
    s._clock = clock
    return s


def test_handler_shapes_and_400s(svc):
    assert svc.handle_agent_utterance(None)[1] == 400
    assert svc.handle_agent_utterance({"transcript": "x"}) == ({"error": "Missing conversation_id or transcript"}, 400)
    assert svc.handle_customer_utterance({"conversation_id": "c"})[1] == 400
    assert svc.redact_utterance_realtime({"conversation_id": "c"}) == ({"error": "Missing conversation_id or utterance"}, 400)
    body, code = svc.handle_agent_utterance({"conversation_id": "c1", "transcript": "Could I get your email address?"})
    assert code == 200 and set(body) == {"redacted_transcript", "context_stored"} and body["context_stored"] is True
    body, code = svc.handle_customer_utterance({"conversation_id": "c1", "transcript": "it is jane.doe@example.com"})
    assert body == {"redacted_transcript": "it is [EMAIL_ADDRESS]", "context_used": True}
    body, _ = svc.handle_customer_utterance({"conversation_id": "c2", "transcript": "hi"})
    assert body == {"redacted_transcript": "hi", "context_used": False}


def test_context_ttl_and_persistence(svc):
    svc.handle_agent_utterance({"conversation_id": "c", "transcript": "What is your card number?"})
    svc._clock.t += 89.0
    assert svc.handle_customer_utterance({"conversation_id": "c", "transcript": "ok"})[0]["context_used"]
    svc.handle_agent_utterance({"conversation_id": "c", "transcript": "Thanks."})      # a miss keeps the record
    assert svc.handle_customer_utterance({"conversation_id": "c", "transcript": "ok"})[0]["context_used"]
    svc._clock.t += 2.0                                                                  # 91 s after the hit
    assert not svc.handle_customer_utterance({"conversation_id": "c", "transcript": "ok"})[0]["context_used"]


def test_error_strings_follow_the_reference(oracle_cfg):
    S, E = pkg("service"), pkg("engine")
    for code, prefix in [(E.PII_E_DEVICE, "[DLP_API_CALL_ERROR]"), (E.PII_E_RULES, "[DLP_TEMPLATE_NOT_FOUND_ERROR]"),
                         (E.PII_E_NOMEM, "[DLP_PROCESSING_ERROR]"), (E.PII_E_ARG, "[DLP_PROCESSING_ERROR]")]:
        s = S.PiiService(engine=OracleEngine(oracle_cfg, fail_code=code))
        assert s.call_dlp_for_redaction("my ssn", None) == f"{prefix} my ssn"
        body, code200 = s.handle_customer_utterance({"conversation_id": "c", "transcript": "t"})
        assert code200 == 200 and body["redacted_transcript"] == f"{prefix} t"


def test_stateless_seam_and_extract(svc, oracle_cfg):
    from oracle import pii_oracle as O
    t = "card 4141-1212-2323-5009 and code 123"
    for ctx in (None, {"expected_pii_type": "CVV_NUMBER"}, {"expected_pii_type": "CREDIT_CARD_NUMBER"}):
        red, _ = O.redact(t.encode(), oracle_cfg, ctx and ctx["expected_pii_type"])
        assert svc.call_dlp_for_redaction(t, ctx) == red.decode()
    assert svc.extract_expected_pii("What's the CVV on the back?") == O.extract_expected_pii(
        b"What's the CVV on the back?", oracle_cfg)
    assert svc.extract_expected_pii("Thanks") is None


def test_slot_map_lru_evicts_and_clears():
    S = pkg("service")
    evicted = []
    m = S.SlotMap(4, on_evict=evicted.append)
    a, b, c = m.get("a"), m.get("b"), m.get("c")
    assert sorted((a, b, c)) == [1, 2, 3]                 # slot 0 reserved
    m.get("a")                                            # a becomes most recent
    d = m.get("d")
    assert d == b and evicted == [b] and m.peek("b") is None and m.get("a") == a


def test_slot_map_keeps_live_contexts_and_grows():
    """Redis keeps context:{id} until its TTL runs out (main.py:163,366-374): a slot whose record is
    still live, or which holds window history, is never reused; the table grows instead (VERDICT r3
    Missing 3)."""
    S = pkg("service")
    evicted, grown = [], []
    m = S.SlotMap(4, on_evict=evicted.append, on_grow=grown.append)
    a, b, c = m.get("a", now_us=0), m.get("b", now_us=0), m.get("c", now_us=0)
    m.note_context(a, 90)
    m.note_context(b, 90)
    m.note_window(c)
    d = m.get("d", now_us=50)                             # every record live / windowed: grow
    assert grown == [8] and evicted == [] and d == 4 and m.n_slots == 8
    for k in range(3):
        m.get(f"x{k}", now_us=50)
    assert m.get("y", now_us=90) == a and evicted == [a]  # a expired at 90: its slot is reused
    assert m.peek("a") is None and m.peek("b") == b and m.peek("c") == c


def test_slot_map_live_block_at_lru_end_does_not_hide_expired_slots():
    """many never-ending (windowed) conversations at the LRU end must not stop the expired
    slots behind them from being reused (the table would double without bound)."""
    S = pkg("service")
    grown = []
    m = S.SlotMap(200, on_grow=grown.append)
    live = [m.get(f"w{k}", now_us=0) for k in range(100)]
    for sl in live:
        m.note_window(sl)
    rest = [m.get(f"e{k}", now_us=0) for k in range(m.capacity - len(live))]
    for sl in rest:
        m.note_context(sl, 10)
    got = [m.get(f"n{k}", now_us=100) for k in range(len(rest))]
    assert grown == [] and sorted(got) == sorted(rest)


def test_slot_map_resize_failure_reuses_any_expired_slot_then_raises():
    """every entry is searched for a reusable slot before the table grows; when it
    cannot grow (no device memory, or max_slots) the PiiError reaches the caller."""
    S, E = pkg("service"), pkg("engine")

    def no_grow(n):
        raise E.PiiError(E.PII_E_NOMEM, "no memory")
    m = S.SlotMap(100, on_grow=no_grow)
    slots = [m.get(f"c{k}", now_us=0) for k in range(m.capacity)]
    for sl in slots[:-1]:
        m.note_context(sl, 1000)                 # live
    m.note_context(slots[-1], 10)                 # expired at 100, the most recently used entry
    assert m.get("x", now_us=100) == slots[-1]
    m.note_context(slots[-1], 1000)
    with pytest.raises(E.PiiError) as ei:
        m.get("y", now_us=100)
    assert ei.value.code == E.PII_E_NOMEM
    cap = S.SlotMap(4, max_slots=4)
    for k in range(3):
        cap.note_context(cap.get(k, now_us=0), 50)
    with pytest.raises(E.PiiError):
        cap.get("z", now_us=10)


class _WindowOracleEngine(OracleEngine):
    """OracleEngine with the window re-scan surface (window_enable / rescan_window): each row joins
    its slot's last window_n utterances (oracle.process_window_rows' rule)."""

    def __init__(self, cfg, n_slots=8, fail_code=None):
        super().__init__(cfg, n_slots, fail_code)
        self.window_n = 0
        self.hist = {}

    def window_enable(self, n, slot_bytes):
        self.window_n = n

    def rescan_window(self, texts, slots, roles, ts):
        E = pkg("engine")
        ctx = self.context_update(texts, slots, roles, ts)
        outs = []
        for t, s, r, now in zip(texts, slots, roles, ts):
            w = self.hist.setdefault(s, [])
            w.append(t)
            del w[:-self.window_n]
            g, t0 = self.context_get(s)
            et = self.group_types[g] if g >= 0 and now - t0 < 90_000_000 else None
            outs.append(self.O.redact(b"\n".join(w), self.cfg, et)[0])
        data, offs = E.pack(outs)
        return E.BatchResult(data, offs, np.zeros(0, E.SPAN_DTYPE), ctx)


class _NoGrowEngine(OracleEngine):
    def context_resize(self, n):
        E = pkg("engine")
        raise E.PiiError(E.PII_E_NOMEM, "injected resize failure")


def test_resize_failure_maps_rows_to_error_strings(oracle_cfg):
    """a slot-table growth failure answers the affected conversations' rows with
    the reference's error string (nothing stored); process_batch / the handlers never raise, and the
    conversations that already hold a slot keep working."""
    from oracle import pii_oracle as O
    S = pkg("service")
    svc = S.PiiService(engine=_NoGrowEngine(oracle_cfg, n_slots=4), clock=Clock(), time_base="payload")
    agent = "Could I get your email address?"
    rows = [{"conversation_id": f"v{c}", "participant_role": "AGENT", "text": agent, "start_timestamp_usec": 10 + c}
            for c in range(5)]
    got = svc.process_batch(rows)
    assert got[:3] == [O.redact(agent.encode(), oracle_cfg, None)[0].decode()] * 3
    assert got[3:] == [f"[DLP_PROCESSING_ERROR] {agent}"] * 2
    cust = "it is jane.doe@example.com"
    got = svc.process_batch([{"conversation_id": "v1", "participant_role": "END_USER", "text": cust,
                              "start_timestamp_usec": 100},
                             {"conversation_id": "v9", "participant_role": "END_USER", "text": cust,
                              "start_timestamp_usec": 100}])
    assert got[0] == O.redact(cust.encode(), oracle_cfg, "EMAIL_ADDRESS")[0].decode()
    assert got[1] == f"[DLP_PROCESSING_ERROR] {cust}"
    body, code = svc.handle_agent_utterance({"conversation_id": "v7", "transcript": agent})
    assert code == 200 and body == {"redacted_transcript": f"[DLP_PROCESSING_ERROR] {agent}", "context_stored": False}
    body, code = svc.handle_customer_utterance({"conversation_id": "v2", "transcript": cust})
    assert code == 200 and body["context_used"] is True
    out = svc.rescan_window_batch([{"conversation_id": "v8", "participant_role": "END_USER", "text": cust,
                                    "start_timestamp_usec": 200}]) if hasattr(svc.engine, "rescan_window") else None
    assert out in (None, [f"[DLP_PROCESSING_ERROR] {cust}"])


def test_window_rescan_without_slots_answers_errors_and_marks_windows(oracle_cfg):
    """the window re-scan of a run some of whose conversations get no slot (the
    table is at max_slots) answers those rows with the reference's error string; the others are
    re-scanned and their slots marked as holding window history (never reused while open)."""
    from oracle import pii_oracle as O
    S = pkg("service")
    svc = S.PiiService(engine=_WindowOracleEngine(oracle_cfg, n_slots=4), clock=Clock(), time_base="payload",
                       max_slots=4)
    cust = "it is jane.doe@example.com"
    rows = [{"conversation_id": f"w{c}", "participant_role": "END_USER", "text": cust, "start_timestamp_usec": 10}
            for c in range(5)]
    got = svc.rescan_window_batch(rows)
    assert got[:3] == [O.redact(cust.encode(), oracle_cfg, None)[0].decode()] * 3
    assert got[3:] == [f"[DLP_PROCESSING_ERROR] {cust}"] * 2
    held = [svc.slots.peek(f"w{c}") for c in range(3)]
    assert all(h is not None for h in held) and all(h in svc.slots.windowed for h in held)
    assert svc.slots.peek("w3") is None and svc.slots.peek("w4") is None
    # a second turn of a windowed conversation joins its window
    got = svc.rescan_window_batch([{"conversation_id": "w0", "participant_role": "END_USER", "text": "ok",
                                    "start_timestamp_usec": 20}])
    assert got == [O.redact(b"\n".join([cust.encode(), b"ok"]), oracle_cfg, None)[0].decode()]


def test_slot_map_growth_failure_is_not_retried_per_conversation():
    """a failed growth is remembered -- a batch of M new conversations makes
    one on_grow attempt (and one victim walk), not M; a released slot allows growth again."""
    S, E = pkg("service"), pkg("engine")
    calls = []

    def no_grow(n):
        calls.append(n)
        raise E.PiiError(E.PII_E_NOMEM, "no memory")
    m = S.SlotMap(8, on_grow=no_grow)
    for k in range(m.capacity):
        m.note_context(m.get(f"c{k}", now_us=0), 1000)        # all live
    out, code = m.assign([f"n{k}" for k in range(50)] + ["c0"], None, 10)
    assert code == E.PII_E_NOMEM and out[:50] == [None] * 50 and out[50] is not None
    assert calls == [16] and m.grow_calls == 1
    for k in range(20):                                         # later calls: no retry for a while
        with pytest.raises(E.PiiError):
            m.get(f"x{k}", now_us=10)
    assert len(calls) == 1
    m.release("c1")
    m.note_context(m.get("y", now_us=10), 1000)               # the freed slot, now live
    with pytest.raises(E.PiiError):
        m.get("z", now_us=10)
    assert len(calls) == 2                                      # growth retried after a release


def test_more_live_conversations_than_slots_match_the_oracle(oracle_cfg):
    """VERDICT r3 Missing 3 (the r03c scenario): 1,300 conversations through a 1,024-slot table, each
    agent's context read by its customer row much later -- every context survives (the table grows),
    results equal the oracle replay."""
    from oracle import pii_oracle as O
    S = pkg("service")
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=1024), clock=Clock(), time_base="payload")
    agent, cust = "Could I get your email address?", "it is jane.doe@example.com and @handle_1"
    rows = [{"conversation_id": f"v{c}", "participant_role": "AGENT", "text": agent, "start_timestamp_usec": 10 + c}
            for c in range(1300)]
    rows += [{"conversation_id": f"v{c}", "participant_role": "END_USER", "text": cust,
              "start_timestamp_usec": 2000 + c} for c in range(1300)]
    got = [svc.process_batch([r])[0] for r in rows]
    exp = O.process_rows([(r["conversation_id"], O.ROLE_AGENT if r["participant_role"] == "AGENT" else
                           O.ROLE_CUSTOMER, r["text"].encode(), r["start_timestamp_usec"]) for r in rows], oracle_cfg)
    assert got == [x[0].decode() for x in exp]
    assert svc.engine.n_slots >= 1301


def test_failed_call_still_stores_agent_context(oracle_cfg):
    """call_dlp_for_redaction never fails the agent handler: extract_expected_pii + SETEX run after
    it (main.py:358-374), so a failed engine call still stores the context (VERDICT r3 Missing 2)."""
    S, E = pkg("service"), pkg("engine")
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, fail_code=E.PII_E_NOMEM), clock=Clock())
    body, _ = svc.handle_agent_utterance({"conversation_id": "f", "transcript": "What is your email address?"})
    assert body == {"redacted_transcript": "[DLP_PROCESSING_ERROR] What is your email address?",
                    "context_stored": True}
    body, _ = svc.handle_customer_utterance({"conversation_id": "f", "transcript": "jane.doe@example.com"})
    assert body == {"redacted_transcript": "[DLP_PROCESSING_ERROR] jane.doe@example.com", "context_used": True}
    svc.engine.fail_code = None
    body, _ = svc.handle_customer_utterance({"conversation_id": "f", "transcript": "jane.doe@example.com"})
    assert body == {"redacted_transcript": "[EMAIL_ADDRESS]", "context_used": True}


def test_realtime_join_split(svc, oracle_cfg):
    from oracle import pii_oracle as O
    agent = "Please confirm your phone number."
    svc.handle_agent_utterance({"conversation_id": "r", "transcript": agent})
    body, _ = svc.redact_utterance_realtime({"conversation_id": "r", "utterance": "it's 555-867-5309"})
    exp = O.realtime_redact(agent.encode(), b"it's 555-867-5309", oracle_cfg, "PHONE_NUMBER")
    assert body == {"redacted_utterance": exp.decode()}
    body, _ = svc.redact_utterance_realtime({"conversation_id": "none", "utterance": "hi 555-867-5309"})
    assert body["redacted_utterance"] == O.redact(b"hi 555-867-5309", oracle_cfg, None)[0].decode()


def _replay_handlers(svc, entries, cid):
    out = []
    for e in entries:
        d = {"conversation_id": cid, "transcript": e["text"]}
        body, _ = (svc.handle_agent_utterance(d) if e["role"] == "AGENT" else svc.handle_customer_utterance(d))
        out.append(body["redacted_transcript"])
    return out


def _oracle_replay(oracle_cfg, entries, cid):
    from oracle import pii_oracle as O
    rows = [(cid, O.ROLE_AGENT if e["role"] == "AGENT" else O.ROLE_CUSTOMER, e["text"].encode(), e["ts"])
            for e in entries]
    return [r[0].decode() for r in O.process_rows(rows, oracle_cfg)]


def test_handler_replay_double(svc, oracle_cfg):
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    for name, t in tr.items():
        assert _replay_handlers(svc, t["entries"], t["conversation_id"]) == _oracle_replay(
            oracle_cfg, t["entries"], t["conversation_id"])


@pytest.mark.gpu
def test_service_on_gpu_matches_oracle(oracle_cfg):
    """The real engine behind the reference's handler sequence, the stateless seam, the realtime
    handler and the batched ingest path -- all vs the oracle replay of main.py:344-466."""
    from oracle import pii_oracle as O
    S = pkg("service")
    clock = Clock()
    svc = S.PiiService(n_slots=64, clock=clock, time_base="payload")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    for name, t in tr.items():
        assert _replay_handlers(svc, t["entries"], t["conversation_id"]) == _oracle_replay(
            oracle_cfg, t["entries"], t["conversation_id"]), name
    for name, t in tr.items():
        rows = [{"conversation_id": "b" + t["conversation_id"], "participant_role": e["role"], "text": e["text"],
                 "start_timestamp_usec": e["ts"]} for e in t["entries"]]
        assert svc.process_batch(rows) == _oracle_replay(oracle_cfg, t["entries"], "b" + t["conversation_id"])
    t = "card 4141-1212-2323-5009, cvv 123, ssn 123-45-6789"
    for g in [None] + list(oracle_cfg.context_keywords.keys()):
        ctx = {"expected_pii_type": g} if g else None
        assert svc.call_dlp_for_redaction(t, ctx) == O.redact(t.encode(), oracle_cfg, g)[0].decode(), g
    agent = "Could you read me the IMEI of the device?"
    svc.handle_agent_utterance({"conversation_id": "rt", "transcript": agent})
    body, _ = svc.redact_utterance_realtime({"conversation_id": "rt", "utterance": "sure 490154203237518"})
    assert body["redacted_utterance"] == O.realtime_redact(agent.encode(), b"sure 490154203237518", oracle_cfg,
                                                           O.extract_expected_pii(agent.encode(), oracle_cfg)).decode()


@pytest.mark.gpu
def test_service_window_rescan_on_gpu(oracle_cfg):
    """The aggregator's re-scan (rescan_window_batch) over the golden transcripts streamed one
    utterance per call, and in one batch, vs oracle.process_window_rows; conversation_ended resets."""
    from oracle import pii_oracle as O
    S = pkg("service")
    svc = S.PiiService(n_slots=64, clock=Clock(), time_base="payload")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    role = {"AGENT": O.ROLE_AGENT}
    for mode in ("stream", "batch"):
        for name, t in tr.items():
            cid = mode + t["conversation_id"]
            rows = [{"conversation_id": cid, "participant_role": e["role"], "text": e["text"],
                     "start_timestamp_usec": e["ts"]} for e in t["entries"]]
            exp = [r.decode() for r, _, _ in O.process_window_rows(
                [(cid, role.get(e["role"], O.ROLE_CUSTOMER), e["text"].encode(), e["ts"]) for e in t["entries"]],
                oracle_cfg, n=5)]
            got = [svc.rescan_window_batch([r])[0] for r in rows] if mode == "stream" else svc.rescan_window_batch(rows)
            assert got == exp, (mode, name)
            slot = svc.slots.peek(cid)
            svc.conversation_ended(cid)
            assert svc.engine.window_count(slot) == 0 and svc.engine.context_get(slot)[0] == -1
            assert svc.slots.peek(cid) is None


def _pubsub_payloads(tr):
    """The golden transcripts as raw Pub/Sub payloads (main_service/main.py:295-302), interleaved
    across conversations and shuffled (seeded): the stream order the subscriber sees."""
    import random
    out = []
    for name, t in tr.items():
        for e in t["entries"]:
            out.append({"conversation_id": "ps" + t["conversation_id"], "original_entry_index": e["i"],
                        "participant_role": e["role"].lower(), "text": e["text"], "user_id": "u-" + name,
                        "start_timestamp_usec": e["ts"]})
    random.Random(20250718).shuffle(out)
    return out


def _check_pubsub(svc, oracle_cfg):
    S = pkg("service")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    pay = _pubsub_payloads(tr)
    bad = [{"conversation_id": "x", "original_entry_index": 0, "participant_role": "AGENT", "text": "  ",
            "start_timestamp_usec": 1}, {"conversation_id": "x", "text": "hi"},
           {"conversation_id": "ps" + next(iter(tr.values()))["conversation_id"], "original_entry_index": 999,
            "participant_role": "system", "text": "card 4141-1212-2323-5009", "start_timestamp_usec": 1}]
    res = svc.process_pubsub_batch(pay + bad)
    assert res[-3]["status"] == 400 and res[-3]["missing_fields"] == ["text"]
    assert res[-2]["status"] == 400 and "original_entry_index" in res[-2]["missing_fields"]
    # subscriber_service/main.py:265-266: an unknown role is skipped (200, nothing published)
    assert res[-1]["status"] == 200 and "skipped" in res[-1] and "text" not in res[-1]
    archive = S.TranscriptArchive()
    archive.add(res)
    for name, t in tr.items():
        cid = "ps" + t["conversation_id"]
        want = _oracle_replay(oracle_cfg, sorted(t["entries"], key=lambda e: e["i"]), cid)
        got = {p["original_entry_index"]: p for p in res if p.get("conversation_id") == cid}
        for e, w in zip(sorted(t["entries"], key=lambda e: e["i"]), want):
            p = got[e["i"]]
            assert p["text"] == w and p["original_text"] == e["text"]
            assert p["participant_role"] == e["role"].upper() and p["user_id"] == "u-" + name
        body = archive.conversation_ended(cid)
        ent = json.loads(body)["entries"]
        assert [x["original_entry_index"] for x in ent] == sorted(e["i"] for e in t["entries"])
        assert [x["text"] for x in ent] == want
    assert archive.conversation_ended("nope") is None


def test_pubsub_batch_and_archive(oracle_cfg):
    """§8(f) stream formats over the engine double: shuffled raw payloads in, redacted payloads
    (subscriber_service/main.py:213-221) out in input order, bad payloads 400, unknown roles
    skipped, and the aggregator's {"entries": [...]} object (transcript_aggregator_service/main.py:
    220-247)."""
    S = pkg("service")
    _check_pubsub(S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=64), clock=Clock(), time_base="payload"),
                  oracle_cfg)


@pytest.mark.gpu
def test_pubsub_batch_and_archive_on_gpu(oracle_cfg):
    S = pkg("service")
    _check_pubsub(S.PiiService(n_slots=64, clock=Clock(), time_base="payload"), oracle_cfg)


# ------------------------------------------------------------------ batching, time base, Flask shim
def _requests(seed=3, n_conv=6, n=120):
    """A seeded interleaving of handler requests over a few conversations (agent questions with
    context keywords, customer answers with PII, realtime chat lines)."""
    import random
    r = random.Random(seed)
    asks = ["Could I get your email address?", "What is your card number?", "Please confirm your phone number.",
            "Can you read me the CVV?", "What's your date of birth?", "Thanks.", "What is your SSN?"]
    answers = ["it is jane.doe@example.com", "4141-1212-2323-5009", "sure, 555-867-5309", "123",
               "01/22/1985", "ok", "123-45-6789", "my ip address is 10.0.0.1"]
    out = []
    for _ in range(n):
        cid = f"c{r.randrange(n_conv)}"
        k = r.random()
        if k < 0.35:
            out.append(("agent", {"conversation_id": cid, "transcript": r.choice(asks)}))
        elif k < 0.75:
            out.append(("customer", {"conversation_id": cid, "transcript": r.choice(answers)}))
        elif k < 0.97:
            out.append(("realtime", {"conversation_id": cid, "utterance": r.choice(answers)}))
        else:
            out.append(("customer", {"conversation_id": cid}))          # 400
    return out


def _sequential(make_svc, reqs):
    s = make_svc()
    fn = {"agent": s.handle_agent_utterance, "customer": s.handle_customer_utterance,
          "realtime": s.redact_utterance_realtime}
    return [fn[k](d) for k, d in reqs]


def test_process_requests_equals_sequential_handlers(oracle_cfg):
    S = pkg("service")
    reqs = _requests()
    make = lambda: S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=16), clock=Clock())
    want = _sequential(make, reqs)
    svc = make()
    got = svc.process_requests(reqs)
    assert got == want
    # fewer engine calls than requests: concurrent requests share an engine call
    assert len(svc.engine.calls) < len(reqs) // 4


def test_batch_larger_than_slot_table_never_mixes_conversations(oracle_cfg):
    """more conversations in one batch than slots must not evict a conversation of the
    same engine call (n_slots=4: 3 usable slots, 9 conversations): the table grows."""
    S = pkg("service")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=4), clock=Clock(), time_base="payload")
    rows, want = [], []
    for k in range(3):
        for name, t in tr.items():
            cid = f"{k}-{t['conversation_id']}"
            rows += [{"conversation_id": cid, "participant_role": e["role"], "text": e["text"],
                      "start_timestamp_usec": e["ts"]} for e in t["entries"]]
            want += _oracle_replay(oracle_cfg, t["entries"], cid)
    assert svc.process_batch(rows) == want
    assert len(svc.engine.calls) == 1 and len({s for s, _ in svc.engine.calls[0]}) == 9 and svc.engine.n_slots == 16


def test_batch_paths_never_raise_on_engine_errors(oracle_cfg):
    S, E = pkg("service"), pkg("engine")
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, fail_code=E.PII_E_DEVICE), clock=Clock())
    rows = [{"conversation_id": "a", "participant_role": "AGENT", "text": "hi", "start_timestamp_usec": 1}]
    assert svc.process_batch(rows) == ["[DLP_API_CALL_ERROR] hi"]
    pay = [dict(rows[0], original_entry_index=0, participant_role="END_USER", text="t")]
    assert svc.process_pubsub_batch(pay)[0]["text"] == "[DLP_API_CALL_ERROR] t"


def test_one_time_base_for_batch_and_realtime(oracle_cfg):
    """payload-stamped batch rows and the realtime handler share one clock."""
    from oracle import pii_oracle as O
    S = pkg("service")
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=16), clock=Clock(5.0), time_base="payload")
    t0 = 1_700_000_000_000_000
    agent = "Please confirm your phone number."
    svc.process_pubsub_batch([{"conversation_id": "m", "original_entry_index": 0, "participant_role": "AGENT",
                               "text": agent, "start_timestamp_usec": t0}])
    body, _ = svc.redact_utterance_realtime({"conversation_id": "m", "utterance": "it's 555-867-5309"})
    assert body["redacted_utterance"] == O.realtime_redact(agent.encode(), b"it's 555-867-5309", oracle_cfg,
                                                           "PHONE_NUMBER").decode()
    # wall-clock service: batch rows are stamped at processing time like the reference's time.time()
    clock = Clock()
    svc2 = S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=16), clock=clock)
    svc2.process_batch([{"conversation_id": "m", "participant_role": "AGENT", "text": agent,
                         "start_timestamp_usec": t0}])
    assert svc2.handle_customer_utterance({"conversation_id": "m", "transcript": "x"})[0]["context_used"]
    clock.t += 91
    assert not svc2.handle_customer_utterance({"conversation_id": "m", "transcript": "x"})[0]["context_used"]


def test_conversation_ended_drops_context(svc):
    svc.handle_agent_utterance({"conversation_id": "e", "transcript": "What is your card number?"})
    assert svc.handle_customer_utterance({"conversation_id": "e", "transcript": "ok"})[0]["context_used"]
    slot = svc.slots.peek("e")
    svc.conversation_ended("e")
    assert svc.slots.peek("e") is None and slot not in svc.agent_text
    assert svc.engine.context_get(slot)[0] == -1
    assert not svc.handle_customer_utterance({"conversation_id": "e", "transcript": "ok"})[0]["context_used"]


def test_non_group_expected_type_has_a_variant():
    """Every engine type is a context group (keyword-less pseudo groups for the rest), so
    call_dlp_for_redaction honours any expected_pii_type it can detect (main.py:614-686)."""
    import copy
    C = pkg("compiler")
    rules = C.Rules.load()
    raw = copy.deepcopy(rules.raw)
    raw["context_keywords"] = {k: v for k, v in raw["context_keywords"].items() if k != "CVV_NUMBER"}
    r2 = C.Rules(raw, rules_builtin())
    names = [t for t, _, _ in r2.kw_groups]
    assert "CVV_NUMBER" in names and names.index("CVV_NUMBER") >= r2.n_keyword_groups
    assert r2.kw_groups[names.index("CVV_NUMBER")][1] is None


def rules_builtin():
    import yaml
    with open(os.path.join(ROOT, "context-based-pii_amd", "rules", "builtin_infotypes.yaml")) as f:
        return yaml.safe_load(f)


def _flask_app(svc, **kw):
    A = pkg("app")
    return A.create_app(svc, **kw)


def test_flask_routes_shapes_and_microbatching(oracle_cfg):
    import threading
    S = pkg("service")
    reqs = _requests(seed=11, n_conv=8, n=160)
    make = lambda: S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=32), clock=Clock())
    app = _flask_app(make(), max_wait_s=0.02)
    client = app.test_client()
    route = {"agent": "/handle-agent-utterance", "customer": "/handle-customer-utterance",
             "realtime": "/redact-utterance-realtime"}
    r = client.post(route["agent"], json={"transcript": "x"})
    assert r.status_code == 400 and r.get_json() == {"error": "Missing conversation_id or transcript"}
    # one thread per conversation, each posting its own requests in order (per-conversation order is
    # what the reference's sequential handlers define); the batcher coalesces across threads
    by_conv = {}
    for i, (k, d) in enumerate(reqs):
        by_conv.setdefault(d["conversation_id"], []).append(i)
    got = [None] * len(reqs)

    def worker(idx):
        c = app.test_client()
        for i in idx:
            k, d = reqs[i]
            resp = c.post(route[k], json=d)
            got[i] = (resp.get_json(), resp.status_code)
    th = [threading.Thread(target=worker, args=(v,)) for v in by_conv.values()]
    for t in th:
        t.start()
    for t in th:
        t.join()
    # expected: each conversation's requests handled in its own order (conversations independent)
    want = [None] * len(reqs)
    for idx in by_conv.values():
        for i, w in zip(idx, _sequential(make, [reqs[i] for i in idx])):
            want[i] = w
    assert got == want
    assert max(app.config["PII_BATCHER"].batches) > 1
    app.config["PII_BATCHER"].close()


def test_malformed_request_fails_alone(oracle_cfg):
    """A body the reference's handler would crash on is that request's own error, never its
    micro-batch's: the well-formed requests batched with it get their sequential answers."""
    S = pkg("service")
    make = lambda: S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=32), clock=Clock())
    good = [("agent", {"conversation_id": "g1", "transcript": "What is your email address?"}),
            ("customer", {"conversation_id": "g1", "transcript": "it is jane.doe@example.com"}),
            ("customer", {"conversation_id": "g2", "transcript": "my ssn is 123-45-6789"})]
    bad = [("customer", ["conversation_id", "transcript"]),                 # JSON list body
           ("customer", "conversation_id transcript"),                     # JSON string body
           ("agent", {"conversation_id": "b", "transcript": None}),         # null text
           ("customer", {"conversation_id": "b", "transcript": 7}),         # non-string text
           ("realtime", {"conversation_id": ["x"], "utterance": "hi"}),     # unhashable id
           ("agent", 5),                                                    # number body
           ("agent", {"conversation_id": "b"})]                             # missing key -> 400
    mixed = [good[0], bad[0], bad[1], good[1], bad[2], bad[3], bad[4], good[2], bad[5], bad[6]]
    got = make().process_requests(mixed)
    want_good = _sequential(make, good)
    assert [got[0], got[3], got[7]] == want_good
    assert [got[i][1] for i in (1, 2, 4, 5, 6, 8, 9)] == [500, 500, 500, 500, 500, 500, 400]
    # and through the Flask micro-batcher: a request that still raises inside the batch (an engine
    # double that fails on one text) only fails itself
    svc = make()
    real = svc._run

    def flaky(texts, *a):
        if b"boom" in texts:
            raise RuntimeError("unforeseen")
        return real(texts, *a)
    svc._run = flaky
    A = pkg("app")
    mb = A.MicroBatcher(svc, max_wait_s=0.05)
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(4) as ex:
        futs = [ex.submit(mb.submit, k, d) for k, d in
                [good[2], ("customer", {"conversation_id": "z", "transcript": "boom"}), good[0]]]
        res = []
        for f in futs:
            try:
                res.append(f.result())
            except RuntimeError:
                res.append("raised")
    mb.close()
    assert res[1] == "raised" and res[0][1] == 200 and res[2][1] == 200


def test_microbatch_failure_after_a_committed_sub_batch_runs_nothing_twice(oracle_cfg):
    """A micro-batch splits into engine calls (a realtime request after an agent request of its
    conversation starts a new one).  When a later call raises, the earlier call's requests are
    committed -- the agent's context is stored -- so the batcher answers them from the partial
    result and re-runs only the failed rest (running them again stored contexts twice)."""
    S = pkg("service")
    svc = S.PiiService(engine=OracleEngine(oracle_cfg, n_slots=32), clock=Clock())
    real = svc._run
    agent_text = b"What is your email address?"
    runs = {"agent": 0}

    def flaky(texts, *a):
        if any(agent_text == t for t in texts):
            runs["agent"] += 1
        if any(b"boom" in t for t in texts):
            raise RuntimeError("unforeseen")
        return real(texts, *a)
    svc._run = flaky
    reqs = [("agent", {"conversation_id": "c1", "transcript": agent_text.decode()}),
            ("realtime", {"conversation_id": "c1", "utterance": "boom"})]
    with pytest.raises(S.PartialBatchError) as ei:
        svc.process_requests(reqs)
    assert set(ei.value.done) == {0} and ei.value.done[0][1] == 200
    assert runs["agent"] == 1
    A = pkg("app")
    mb = A.MicroBatcher(svc, max_wait_s=0.05)
    import concurrent.futures as cf
    runs["agent"] = 0
    with cf.ThreadPoolExecutor(2) as ex:
        f0 = ex.submit(mb.submit, *reqs[0])
        time.sleep(0.005)
        f1 = ex.submit(mb.submit, *reqs[1])
        r0 = f0.result()
        with pytest.raises(RuntimeError):
            f1.result()
    mb.close()
    assert r0[1] == 200 and runs["agent"] == 1


@pytest.mark.gpu
def test_flask_concurrent_requests_on_gpu(oracle_cfg):
    """The Flask shim on the real engine: 8 client threads replay the golden transcripts' handler
    sequence concurrently (one conversation each); every response equals the oracle replay."""
    import threading
    S = pkg("service")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    svc = S.PiiService(n_slots=64, clock=Clock())
    app = _flask_app(svc, max_wait_s=0.005)
    convs = []
    for k in range(8):
        name, t = list(tr.items())[k % len(tr)]
        convs.append((f"f{k}-{t['conversation_id']}", t["entries"]))
    got = {}

    def worker(cid, entries):
        c = app.test_client()
        out = []
        for e in entries:
            route = "/handle-agent-utterance" if e["role"] == "AGENT" else "/handle-customer-utterance"
            out.append(c.post(route, json={"conversation_id": cid, "transcript": e["text"]}).get_json())
        got[cid] = out
    th = [threading.Thread(target=worker, args=c) for c in convs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for cid, entries in convs:
        # the handlers stamp with the (fixed) wall clock: no TTL expiry inside a conversation
        want = _oracle_replay(oracle_cfg, [dict(e, ts=0) for e in entries], cid)
        assert [b["redacted_transcript"] for b in got[cid]] == want, cid
    assert max(app.config["PII_BATCHER"].batches) > 1
    app.config["PII_BATCHER"].close()


@pytest.mark.gpu
def test_service_maps_engine_nomem_and_capacity_to_processing_error(oracle_cfg):
    """The engine runs out of device memory (its work buffers capped with pii_set_scratch_limit) inside
    a batch, a handler call and a queue-overflow re-run: every row gets the reference's
    "[DLP_PROCESSING_ERROR] {transcript}" (main.py:770-773), nothing is committed, and the same calls
    succeed once the limit is lifted.  A device call whose output buffer is too small reports
    PII_E_CAPACITY, which maps to the same string."""
    import torch
    from oracle import pii_oracle as O
    S, E = pkg("service"), pkg("engine")
    svc = S.PiiService(n_slots=1024, clock=Clock(), time_base="payload")     # 1300 conversations below: the table grows
    eng = svc.engine
    small = [{"conversation_id": "s", "participant_role": "AGENT", "text": "What is your email address?",
              "start_timestamp_usec": 1}]
    assert svc.process_batch(small) == ["What is your email address?"]
    svc.process_batch([dict(small[0], conversation_id="w", text="x" * 4096)])   # staging sized for 4 KiB calls
    eng.set_scratch_limit(eng.scratch_bytes())                 # no room to grow any work buffer
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    texts = [e["text"] for t in tr.values() for e in t["entries"]] * 400             # ~0.5 MB
    big = [{"conversation_id": f"b{i // 20}", "participant_role": "AGENT" if i % 2 == 0 else "END_USER",
            "text": t, "start_timestamp_usec": 10 + i} for i, t in enumerate(texts)]
    out = svc.process_batch(big)
    assert out == [f"[DLP_PROCESSING_ERROR] {r['text']}" for r in big]
    long_t = " ".join(texts[:2000])
    body, code = svc.handle_customer_utterance({"conversation_id": "s", "transcript": long_t})
    # (context_used reports the context record, as the reference's Redis GET does, main.py:425)
    assert code == 200 and body == {"redacted_transcript": f"[DLP_PROCESSING_ERROR] {long_t}", "context_used": True}
    # the failed batch still stored its agent rows' context (main.py:358-374), split until it fit
    exp = O.process_rows([(r["conversation_id"], O.ROLE_AGENT if r["participant_role"] == "AGENT" else O.ROLE_CUSTOMER,
                           r["text"].encode(), r["start_timestamp_usec"]) for r in big], oracle_cfg)
    store = {}
    for r, x in zip(big, exp):
        if x[3]:
            store[r["conversation_id"]] = x[3]
    for cid in ("b0", "b7", "b64"):
        g = eng.context_get(svc.slots.peek(cid))[0]
        assert (eng.group_types[g] if g >= 0 else None) == store.get(cid), cid

    eng.set_scratch_limit(0)
    out = svc.process_batch(big)
    rows = [(r["conversation_id"], O.ROLE_AGENT if r["participant_role"] == "AGENT" else O.ROLE_CUSTOMER,
             r["text"].encode(), r["start_timestamp_usec"]) for r in big]
    assert out == [x[0].decode() for x in O.process_rows(rows, oracle_cfg)]
    # PII_E_CAPACITY from the device entry point (a caller-sized output buffer that is too small)
    data, offs = E.pack([b"my email is jane.doe@example.com"] * 4)
    dev = torch.device("cuda:0")
    d_t = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).to(dev)
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    z32, z8, z64 = (torch.zeros(4, dtype=d, device=dev) for d in (torch.int32, torch.uint8, torch.int64))
    out_b = torch.empty(16, dtype=torch.uint8, device=dev)
    oo = torch.empty(5, dtype=torch.int64, device=dev)
    sp = torch.empty(64 * 16, dtype=torch.uint8, device=dev)
    eng.scan_redact_device_ex(d_t.data_ptr(), d_o.data_ptr(), 4, 0, int(offs[-1]), z32.data_ptr(), z8.data_ptr(),
                              z64.data_ptr(), out_b.data_ptr(), 16, oo.data_ptr(), sp.data_ptr(), 64)
    with pytest.raises(E.PiiError) as ei:
        eng.sync()
    assert ei.value.code == E.PII_E_CAPACITY
    assert S.error_string(ei.value.code, "x") == "[DLP_PROCESSING_ERROR] x"
    eng.close()
