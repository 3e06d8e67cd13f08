"""Host-side mirror of the reference's main_service hot path, over the HIP engine's C-ABI.

The reference (iyngr/context-based-pii, main_service/main.py) exposes the path as four functions;
this module keeps their names, argument meaning, return shapes and error behaviour:

* ``call_dlp_for_redaction(transcript, context)``  main.py:580-773 -- str in, str out, never raises;
  engine errors map onto the reference's ``[DLP_*_ERROR] {transcript}`` strings (main.py:752-773).
* ``extract_expected_pii(transcript)``             main.py:558-578 -- the first YAML type whose
  keyword occurs (ASCII lower-case substring), or None.
* ``handle_agent_utterance(data)``                 main.py:344-384 -- ({redacted_transcript,
  context_stored}, 200); the context record moves from Redis (SETEX 90 s, main.py:366-374) into the
  engine's HBM table.
* ``handle_customer_utterance(data)``              main.py:386-425 -- ({redacted_transcript,
  context_used}, 200).
* ``redact_utterance_realtime(data)``              main.py:427-466 -- ({redacted_utterance}, 200):
  agent transcript + "\\n" + utterance, redacted with the context, last line kept.

Conversation ids map onto engine context slots (``SlotMap``, least-recently-used reuse).  The agent
transcript of the last keyword hit -- the record's ``agent_transcript`` field -- is host data (only
the realtime handler reads it) and lives beside the slot map; its expiry follows the engine's TTL.

Throughput path: ``process_batch`` runs many rows in one engine call (the batch contract of
include/pii_engine.h: a conversation's rows contiguous and in entry order).

Stream formats: ``process_pubsub_batch`` takes the raw Pub/Sub utterance
payloads (``{conversation_id, original_entry_index, participant_role, text, user_id,
start_timestamp_usec}``, main_service/main.py:295-302) in any order, validates them as
subscriber_service/main.py:172-190 does, redacts them in one engine call and returns the redacted
payloads the subscriber publishes (subscriber_service/main.py:213-221, ``original_text`` kept).
``TranscriptArchive`` keeps those per conversation and emits the aggregator's GCS object
``{"entries": [...]}`` ordered by ``original_entry_index`` (transcript_aggregator_service/main.py:
150-160, 220-247) directly, without the Firestore round trip.

Aggregator path (transcript_aggregator_service, README.md:131-134, 159-168): ``rescan_window_batch``
appends each row to its conversation's window of the last N utterances (N = 5,
transcript_aggregator_service/cloudbuild.yaml:33) and returns the redacted "\\n"-joined window, the
re-scan the README describes; ``conversation_ended`` drops a conversation's window (the
``/conversation-ended`` endpoint, transcript_aggregator_service/main.py).  The window lives in HBM
(pii_rescan_window); only the new utterance is scanned.
"""
from __future__ import annotations

import threading
import time
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .engine import (PII_E_ARG, PII_E_CAPACITY, PII_E_DEVICE, PII_E_NOMEM, PII_E_ORDER, PII_E_RULES,
                     ROLE_AGENT, ROLE_CUSTOMER, ROLE_OTHER, Engine, PiiError)

CONTEXT_TTL_SECONDS = 90          # main_service/main.py:163

# engine error -> the reference's fallback prefix (main.py:752-773)
ERROR_PREFIX = {
    PII_E_RULES: "[DLP_TEMPLATE_NOT_FOUND_ERROR]",      # the compiled rules (== DLP templates) are unusable
    PII_E_DEVICE: "[DLP_API_CALL_ERROR]",               # the device (== the DLP service) failed
    PII_E_NOMEM: "[DLP_PROCESSING_ERROR]",
    PII_E_CAPACITY: "[DLP_PROCESSING_ERROR]",
    PII_E_ARG: "[DLP_PROCESSING_ERROR]",
    PII_E_ORDER: "[DLP_PROCESSING_ERROR]",
}


def error_string(code: int, transcript: str) -> str:
    return f"{ERROR_PREFIX.get(code, '[DLP_PROCESSING_ERROR]')} {transcript}"


def _enc(s: str) -> bytes:
    return s.encode("utf-8", "surrogateescape")


def _dec(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


class SlotMap:
    """conversation_id -> engine context slot; slot 0 is reserved for stateless calls.  When all
    slots are taken the least recently used conversation is evicted (its context is cleared)."""

    def __init__(self, n_slots: int, on_evict: Optional[Callable[[int], None]] = None):
        if n_slots < 2:
            raise ValueError("need at least 2 slots (slot 0 is reserved)")
        self.n_slots = n_slots
        self.on_evict = on_evict
        self._map: "OrderedDict[object, int]" = OrderedDict()
        self._free = list(range(n_slots - 1, 0, -1))

    def __len__(self):
        return len(self._map)

    def get(self, conversation_id) -> int:
        s = self._map.get(conversation_id)
        if s is not None:
            self._map.move_to_end(conversation_id)
            return s
        if self._free:
            s = self._free.pop()
        else:
            _, s = self._map.popitem(last=False)
            if self.on_evict:
                self.on_evict(s)
        self._map[conversation_id] = s
        return s

    def peek(self, conversation_id) -> Optional[int]:
        return self._map.get(conversation_id)


class PiiService:
    """The main_service hot path on one engine (one GPU).  Thread-safe: calls serialize per engine,
    like the reference's single DLP client shared by gunicorn threads."""

    STATELESS_SLOT = 0

    def __init__(self, engine: Optional[Engine] = None, n_slots: int = 1 << 16,
                 ttl_seconds: int = CONTEXT_TTL_SECONDS, clock: Callable[[], float] = time.time, device: int = 0):
        self.engine = engine if engine is not None else Engine.from_rules(device=device, n_conv_slots=n_slots,
                                                                          ttl_seconds=ttl_seconds)
        self.ttl_us = int(ttl_seconds) * 1_000_000
        self.clock = clock
        self.lock = threading.Lock()
        self.slots = SlotMap(self.engine.n_slots, on_evict=self._evict)
        self.group_of_type: Dict[str, int] = {}
        for g, t in enumerate(self.engine.group_types):
            self.group_of_type.setdefault(t, g)
        self.agent_text: Dict[int, Tuple[str, int]] = {}     # slot -> (agent transcript, ts_us)

    # ---------------------------------------------------------------- helpers
    def _now_us(self) -> int:
        return int(self.clock() * 1_000_000)

    def _evict(self, slot: int):
        self.engine.context_set(slot, -1, 0)
        self.agent_text.pop(slot, None)
        if getattr(self.engine, "window_n", 0):
            self.engine.window_reset(slot)

    def _context_record(self, slot: int, now_us: int) -> Optional[dict]:
        """The Redis record of main.py:366-374 as the reference's GET returns it (None when absent
        or expired)."""
        g, ts = self.engine.context_get(slot)
        if g < 0 or now_us - ts >= self.ttl_us:        # the engine's rule: valid while now - ts < ttl
            return None
        rec = {"expected_pii_type": self.engine.group_types[g], "timestamp": ts / 1e6}
        at = self.agent_text.get(slot)
        if at is not None:
            rec["agent_transcript"] = at[0]
        return rec

    def _run(self, texts: Sequence[bytes], slots: Sequence[int], roles: Sequence[int], ts: Sequence[int]):
        return self.engine.scan_redact(texts, slots, roles, ts)

    # ---------------------------------------------------------------- reference seam (main.py:580)
    def call_dlp_for_redaction(self, transcript: str, context: Optional[dict]) -> str:
        """Redact one transcript with an optional context record ({"expected_pii_type": ...}).
        Stateless: the conversation table is not touched."""
        try:
            with self.lock:
                now = self._now_us()
                role = ROLE_OTHER
                if context and context.get("expected_pii_type") in self.group_of_type:
                    self.engine.context_set(self.STATELESS_SLOT, self.group_of_type[context["expected_pii_type"]], now)
                    role = ROLE_CUSTOMER
                res = self._run([_enc(transcript)], [self.STATELESS_SLOT], [role], [now])
                return _dec(res.text(0))
        except PiiError as e:
            return error_string(e.code, transcript)

    def extract_expected_pii(self, transcript: str) -> Optional[str]:
        """main.py:558-578 through the engine's keyword automaton (stateless)."""
        with self.lock:
            self.engine.context_set(self.STATELESS_SLOT, -1, 0)
            res = self._run([_enc(transcript)], [self.STATELESS_SLOT], [ROLE_AGENT], [self._now_us()])
            g = int(res.ctx_info[0])
            self.engine.context_set(self.STATELESS_SLOT, -1, 0)
        return self.engine.group_types[g] if g >= 0 else None

    # ---------------------------------------------------------------- handlers (main.py:344-466)
    def handle_agent_utterance(self, data: Optional[dict]) -> Tuple[dict, int]:
        if not data or "conversation_id" not in data or "transcript" not in data:
            return {"error": "Missing conversation_id or transcript"}, 400
        transcript = data["transcript"]
        try:
            with self.lock:
                slot = self.slots.get(data["conversation_id"])
                now = self._now_us()
                res = self._run([_enc(transcript)], [slot], [ROLE_AGENT], [now])
                g = int(res.ctx_info[0])
                if g >= 0:
                    self.agent_text[slot] = (transcript, now)
                return {"redacted_transcript": _dec(res.text(0)), "context_stored": g >= 0}, 200
        except PiiError as e:
            return {"redacted_transcript": error_string(e.code, transcript), "context_stored": False}, 200

    def handle_customer_utterance(self, data: Optional[dict]) -> Tuple[dict, int]:
        if not data or "conversation_id" not in data or "transcript" not in data:
            return {"error": "Missing conversation_id or transcript"}, 400
        transcript = data["transcript"]
        try:
            with self.lock:
                slot = self.slots.get(data["conversation_id"])
                now = self._now_us()
                used = self._context_record(slot, now) is not None
                res = self._run([_enc(transcript)], [slot], [ROLE_CUSTOMER], [now])
                return {"redacted_transcript": _dec(res.text(0)), "context_used": used}, 200
        except PiiError as e:
            return {"redacted_transcript": error_string(e.code, transcript), "context_used": False}, 200

    def redact_utterance_realtime(self, data: Optional[dict]) -> Tuple[dict, int]:
        if not data or "conversation_id" not in data or "utterance" not in data:
            return {"error": "Missing conversation_id or utterance"}, 400
        utterance = data["utterance"]
        with self.lock:
            slot = self.slots.peek(data["conversation_id"])
            now = self._now_us()
            rec = self._context_record(slot, now) if slot is not None else None
        if rec and "agent_transcript" in rec:
            full = self.call_dlp_for_redaction(f"{rec['agent_transcript']}\n{utterance}", rec)
            lines = full.splitlines()
            redacted = lines[-1] if lines else ""
        else:
            redacted = self.call_dlp_for_redaction(utterance, rec)
        return {"redacted_utterance": redacted}, 200

    # ---------------------------------------------------------------- aggregator re-scan (a12)
    def rescan_window_batch(self, rows: Sequence[dict], window_n: int = 5, slot_bytes: int = 8192) -> List[str]:
        """Rows as process_batch (original text) -> per row the redacted window
        "\\n".join(last window_n utterances of its conversation), re-scanned with the conversation's
        current expected_pii_type.  Agent rows update the context as handle_agent_utterance does."""
        texts, slots, roles, ts = [], [], [], []
        with self.lock:
            if getattr(self.engine, "window_n", 0) == 0:
                self.engine.window_enable(window_n, slot_bytes)
            elif self.engine.window_n != window_n:
                raise ValueError(f"window already enabled with N={self.engine.window_n}")
            for r in rows:
                texts.append(_enc(r["text"]))
                slots.append(self.slots.get(r["conversation_id"]))
                pr = str(r.get("participant_role", "")).upper()
                roles.append(ROLE_AGENT if pr == "AGENT" else ROLE_CUSTOMER if pr in ("END_USER", "CUSTOMER")
                             else ROLE_OTHER)
                ts.append(int(r.get("start_timestamp_usec", self._now_us())))
            res = self.engine.rescan_window(texts, slots, roles, ts)
            return [_dec(res.text(i)) for i in range(len(rows))]

    def conversation_ended(self, conversation_id) -> None:
        """/conversation-ended: the conversation's window and context are dropped."""
        with self.lock:
            slot = self.slots.peek(conversation_id)
            if slot is not None and getattr(self.engine, "window_n", 0):
                self.engine.window_reset(slot)

    # ---------------------------------------------------------------- batched ingest
    def process_batch(self, rows: Sequence[dict]) -> List[str]:
        """Pub/Sub-shaped rows {conversation_id, participant_role ('AGENT' | 'END_USER' | ...),
        text, start_timestamp_usec}, grouped by conversation in entry order -> redacted texts.
        Agent rows update their conversation's context exactly as handle_agent_utterance would."""
        texts, slots, roles, ts = [], [], [], []
        with self.lock:
            for r in rows:
                texts.append(_enc(r["text"]))
                slots.append(self.slots.get(r["conversation_id"]))
                pr = str(r.get("participant_role", "")).upper()
                roles.append(ROLE_AGENT if pr == "AGENT" else ROLE_CUSTOMER if pr in ("END_USER", "CUSTOMER")
                             else ROLE_OTHER)
                ts.append(int(r.get("start_timestamp_usec", self._now_us())))
            res = self._run(texts, slots, roles, ts)
            for i, r in enumerate(rows):
                if roles[i] == ROLE_AGENT and int(res.ctx_info[i]) >= 0:
                    self.agent_text[slots[i]] = (r["text"], ts[i])
            return [_dec(res.text(i)) for i in range(len(rows))]

    # ---------------------------------------------------------------- Pub/Sub stream formats (§8(f))
    REQUIRED_FIELDS = ("conversation_id", "original_entry_index", "participant_role", "text",
                       "start_timestamp_usec")

    def process_pubsub_batch(self, payloads: Sequence[dict]) -> List[dict]:
        """Raw utterance payloads -> redacted payloads (subscriber_service/main.py:213-221), in input
        order.  A payload missing a required field (subscriber_service/main.py:172-187, same field
        list and emptiness test) or with an empty role yields {"error": "Bad Request", "status": 400}
        in its place and is not sent to the engine.  Rows are grouped by conversation and ordered by
        original_entry_index before the engine call (the batch contract), so agent context reaches
        the later customer rows of the same batch exactly as the per-message handlers would."""
        out: List[Optional[dict]] = [None] * len(payloads)
        good = []
        for i, m in enumerate(payloads):
            missing = [f for f in self.REQUIRED_FIELDS
                       if m.get(f) is None or (isinstance(m.get(f), str) and not m.get(f).strip())]
            role = str(m.get("participant_role") or "").upper()
            if missing or not role:
                out[i] = {"error": "Bad Request", "status": 400, "missing_fields": missing}
                continue
            good.append(i)
        first = {}
        for i in good:
            first.setdefault(payloads[i]["conversation_id"], len(first))
        order = sorted(good, key=lambda i: (first[payloads[i]["conversation_id"]],
                                            int(payloads[i]["original_entry_index"]), i))
        rows = [dict(payloads[i], participant_role=str(payloads[i]["participant_role"]).upper()) for i in order]
        red = self.process_batch(rows) if rows else []
        for i, r, t in zip(order, rows, red):
            out[i] = {"conversation_id": r["conversation_id"],
                      "original_entry_index": r["original_entry_index"],
                      "text": t,
                      "original_text": r["text"],
                      "participant_role": r["participant_role"],
                      "user_id": r.get("user_id"),
                      "start_timestamp_usec": r["start_timestamp_usec"]}
        return out


class TranscriptArchive:
    """The aggregator's per-conversation store of redacted utterances (Firestore
    conversations/{id}/utterances, transcript_aggregator_service/main.py:150-160) and its final
    object {"entries": [...]} ordered by original_entry_index (main.py:220-247)."""

    FIELDS = ("text", "original_entry_index", "participant_role", "user_id", "start_timestamp_usec")

    def __init__(self):
        self.conv: Dict[object, Dict[int, dict]] = {}

    def add(self, redacted_payloads: Sequence[dict]) -> None:
        for p in redacted_payloads:
            if not p or "error" in p:
                continue
            e = {f: p.get(f) for f in self.FIELDS}
            if p.get("original_text"):
                e["original_text"] = p["original_text"]
            self.conv.setdefault(p["conversation_id"], {})[int(p["original_entry_index"])] = e

    def entries(self, conversation_id) -> dict:
        utts = self.conv.get(conversation_id, {})
        return {"entries": [utts[k] for k in sorted(utts)]}

    def conversation_ended(self, conversation_id) -> Optional[str]:
        """The GCS object body (json.dumps(..., indent=2), main.py:236) or None when the conversation
        has no utterances (the reference skips the upload); the conversation is dropped."""
        import json
        utts = self.conv.pop(conversation_id, None)
        if not utts:
            return None
        return json.dumps({"entries": [utts[k] for k in sorted(utts)]}, indent=2)
