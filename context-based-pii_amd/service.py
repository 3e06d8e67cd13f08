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

Conversation ids map onto engine context slots (``SlotMap``): a slot is reused only once its
conversation's record has expired (Redis TTL semantics), otherwise the engine's table grows.  The agent
transcript of the last keyword hit -- the record's ``agent_transcript`` field -- is host data (only
the realtime handler reads it) and lives beside the slot map; its expiry follows the engine's TTL.

Throughput path: ``process_batch`` runs many rows in one engine call (the batch contract of
include/pii_engine.h: a conversation's rows contiguous and in entry order), and
``process_requests`` runs a micro-batch of concurrent handler requests in one engine call with the
same results as calling the handlers one after another (``app.py`` is the Flask front end that
coalesces concurrent HTTP requests into such micro-batches).  A failed engine call (its rows get
the reference's ``[DLP_*_ERROR]`` strings) still stores the agent rows' context, as the reference
does after a failed DLP call.

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

import logging
import threading
import time
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

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


class PartialBatchError(Exception):
    """process_requests raised in a sub-batch after earlier sub-batches had committed: `done` maps
    request index -> response for every request that completed (and must not run again)."""

    def __init__(self, done: Dict[int, Tuple[dict, int]], cause: Exception):
        super().__init__(f"{type(cause).__name__}: {cause}")
        self.done = done
        self.cause = cause


class SlotMap:
    """conversation_id -> engine context slot (the Redis key ``context:{conversation_id}`` -> its HBM
    record); slot 0 is reserved for stateless calls.

    Redis keeps a key until its TTL runs out (main.py:163, 366-374), so a slot is reused only when
    nothing the reference would still read lives in it: the conversation stored no context record,
    or its record has expired (``now - ts >= ttl``, the engine's validity rule), and it has no
    window history (the aggregator keeps a conversation's utterances until it ends).  Among those,
    the least recently used conversation that is not pinned (part of the batch being built) goes
    first; its slot is cleared (``on_evict``).  When no slot can be reused the table GROWS
    (``on_grow(n)``, pii_context_resize: live records are kept), so a live context is never dropped.

    The victim search walks the whole LRU order (the table grows only when NO slot is reusable); the
    live entries it passes over move to the most-recently-used end, so the next search starts at
    entries it has not just examined and a block of long-lived (e.g. windowed, never ended)
    conversations at the LRU end costs one pass, not one per call.  (A search runs only when the
    free list is empty, and a failed one doubles it, so the cost per slot handed out stays O(1)
    amortised.)  When the table cannot grow -- the device has no memory for the doubled table
    (``on_grow`` raises PiiError NOMEM) or ``max_slots`` is reached -- the PiiError goes to the
    caller, which answers that conversation's rows with the reference's error string.  A failed
    growth is remembered: until a slot is released or ``grow_retry_s`` has passed, the table does not
    try to grow again (no repeated doubled allocation under the service lock), and within one
    ``assign`` call the new conversations after the first that got no slot fail without another walk
    (nothing in that call can free a slot)."""

    grow_retry_s = 1.0

    def __init__(self, n_slots: int, on_evict: Optional[Callable[[int], None]] = None,
                 on_grow: Optional[Callable[[int], None]] = None, max_slots: Optional[int] = None):
        if n_slots < 3:
            raise ValueError("need at least 3 slots (slot 0 is reserved)")
        self.n_slots = n_slots
        self.on_evict = on_evict
        self.on_grow = on_grow
        self.max_slots = max_slots
        self._map: "OrderedDict[object, int]" = OrderedDict()
        self._free = list(range(n_slots - 1, 0, -1))
        self.live_until: Dict[int, int] = {}      # slot -> time its context record expires (us)
        self.windowed: set = set()                 # slots holding window history
        self._grow_failed: Optional[Tuple[int, float, PiiError]] = None   # (n_slots, when, error)
        self.grow_calls = 0                        # on_grow attempts (accounting / tests)

    @property
    def capacity(self) -> int:
        return self.n_slots - 1

    def __len__(self):
        return len(self._map)

    def note_context(self, slot: int, until_us: int) -> None:
        """a context record was stored in `slot`, valid until `until_us` (ts + ttl)"""
        self.live_until[slot] = max(self.live_until.get(slot, until_us), until_us)

    def note_window(self, slot: int) -> None:
        self.windowed.add(slot)

    def reusable(self, slot: int, now_us: Optional[int]) -> bool:
        if slot in self.windowed:
            return False
        until = self.live_until.get(slot)
        return until is None or (now_us is not None and now_us >= until)

    def _forget(self, slot: int) -> None:
        self.live_until.pop(slot, None)
        self.windowed.discard(slot)

    def _victim(self, pinned: Optional[set], now_us: Optional[int]):
        """the least recently used reusable unpinned conversation, or None; the live entries passed
        over move to the MRU end"""
        victim, passed = None, []
        for c, cs in self._map.items():
            if pinned and c in pinned:
                continue
            if self.reusable(cs, now_us):
                victim = c
                break
            passed.append(c)
        for c in passed:
            self._map.move_to_end(c)
        return victim

    def get(self, conversation_id, pinned: Optional[set] = None, now_us: Optional[int] = None) -> int:
        s = self._map.get(conversation_id)
        if s is not None:
            self._map.move_to_end(conversation_id)
            return s
        if not self._free:
            victim = self._victim(pinned, now_us)
            if victim is None:
                self._grow()
            else:
                s = self._map.pop(victim)
                self._forget(s)
                if self.on_evict:
                    self.on_evict(s)
                self._map[conversation_id] = s
                return s
        s = self._free.pop()
        self._map[conversation_id] = s
        return s

    def _grow(self) -> None:
        n = self.n_slots * 2
        if self.max_slots is not None and n > self.max_slots:
            raise PiiError(PII_E_NOMEM, f"conversation table at its maximum of {self.max_slots} slots")
        f = self._grow_failed
        if f is not None and f[0] == self.n_slots and time.monotonic() - f[1] < self.grow_retry_s:
            raise f[2]                            # the same growth failed a moment ago: do not retry
        if self.on_grow:
            self.grow_calls += 1
            try:
                self.on_grow(n)                   # raises PiiError if the device cannot hold the larger table
            except PiiError as e:
                self._grow_failed = (self.n_slots, time.monotonic(), e)
                raise
        self._grow_failed = None
        self._free = list(range(n - 1, self.n_slots - 1, -1)) + self._free
        self.n_slots = n

    def assign(self, conversation_ids: Sequence, pinned: Optional[set], now_us: Optional[int]
               ) -> Tuple[List[Optional[int]], int]:
        """slots for a run of rows: None for the rows of a conversation that got no slot (the table
        could neither reuse a slot nor grow), with the PiiError code of that failure (0: none)"""
        out: List[Optional[int]] = []
        failed: Dict[object, int] = {}
        code = 0
        for cid in conversation_ids:
            if cid in failed or (code and cid not in self._map):
                # (a new conversation after a failure of this call: nothing since has freed a slot)
                failed.setdefault(cid, code)
                out.append(None)
                continue
            try:
                out.append(self.get(cid, pinned, now_us))
            except PiiError as e:
                failed[cid] = e.code
                code = e.code
                out.append(None)
        return out, code

    def peek(self, conversation_id) -> Optional[int]:
        return self._map.get(conversation_id)

    def release(self, conversation_id) -> Optional[int]:
        s = self._map.pop(conversation_id, None)
        if s is not None:
            self._forget(s)
            self._free.append(s)
            self._grow_failed = None
        return s


def role_code(participant_role) -> int:
    """subscriber_service/main.py:189,200,229: AGENT -> agent handler, END_USER / CUSTOMER ->
    customer handler; anything else is not a handler role."""
    pr = str(participant_role or "").upper()
    return ROLE_AGENT if pr == "AGENT" else ROLE_CUSTOMER if pr in ("END_USER", "CUSTOMER") else ROLE_OTHER


class PiiService:
    """The main_service hot path on one engine (one GPU).  Thread-safe: calls serialize per engine,
    like the reference's single DLP client shared by gunicorn threads.

    One time base per service (the context TTL compares two stamps of the same clock):
    ``time_base="wall"`` (the reference: every record is stamped with time.time() when the handler
    runs, main.py:370) stamps batch rows with the wall clock too; ``time_base="payload"`` (replays)
    stamps rows with their ``start_timestamp_usec`` and makes the handlers' "now" the latest payload
    time seen."""

    STATELESS_SLOT = 0

    def __init__(self, engine: Optional[Engine] = None, n_slots: int = 1 << 16,
                 ttl_seconds: int = CONTEXT_TTL_SECONDS, clock: Callable[[], float] = time.time, device: int = 0,
                 time_base: str = "wall", ner=None, ner_max_len: int = 64, max_slots: Optional[int] = None):
        if time_base not in ("wall", "payload"):
            raise ValueError("time_base must be 'wall' or 'payload'")
        self.engine = engine if engine is not None else Engine.from_rules(device=device, n_conv_slots=n_slots,
                                                                          ttl_seconds=ttl_seconds)
        self.ttl_us = int(ttl_seconds) * 1_000_000
        self.clock = clock
        self.time_base = time_base
        self._payload_now: Optional[int] = None
        self.lock = threading.Lock()
        self.slots = SlotMap(self.engine.n_slots, on_evict=self._evict, on_grow=self.engine.context_resize,
                             max_slots=max_slots)
        self.group_of_type: Dict[str, int] = {}
        for g, t in enumerate(self.engine.group_types):
            self.group_of_type.setdefault(t, g)
        self.agent_text: Dict[int, Tuple[str, int]] = {}     # slot -> (agent transcript, ts_us)
        # optional NER detector (ner.BertNer): its PERSON_NAME spans join every engine call's overlap
        # resolution as external candidates (pii_scan_redact_ext), so they are redacted like any finding
        self.ner = ner
        self.ner_max_len = ner_max_len
        if ner is not None:
            if "PERSON_NAME" not in self.engine.type_names:
                raise ValueError("the rules have no PERSON_NAME type (builtin_infotypes.yaml external_types)")
            self.ner_type = self.engine.type_names.index("PERSON_NAME")

    # ---------------------------------------------------------------- helpers
    def _now_us(self) -> int:
        if self.time_base == "payload" and self._payload_now is not None:
            return self._payload_now
        return int(self.clock() * 1_000_000)

    def _row_ts(self, r: dict, now: int) -> int:
        if self.time_base == "wall" or r.get("start_timestamp_usec") is None:
            return now
        t = int(r["start_timestamp_usec"])
        self._payload_now = t if self._payload_now is None else max(self._payload_now, t)
        return t

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
        if self.ner is None:
            return self.engine.scan_redact(texts, slots, roles, ts)
        ext = self.ner.ext_candidates(texts, self.ner_type, max_len=self.ner_max_len)
        return self.engine.scan_redact(texts, slots, roles, ts, ext=ext)

    def _sub_batches(self, keys: Sequence[object], split_before: Optional[Sequence[bool]] = None) -> List[List[int]]:
        """Row indices cut into runs at the marked rows (the slot table grows instead of evicting a
        live conversation, so a run may hold any number of conversations)."""
        out, cur = [], []
        for i in range(len(keys)):
            if cur and split_before and split_before[i]:
                out.append(cur)
                cur = []
            cur.append(i)
        if cur:
            out.append(cur)
        return out

    def _note(self, slots, roles, texts, ts, ctx_info) -> None:
        """After an engine call (or its context-only fallback): AGENT rows whose keyword hit stored a
        context record -- the Redis SETEX of main.py:366-374, with the record's agent_transcript."""
        for k, (sl, r) in enumerate(zip(slots, roles)):
            if r == ROLE_AGENT and int(ctx_info[k]) >= 0:
                self.agent_text[sl] = (texts[k], ts[k])
                self.slots.note_context(sl, ts[k] + self.ttl_us)

    def _context_fallback(self, texts: Sequence[bytes], slots, roles, ts) -> np.ndarray:
        """After a failed engine call: the context half alone (pii_context_update), so AGENT rows
        still store their context, as the reference's extract_expected_pii + SETEX run after a
        failed DLP call (call_dlp_for_redaction never raises, main.py:358-374).  A batch too big for
        the engine's memory is halved until the parts fit (in row order: a conversation's context
        flows from one part into the next).  ctx_info per row, -2 where the device could not run it."""
        n = len(texts)
        try:
            return np.asarray(self.engine.context_update(texts, slots, roles, ts), dtype=np.int16)
        except PiiError as e:
            if e.code != PII_E_NOMEM or n <= 1:
                return np.full(n, -2, np.int16)
        h = n // 2
        return np.concatenate([self._context_fallback(texts[:h], slots[:h], roles[:h], ts[:h]),
                               self._context_fallback(texts[h:], slots[h:], roles[h:], ts[h:])])

    def _without_slots(self, part, slots, code, texts, ts, call, window=False) -> List[str]:
        """A run some of whose conversations got no slot (SlotMap.assign): those rows get the
        reference's error string and store nothing; the other rows run as usual (dropping whole
        conversations keeps the batch contract).  Called with the service lock held."""
        keep = [k for k, sl in enumerate(slots) if sl is not None]
        red: Dict[int, str] = {k: error_string(code, part[k]["text"]) for k in range(len(part)) if slots[k] is None}
        if keep:
            k_texts = [texts[k] for k in keep]
            k_slots = [slots[k] for k in keep]
            k_roles = [role_code(part[k].get("participant_role")) for k in keep]
            k_ts = [ts[k] for k in keep]
            try:
                res = call(k_texts, k_slots, k_roles, k_ts)
            except PiiError as e:
                self._note(k_slots, k_roles, [part[k]["text"] for k in keep], k_ts,
                           self._context_fallback(k_texts, k_slots, k_roles, k_ts))
                red.update({k: error_string(e.code, part[k]["text"]) for k in keep})
            else:
                if window:
                    for sl in k_slots:
                        self.slots.note_window(sl)
                self._note(k_slots, k_roles, [part[k]["text"] for k in keep], k_ts, res.ctx_info)
                red.update({k: _dec(res.text(j)) for j, k in enumerate(keep)})
        return [red[k] for k in range(len(part))]

    # ---------------------------------------------------------------- reference seam (main.py:580)
    def call_dlp_for_redaction(self, transcript: str, context: Optional[dict]) -> str:
        """Redact one transcript with an optional context record ({"expected_pii_type": ...}).
        Stateless: the conversation table is not touched.  Any expected_pii_type the engine has a
        type for selects its compiled variant (main.py:614-686); a name the engine has no detector
        for changes nothing the engine reports (the reference would add an info type and a rule set
        for it, both of which only affect findings of that type)."""
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
        return self.process_requests([("agent", data)])[0]

    def handle_customer_utterance(self, data: Optional[dict]) -> Tuple[dict, int]:
        return self.process_requests([("customer", data)])[0]

    def redact_utterance_realtime(self, data: Optional[dict]) -> Tuple[dict, int]:
        return self.process_requests([("realtime", data)])[0]

    REQUEST_KEYS = {"agent": "transcript", "customer": "transcript", "realtime": "utterance"}

    @classmethod
    def request_error(cls, kind: str, data) -> Optional[Tuple[dict, int]]:
        """The response a request gets on its own, before any engine call, or None when it is
        well-formed.  A body without the two keys is the reference's 400 (main.py:351-352,
        393-394, 434-435).  A body the reference's handler would crash on after that check -- a
        JSON string (``data['conversation_id']`` on a str), a non-string text (``.lower()`` in
        extract_expected_pii, the f-string join of main.py:457) or an unhashable id (the Redis key
        is built from it, here the slot map) -- is that request's own 500, never its batch's."""
        key = cls.REQUEST_KEYS[kind]
        missing = ({"error": f"Missing conversation_id or {key}"}, 400)
        if not data:
            return missing
        if not isinstance(data, (dict, list, str)):           # `key in 5` raises in the reference
            return ({"error": "Internal Server Error"}, 500)
        if "conversation_id" not in data or key not in data:
            return missing
        if not isinstance(data, dict) or not isinstance(data[key], str):
            return ({"error": "Internal Server Error"}, 500)
        try:
            hash(data["conversation_id"])
        except TypeError:
            return ({"error": "Internal Server Error"}, 500)
        return None

    def process_requests(self, reqs: Sequence[Tuple[str, Optional[dict]]]) -> List[Tuple[dict, int]]:
        """A micro-batch of handler requests [(kind, json body)] in arrival order, kind in
        {"agent", "customer", "realtime"} (/handle-agent-utterance, /handle-customer-utterance,
        /redact-utterance-realtime) -> [(response json, status)], in ONE engine call where possible.

        Equivalent to calling the handlers one by one in arrival order: a conversation's requests
        stay in arrival order (the engine's row order), conversations are independent.  A realtime
        request reads the host-side agent transcript, which an AGENT row of its conversation earlier
        in the same engine call would only update after the call, so such a request starts a new
        engine call."""
        out: List[Optional[Tuple[dict, int]]] = [None] * len(reqs)
        valid = []
        for i, (kind, data) in enumerate(reqs):
            err = self.request_error(kind, data)
            if err is not None:
                out[i] = err
            else:
                valid.append(i)
        split, agents = [], set()
        for i in valid:
            kind, data = reqs[i]
            cid = data["conversation_id"]
            cut = kind == "realtime" and cid in agents
            if cut:
                agents = set()
            split.append(cut)
            if kind == "agent":
                agents.add(cid)
        committed = False
        for run in self._sub_batches([reqs[i][1]["conversation_id"] for i in valid], split):
            idx = [valid[j] for j in run]
            try:
                self._run_requests(reqs, idx, out)
            except Exception as e:
                if not committed:
                    raise
                # earlier sub-batches are committed (their context is stored): report them, so a
                # caller re-runs only the requests that did not complete
                failed = set(idx)
                done = {i: r for i, r in enumerate(out) if r is not None and i not in failed}
                raise PartialBatchError(done, e) from e
            committed = True
        return out

    def _run_requests(self, reqs, idxs: List[int], out) -> None:
        with self.lock:
            now = self._now_us()
            pinned = {reqs[i][1]["conversation_id"] for i in idxs}
            rows = []                     # (slot, request index, text, role, realtime split)
            for i in idxs:
                kind, data = reqs[i]
                cid = data["conversation_id"]
                if kind == "realtime":
                    slot = self.slots.peek(cid)
                    rec = self._context_record(slot, now) if slot is not None else None
                    utt = data["utterance"]
                    if rec is None:                             # main.py:464 with no context
                        rows.append((self.STATELESS_SLOT, i, utt, ROLE_OTHER, False))
                    elif "agent_transcript" in rec:             # main.py:457-461
                        rows.append((slot, i, f"{rec['agent_transcript']}\n{utt}", ROLE_CUSTOMER, True))
                    else:
                        rows.append((slot, i, utt, ROLE_CUSTOMER, False))
                else:
                    try:
                        slot = self.slots.get(cid, pinned, now)
                    except PiiError as e:
                        # no slot for the conversation (the table could neither reuse one nor grow):
                        # the request is answered as after a failed DLP call, nothing is stored
                        key = "context_stored" if kind == "agent" else "context_used"
                        out[i] = ({"redacted_transcript": error_string(e.code, data["transcript"]), key: False}, 200)
                        continue
                    rows.append((slot, i, data["transcript"], ROLE_AGENT if kind == "agent" else ROLE_CUSTOMER, False))
            if not rows:
                return
            # the batch contract: a slot's rows contiguous, in arrival order
            first: Dict[int, int] = {}
            for k, r in enumerate(rows):
                first.setdefault(r[0], k)
            order = sorted(range(len(rows)), key=lambda k: (first[rows[k][0]], k))
            rows = [rows[k] for k in order]
            texts = [_enc(r[2]) for r in rows]
            slots, roles, ts = [r[0] for r in rows], [r[3] for r in rows], [now] * len(rows)
            try:
                res = self._run(texts, slots, roles, ts)
            except PiiError as e:
                # The reference's handlers never fail on a DLP error: the error string is the transcript
                # (main.py:752-773), the agent handler still extracts and stores the context
                # (main.py:358-374) and context_used reports the Redis GET (main.py:425).  The engine
                # call is atomic (nothing committed), so its context half runs again alone.
                ctx = self._context_fallback(texts, slots, roles, ts)
                self._note(slots, roles, [r[2] for r in rows], ts, ctx)
                for k, (slot, i, text, role, split_last) in enumerate(rows):
                    kind, data = reqs[i]
                    g = int(ctx[k])
                    if kind == "agent":
                        out[i] = ({"redacted_transcript": error_string(e.code, text), "context_stored": g >= 0}, 200)
                    elif kind == "customer":
                        used = g >= 0
                        if g == -2:
                            try:
                                used = self._context_record(slot, now) is not None
                            except PiiError:
                                used = False
                        out[i] = ({"redacted_transcript": error_string(e.code, text), "context_used": used}, 200)
                    else:                                   # main.py:458-461 on the error string
                        red = error_string(e.code, text)
                        lines = red.splitlines() if split_last else [red]
                        out[i] = ({"redacted_utterance": lines[-1] if lines else ""}, 200)
                return
            # The engine call has committed (context stored on the device): from here on every request
            # of the call is answered, so a caller never re-runs it (a re-run would store its context
            # twice).  A failure while building a response is that request's own 500, as an exception
            # raised after the SETEX in the reference's handler would be.
            try:
                self._note(slots, roles, [r[2] for r in rows], ts, res.ctx_info)
            except Exception:                           # noqa: BLE001 - the call stays answered
                # the device may hold a record for any AGENT slot of the call: mark them all live, so
                # the slot map never reuses a slot whose context the reference would still read
                for sl, r, t_ in zip(slots, roles, ts):
                    if r == ROLE_AGENT:
                        self.slots.note_context(sl, t_ + self.ttl_us)
                logging.getLogger(__name__).exception("host context bookkeeping failed after a committed call")
            for k, (slot, i, text, role, split_last) in enumerate(rows):
                kind, data = reqs[i]
                try:
                    red = _dec(res.text(k))
                    g = int(res.ctx_info[k])
                    if kind == "agent":
                        out[i] = ({"redacted_transcript": red, "context_stored": g >= 0}, 200)
                    elif kind == "customer":
                        out[i] = ({"redacted_transcript": red, "context_used": g >= 0}, 200)
                    else:
                        if split_last:
                            lines = red.splitlines()
                            red = lines[-1] if lines else ""
                        out[i] = ({"redacted_utterance": red}, 200)
                except Exception:                       # noqa: BLE001 - answered, never re-run
                    out[i] = ({"error": "Internal Server Error"}, 500)

    # ---------------------------------------------------------------- aggregator re-scan (a12)
    def rescan_window_batch(self, rows: Sequence[dict], window_n: int = 5, slot_bytes: int = 8192) -> List[str]:
        """Rows as process_batch (original text) -> per row the redacted window
        "\\n".join(last window_n utterances of its conversation), re-scanned with the conversation's
        current expected_pii_type.  Agent rows update the context as handle_agent_utterance does."""
        with self.lock:
            if getattr(self.engine, "window_n", 0) == 0:
                self.engine.window_enable(window_n, slot_bytes)
            elif self.engine.window_n != window_n:
                raise ValueError(f"window already enabled with N={self.engine.window_n}")
        out: List[str] = []
        for run in self._sub_batches([r["conversation_id"] for r in rows]):
            with self.lock:
                now = self._now_us()
                part = [rows[i] for i in run]
                pinned = {r["conversation_id"] for r in part}
                texts = [_enc(r["text"]) for r in part]
                ts = [self._row_ts(r, now) for r in part]
                now = self._now_us()
                slots, code = self.slots.assign([r["conversation_id"] for r in part], pinned, now)
                if code:
                    out.extend(self._without_slots(part, slots, code, texts, ts, self.engine.rescan_window,
                                                   window=True))
                    continue
                roles = [role_code(r.get("participant_role")) for r in part]
                try:
                    res = self.engine.rescan_window(texts, slots, roles, ts)
                except PiiError as e:
                    # the context is stored regardless (main.py:358-374); the rows do not enter the windows
                    self._note(slots, roles, [r["text"] for r in part], ts,
                               self._context_fallback(texts, slots, roles, ts))
                    out.extend(error_string(e.code, r["text"]) for r in part)
                    continue
                for sl in slots:
                    self.slots.note_window(sl)
                self._note(slots, roles, [r["text"] for r in part], ts, res.ctx_info)
                out.extend(_dec(res.text(i)) for i in range(len(part)))
        return out

    def conversation_ended(self, conversation_id) -> None:
        """/conversation-ended: the conversation's window, its context record (Redis
        context:{id}) and its host-side agent transcript are dropped and its slot is freed."""
        with self.lock:
            slot = self.slots.release(conversation_id)
            if slot is not None:
                self._evict(slot)

    # ---------------------------------------------------------------- batched ingest
    def process_batch(self, rows: Sequence[dict]) -> List[str]:
        """Pub/Sub-shaped rows {conversation_id, participant_role ('AGENT' | 'END_USER' | ...),
        text, start_timestamp_usec}, grouped by conversation in entry order -> redacted texts.
        Agent rows update their conversation's context exactly as handle_agent_utterance would;
        other roles are redacted without context.  Never raises for engine errors: a failed
        engine call yields the reference's error strings for its rows (main.py:752-773)."""
        out: List[str] = []
        for run in self._sub_batches([r["conversation_id"] for r in rows]):
            with self.lock:
                now = self._now_us()
                part = [rows[i] for i in run]
                pinned = {r["conversation_id"] for r in part}
                texts = [_enc(r["text"]) for r in part]
                ts = [self._row_ts(r, now) for r in part]
                now = self._now_us()
                slots, code = self.slots.assign([r["conversation_id"] for r in part], pinned, now)
                if code:
                    out.extend(self._without_slots(part, slots, code, texts, ts, self._run))
                    continue
                roles = [role_code(r.get("participant_role")) for r in part]
                try:
                    res = self._run(texts, slots, roles, ts)
                except PiiError as e:
                    # the agent rows' context is stored regardless (main.py:358-374)
                    self._note(slots, roles, [r["text"] for r in part], ts,
                               self._context_fallback(texts, slots, roles, ts))
                    out.extend(error_string(e.code, r["text"]) for r in part)
                    continue
                self._note(slots, roles, [r["text"] for r in part], ts, res.ctx_info)
                out.extend(_dec(res.text(i)) for i in range(len(part)))
        return out

    # ---------------------------------------------------------------- Pub/Sub stream formats (§8(f))
    REQUIRED_FIELDS = ("conversation_id", "original_entry_index", "participant_role", "text",
                       "start_timestamp_usec")

    def process_pubsub_batch(self, payloads: Sequence[dict]) -> List[dict]:
        """Raw utterance payloads -> redacted payloads (subscriber_service/main.py:213-221), in input
        order.  A payload missing a required field (subscriber_service/main.py:172-187, same field
        list and emptiness test) or with an empty role yields {"error": "Bad Request", "status": 400}
        in its place and is not sent to the engine.  A role other than AGENT / END_USER / CUSTOMER
        is logged and skipped by the reference (subscriber_service/main.py:265-266: nothing is
        published, the push is acknowledged with 200); it yields {"status": 200, "skipped": ...}
        here and is not sent to the engine either.  Rows are grouped by conversation and ordered by
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
            if role_code(role) == ROLE_OTHER:
                out[i] = {"status": 200, "skipped": f"Unknown participant_role: '{role}'",
                          "conversation_id": m["conversation_id"], "original_entry_index": m["original_entry_index"]}
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
            if not p or "error" in p or "skipped" in p:
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
