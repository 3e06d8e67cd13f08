"""Config 4 ingest: a host-side stream of utterance batches through one GPU's engine, with the
host->device copy of batch i+1 and the device->host copy of batch i-1 overlapped with the scan of
batch i.

In the reference every Pub/Sub message is one HTTP request and one blocking DLP RPC
(main_service/main.py:522-562 subscriber -> :386-425 handler -> :580 call_dlp_for_redaction).  Here
the subscriber's messages are packed into batches (utterance bytes + offsets + conversation slot +
role + timestamp, as ``Engine.scan_redact`` takes them), and :class:`StreamIngest` keeps two sets of
device buffers so the three copies/compute of neighbouring batches run at the same time:

    h2d stream :  H2D(i+1)             H2D(i+2)
    compute    :  scan+redact(i)       scan+redact(i+1)
    d2h stream :  D2H(i-1)             D2H(i)

``pii_scan_redact_device_ex`` takes the batch size from the host (no device->host offset read) and
``pii_reserve`` pre-sizes the engine's work buffers, so a batch enqueues without any allocation or
synchronisation; the only host wait per batch is ``pii_sync`` (the totals the D2H copy needs).
Conversation context carries from batch to batch exactly as in one big call, since the batches run
in order on one engine.

A batch whose output does not fit the stream's output buffers (PII_E_CAPACITY: nothing committed) is
run again through the engine's own host-buffer entry point with exact capacities.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Iterable, Optional

import numpy as np

from .engine import SPAN_DTYPE, BatchResult, PiiError, PII_E_CAPACITY


@dataclass
class HostBatch:
    """One batch of the stream.  ``data``/``offsets``/... are numpy arrays or pinned torch CPU
    tensors (pinned ones are copied to the device directly; others go through pinned staging).
    ``offsets`` are relative to the batch: offsets[0] == 0, offsets[n] == len(data)."""
    data: object
    offsets: object
    slot: object
    role: object
    ts_us: object
    n: int
    n_bytes: int
    perm: Optional[np.ndarray] = None     # batch row k = source row perm[k] (from_rows(group=True))

    @classmethod
    def from_rows(cls, rows, pin: bool = False, group: bool = True) -> "HostBatch":
        """rows = [(slot, role, bytes, ts_us)] in arrival order.  The engine's batch contract wants a
        conversation's rows contiguous (include/pii_engine.h; PII_E_ORDER otherwise): with `group`
        the rows are stably grouped by conversation slot, as the subscriber would before handing a
        batch over, and `perm` maps batch rows back to arrival order."""
        perm = None
        if group and rows:
            perm = np.argsort(np.array([r[0] for r in rows], dtype=np.int64), kind="stable")
            rows = [rows[int(k)] for k in perm]
        texts = [r[2] for r in rows]
        lens = np.fromiter((len(t) for t in texts), dtype=np.int64, count=len(texts))
        offs = np.zeros(len(texts) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.frombuffer(b"".join(texts), dtype=np.uint8).copy() if texts else np.zeros(0, np.uint8)
        b = cls(data, offs, np.array([r[0] for r in rows], dtype=np.int32), np.array([r[1] for r in rows], np.uint8),
                np.array([r[3] for r in rows], dtype=np.int64), len(rows), int(offs[-1]), perm)
        return b.pinned() if pin else b

    def pinned(self) -> "HostBatch":
        import torch

        def pin(a):
            t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
            return t.pin_memory()
        return HostBatch(pin(self.data), pin(self.offsets), pin(self.slot), pin(self.role), pin(self.ts_us), self.n,
                         self.n_bytes, self.perm)

    def rows(self):
        d, o = _np(self.data), _np(self.offsets)
        s, r, t = _np(self.slot), _np(self.role), _np(self.ts_us)
        return [(int(s[i]), int(r[i]), d[int(o[i]):int(o[i + 1])].tobytes(), int(t[i])) for i in range(self.n)]


def _np(a):
    return a.numpy() if hasattr(a, "numpy") else a


class _Set:
    """one batch's device buffers + pinned output buffers"""

    def __init__(self, torch, dev, max_bytes, max_rows, out_cap, span_cap):
        e = dict(device=dev)
        self.d_text = torch.empty(max_bytes + 64, dtype=torch.uint8, **e)
        self.d_offs = torch.empty(max_rows + 1, dtype=torch.int64, **e)
        self.d_slot = torch.empty(max_rows, dtype=torch.int32, **e)
        self.d_role = torch.empty(max_rows, dtype=torch.uint8, **e)
        self.d_ts = torch.empty(max_rows, dtype=torch.int64, **e)
        self.d_out = torch.empty(out_cap + 64, dtype=torch.uint8, **e)
        self.d_oo = torch.empty(max_rows + 1, dtype=torch.int64, **e)
        self.d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, **e)
        self.d_ctx = torch.empty(max(max_rows, 1), dtype=torch.int16, **e)
        pin = dict(pin_memory=True)
        self.h_out = torch.empty(out_cap + 64, dtype=torch.uint8, **pin)
        self.h_oo = torch.empty(max_rows + 1, dtype=torch.int64, **pin)
        self.h_sp = torch.empty(span_cap * 16, dtype=torch.uint8, **pin)
        self.h_ctx = torch.empty(max(max_rows, 1), dtype=torch.int16, **pin)
        # staging for batches that are not already in pinned memory
        self.s_text = torch.empty(max_bytes + 64, dtype=torch.uint8, **pin)
        self.s_offs = torch.empty(max_rows + 1, dtype=torch.int64, **pin)
        self.s_slot = torch.empty(max_rows, dtype=torch.int32, **pin)
        self.s_role = torch.empty(max_rows, dtype=torch.uint8, **pin)
        self.s_ts = torch.empty(max_rows, dtype=torch.int64, **pin)
        self.ev_h2d = torch.cuda.Event()
        self.ev_d2h = torch.cuda.Event()


class StreamIngest:
    """Double-buffered batch stream through one engine (one GPU).  ``run`` calls
    ``consume(i, result)`` for every batch in order; ``result`` is a BatchResult whose arrays are views
    of pinned buffers, valid until ``consume`` returns (copy what must outlive it)."""

    def __init__(self, engine, max_bytes: int, max_rows: int, out_cap: Optional[int] = None,
                 span_cap: Optional[int] = None):
        import torch
        self.torch = torch
        self.eng = engine
        self.dev = torch.device("cuda", engine.device)
        self.max_bytes, self.max_rows = int(max_bytes), int(max_rows)
        self.out_cap = int(out_cap if out_cap is not None else max_bytes + 48 * max_rows)
        self.span_cap = int(span_cap if span_cap is not None else max(16, 2 * max_rows))
        self.sets = [_Set(torch, self.dev, self.max_bytes, self.max_rows, self.out_cap, self.span_cap)
                     for _ in range(2)]
        self.s_h2d = torch.cuda.Stream(self.dev)
        self.s_comp = torch.cuda.Stream(self.dev)
        self.s_d2h = torch.cuda.Stream(self.dev)
        engine.reserve(self.max_rows, self.max_bytes, self.out_cap, self.span_cap)
        self.stats = {"batches": 0, "bytes_in": 0, "bytes_out": 0, "spans": 0, "capacity_reruns": 0}

    # ------------------------------------------------------------------ stages
    def _h2d(self, S: _Set, b: HostBatch) -> None:
        torch = self.torch
        if b.n > self.max_rows or b.n_bytes > self.max_bytes:
            raise ValueError(f"batch of {b.n} rows / {b.n_bytes} bytes exceeds the stream's "
                             f"{self.max_rows} / {self.max_bytes}")
        src = []
        for a, stage in ((b.data, S.s_text), (b.offsets, S.s_offs), (b.slot, S.s_slot), (b.role, S.s_role),
                         (b.ts_us, S.s_ts)):
            if isinstance(a, torch.Tensor) and a.is_pinned():
                src.append(a)
            else:                       # stage through pinned memory (its last H2D has finished: see run)
                t = torch.from_numpy(np.ascontiguousarray(a))
                stage[:t.numel()].copy_(t.view(stage.dtype))
                src.append(stage[:t.numel()])
        with torch.cuda.stream(self.s_h2d):
            for d, s, k in ((S.d_text, src[0], b.n_bytes), (S.d_offs, src[1], b.n + 1), (S.d_slot, src[2], b.n),
                            (S.d_role, src[3], b.n), (S.d_ts, src[4], b.n)):
                if k:
                    d[:k].copy_(s[:k].view(d.dtype), non_blocking=True)
            S.ev_h2d.record(self.s_h2d)

    def _compute(self, S: _Set, b: HostBatch) -> None:
        self.s_comp.wait_event(S.ev_h2d)
        self.s_comp.wait_event(S.ev_d2h)            # the previous batch of this set has left d_out
        self.eng.scan_redact_device_ex(S.d_text.data_ptr(), S.d_offs.data_ptr(), b.n, 0, b.n_bytes,
                                       S.d_slot.data_ptr(), S.d_role.data_ptr(), S.d_ts.data_ptr(),
                                       S.d_out.data_ptr(), self.out_cap, S.d_oo.data_ptr(), S.d_sp.data_ptr(),
                                       self.span_cap, S.d_ctx.data_ptr(), self.s_comp.cuda_stream)

    def _finish(self, S: _Set, b: HostBatch):
        """wait for the set's compute; enqueue its D2H (or re-run it on a capacity miss)"""
        torch = self.torch
        try:
            ob, ns, _ = self.eng.sync()
        except PiiError as e:
            if e.code != PII_E_CAPACITY:
                raise
            self.stats["capacity_reruns"] += 1
            return self.eng.scan_redact([t for _, _, t, _ in b.rows()], _np(b.slot), _np(b.role), _np(b.ts_us))
        with torch.cuda.stream(self.s_d2h):
            S.h_oo[:b.n + 1].copy_(S.d_oo[:b.n + 1], non_blocking=True)
            if ob:
                S.h_out[:ob].copy_(S.d_out[:ob], non_blocking=True)
            if ns:
                S.h_sp[:ns * 16].copy_(S.d_sp[:ns * 16], non_blocking=True)
            if b.n:
                S.h_ctx[:b.n].copy_(S.d_ctx[:b.n], non_blocking=True)
            S.ev_d2h.record(self.s_d2h)
        return (ob, ns)

    def _deliver(self, i, S: _Set, b: HostBatch, fin, consume) -> None:
        if isinstance(fin, BatchResult):
            res = fin
            ob, ns = int(fin.out_offsets[-1]), len(fin.spans)
        else:
            ob, ns = fin
            S.ev_d2h.synchronize()
            res = BatchResult(S.h_out[:ob].numpy(), S.h_oo[:b.n + 1].numpy().view(np.uint64),
                              S.h_sp[:ns * 16].numpy().view(SPAN_DTYPE), S.h_ctx[:b.n].numpy())
        self.stats["batches"] += 1
        self.stats["bytes_in"] += b.n_bytes
        self.stats["bytes_out"] += ob
        self.stats["spans"] += ns
        if consume is not None:
            consume(i, res)

    # ------------------------------------------------------------------ driver
    def run(self, batches: Iterable[HostBatch], consume: Optional[Callable[[int, BatchResult], None]] = None) -> dict:
        """Stream `batches` through the engine in order.  H2D(0) is enqueued up front; then per batch
        i: wait for scan(i-1) (pii_sync) and enqueue D2H(i-1); enqueue scan(i) (after H2D(i), and
        after D2H(i-2) has left the same output buffers); enqueue H2D(i+1) into the buffers scan(i-1)
        has finished with; wait for D2H(i-1) and hand it to `consume`.  So H2D(i+1), scan(i) and
        D2H(i-1) are in flight together."""
        it = iter(batches)
        nxt = next(it, None)
        if nxt is not None:
            self._h2d(self.sets[0], nxt)
        prev = None                              # (index, set, batch) whose scan is in flight
        i = 0
        while nxt is not None:
            S, b = self.sets[i & 1], nxt
            fin = self._finish(prev[1], prev[2]) if prev is not None else None
            self._compute(S, b)
            nxt = next(it, None)
            if nxt is not None:
                self._h2d(self.sets[(i + 1) & 1], nxt)
            if prev is not None:
                self._deliver(prev[0], prev[1], prev[2], fin, consume)
            prev = (i, S, b)
            i += 1
        if prev is not None:
            fin = self._finish(prev[1], prev[2])
            self._deliver(prev[0], prev[1], prev[2], fin, consume)
        self.torch.cuda.synchronize(self.dev)
        return dict(self.stats)


def split_batches(meta_offsets: np.ndarray, batch_bytes: int, max_rows: Optional[int] = None):
    """[lo, hi) row ranges of at most `batch_bytes` bytes (and `max_rows` rows); a row longer than
    `batch_bytes` gets a batch of its own."""
    o = np.asarray(meta_offsets, dtype=np.int64)
    n = len(o) - 1
    out = []
    lo = 0
    while lo < n:
        hi = int(np.searchsorted(o, o[lo] + batch_bytes, side="right")) - 1
        hi = max(hi, lo + 1)
        if max_rows is not None:
            hi = min(hi, lo + max_rows)
        out.append((lo, min(hi, n)))
        lo = min(hi, n)
    return out
