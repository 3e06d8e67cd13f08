"""ctypes binding of libpii.so (include/pii_engine.h) - the engine behind the reference's
``call_dlp_for_redaction`` seam (main_service/main.py:580).

The product path has NO CPU fallback: if libpii.so is missing or the GPU is unusable, constructing
an :class:`Engine` raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PII_LIB") or os.path.join(HERE, "libpii.so")   # PII_LIB: kernel experiments

PII_OK, PII_E_ARG, PII_E_RULES, PII_E_DEVICE, PII_E_CAPACITY, PII_E_ORDER, PII_E_NOMEM = 0, -1, -2, -3, -4, -5, -6
ROLE_CUSTOMER, ROLE_AGENT, ROLE_OTHER = 0, 1, 2
ERROR_NAMES = {PII_E_ARG: "PII_E_ARG", PII_E_RULES: "PII_E_RULES", PII_E_DEVICE: "PII_E_DEVICE",
               PII_E_CAPACITY: "PII_E_CAPACITY", PII_E_ORDER: "PII_E_ORDER", PII_E_NOMEM: "PII_E_NOMEM"}
EXPORTS = ["pii_engine_create", "pii_engine_destroy", "pii_engine_info", "pii_type_name", "pii_context_group_type",
           "pii_last_error", "pii_scan_redact", "pii_scan_redact_device", "pii_scan_redact_device_ex",
           "pii_reserve", "pii_sync", "pii_context_get",
           "pii_context_set", "pii_histogram", "pii_histogram_reset", "pii_last_timings",
           "pii_last_timings_ex", "pii_last_queue_sizes", "pii_last_stats", "pii_window_enable", "pii_window_reset",
           "pii_window_count", "pii_rescan_window", "pii_rescan_window_device",
           "pii_rescan_window_device_ex", "pii_scan_redact_ext", "pii_scan_redact_device_ext", "pii_window_enable_ex",
           "pii_window_mode", "pii_set_scratch_limit", "pii_scratch_bytes", "pii_context_resize",
           "pii_context_update", "pii_set_timing"]
PII_WINDOW_FULL = 1


class PiiError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class pii_span(ctypes.Structure):
    _fields_ = [("utt", ctypes.c_uint32), ("start", ctypes.c_uint32), ("end", ctypes.c_uint32),
                ("info_type", ctypes.c_uint16), ("likelihood", ctypes.c_uint8), ("flags", ctypes.c_uint8)]


SPAN_DTYPE = np.dtype([("utt", "<u4"), ("start", "<u4"), ("end", "<u4"), ("info_type", "<u2"),
                       ("likelihood", "u1"), ("flags", "u1")])
assert SPAN_DTYPE.itemsize == ctypes.sizeof(pii_span) == 16


class pii_info(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("n_types", "n_patterns", "n_context_groups", "n_conv_slots",
                                               "scan_states_d", "scan_states_k", "scan_lds_bytes", "reserved")]


_LIB = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run __graft_entry__.build() (no CPU fallback exists)")
    try:
        # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's): load it first so the
        # process has ONE HIP runtime that both torch tensors and libpii.so use
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        pass
    lib = ctypes.CDLL(path)
    P, U8, U16, U32, U64, I16, I32, I64 = (ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8),
                                          ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int16),
                                          ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64))
    c = ctypes
    lib.pii_engine_create.argtypes = [c.c_void_p, c.c_size_t, c.c_int, c.c_uint32, c.c_int64, c.POINTER(c.c_void_p)]
    lib.pii_engine_destroy.argtypes = [P]
    lib.pii_engine_info.argtypes = [P, c.POINTER(pii_info)]
    lib.pii_type_name.argtypes = [P, c.c_uint32, c.c_char_p, c.c_size_t]
    lib.pii_context_group_type.argtypes = [P, c.c_uint32]
    lib.pii_last_error.argtypes = [P]
    lib.pii_last_error.restype = c.c_char_p
    lib.pii_scan_redact.argtypes = [P, P, P, c.c_uint32, P, P, P, P, c.c_uint64, P, P, c.c_uint32,
                                    c.POINTER(c.c_uint32), P]
    lib.pii_scan_redact_device.argtypes = [P, P, P, c.c_uint32, P, P, P, P, c.c_uint64, P, P, c.c_uint32, P, P]
    lib.pii_scan_redact_device_ex.argtypes = [P, P, P, c.c_uint32, c.c_uint64, c.c_uint64, P, P, P, P, c.c_uint64,
                                              P, P, c.c_uint32, P, P]
    lib.pii_scan_redact_ext.argtypes = lib.pii_scan_redact.argtypes + [P, P, c.c_uint32]
    lib.pii_scan_redact_device_ext.argtypes = lib.pii_scan_redact_device_ex.argtypes[:-1] + [P, P, c.c_uint32, P]
    lib.pii_reserve.argtypes = [P, c.c_uint32, c.c_uint64, c.c_uint64, c.c_uint32]
    lib.pii_sync.argtypes = [P, U64]
    lib.pii_context_get.argtypes = [P, c.c_uint32, I32, I64]
    lib.pii_context_set.argtypes = [P, c.c_uint32, c.c_int32, c.c_int64]
    lib.pii_context_resize.argtypes = [P, c.c_uint32]
    lib.pii_context_update.argtypes = [P, P, P, c.c_uint32, P, P, P, P]
    lib.pii_histogram.argtypes = [P, U64, c.c_uint32]
    lib.pii_histogram_reset.argtypes = [P]
    lib.pii_set_timing.argtypes = [P, c.c_int]
    lib.pii_last_timings.argtypes = [P, c.POINTER(c.c_float)]
    lib.pii_last_timings_ex.argtypes = [P, c.POINTER(c.c_float), c.c_uint32]
    lib.pii_last_queue_sizes.argtypes = [P, U64, U64]
    lib.pii_last_stats.argtypes = [P, U64, c.c_uint32]
    lib.pii_window_enable.argtypes = [P, c.c_uint32, c.c_uint32]
    lib.pii_window_enable_ex.argtypes = [P, c.c_uint32, c.c_uint32, c.c_uint32]
    lib.pii_window_mode.argtypes = [P]
    lib.pii_set_scratch_limit.argtypes = [P, c.c_uint64]
    lib.pii_scratch_bytes.argtypes = [P, U64]
    lib.pii_window_reset.argtypes = [P, c.c_uint32]
    lib.pii_window_count.argtypes = [P, c.c_uint32, U32]
    lib.pii_rescan_window.argtypes = lib.pii_scan_redact.argtypes
    lib.pii_rescan_window_device.argtypes = lib.pii_scan_redact_device.argtypes
    lib.pii_rescan_window_device_ex.argtypes = lib.pii_scan_redact_device_ex.argtypes
    for name in EXPORTS:
        if name != "pii_last_error":
            getattr(lib, name).restype = c.c_int
    _LIB = lib
    return lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pack(texts: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    lens = np.fromiter((len(t) for t in texts), dtype=np.uint64, count=len(texts))
    offs = np.zeros(len(texts) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(texts), dtype=np.uint8) if len(texts) else np.zeros(0, np.uint8)
    return data, offs


def ext_arrays(ext: Sequence[Sequence[tuple]], n: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Per-row candidate lists [(start, end, info_type, likelihood)] -> (pii_span rows padded to one
    stride, counts uint32[n], stride), the layout of pii_scan_redact_ext."""
    if len(ext) != n:
        raise ValueError("one external candidate list per row")
    stride = max(1, max((len(x) for x in ext), default=0))
    spans = np.zeros(n * stride, dtype=SPAN_DTYPE)
    counts = np.zeros(max(1, n), dtype=np.uint32)
    for i, xs in enumerate(ext):
        counts[i] = len(xs)
        for k, (s, e, t, lik) in enumerate(xs):
            spans[i * stride + k] = (i, s, e, t, lik, 0)
    return spans, counts, stride


@dataclass
class BatchResult:
    out: np.ndarray           # uint8 packed redacted rows
    out_offsets: np.ndarray   # uint64 [n+1]
    spans: np.ndarray         # SPAN_DTYPE
    ctx_info: np.ndarray      # int16 [n]

    def text(self, i: int) -> bytes:
        return self.out[int(self.out_offsets[i]):int(self.out_offsets[i + 1])].tobytes()


class Engine:
    """One engine per GPU (the drop-in for one DLP client)."""

    def __init__(self, blob: bytes, device: int = 0, n_conv_slots: int = 1 << 16, ttl_seconds: int = 90):
        self.lib = load_library()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(blob, len(blob))
        rc = self.lib.pii_engine_create(buf, len(blob), device, n_conv_slots, int(ttl_seconds) * 1_000_000,
                                        ctypes.byref(h))
        if rc != PII_OK:
            raise PiiError(rc, "pii_engine_create failed")
        self.h = h
        self.device = device
        info = pii_info()
        self.lib.pii_engine_info(self.h, ctypes.byref(info))
        self.info = info
        self.n_slots = n_conv_slots
        self.window_n = 0
        self.type_names = [self._name(t) for t in range(info.n_types)]
        self.group_types = [self.type_names[self.lib.pii_context_group_type(self.h, g)]
                            for g in range(info.n_context_groups)]

    @classmethod
    def from_rules(cls, dlp_config_path: Optional[str] = None, **kw) -> "Engine":
        import importlib
        compiler = importlib.import_module(__package__ + ".compiler") if __package__ else __import__("compiler")
        comp = compiler.compile_default(dlp_config_path)
        return cls(comp.blob, **kw)

    def _name(self, t: int) -> str:
        buf = ctypes.create_string_buffer(128)
        self.lib.pii_type_name(self.h, t, buf, 128)
        return buf.value.decode()

    def close(self):
        if getattr(self, "h", None):
            self.lib.pii_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc, what):
        msg = self.lib.pii_last_error(self.h)
        return PiiError(rc, f"{what}: {msg.decode() if msg else ''}")

    # ------------------------------------------------------------------ host-buffer batch API
    def scan_redact(self, texts: Sequence[bytes], conv_slot: Sequence[int], role: Sequence[int],
                    ts_us: Optional[Sequence[int]] = None, ext: Optional[Sequence[Sequence[tuple]]] = None
                    ) -> BatchResult:
        """ext[i]: row i's external-detector candidates [(start, end, info_type, likelihood)], sorted by
        start (pii_scan_redact_ext: they join overlap resolution with the rule findings)."""
        if ext is None:
            return self._host_call(self.lib.pii_scan_redact, "pii_scan_redact", texts, conv_slot, role, ts_us, 1)
        spans, counts, stride = ext_arrays(ext, len(texts))
        fn = lambda *a: self.lib.pii_scan_redact_ext(*a, _ptr(spans), _ptr(counts), stride)   # noqa: E731
        return self._host_call(fn, "pii_scan_redact_ext", texts, conv_slot, role, ts_us, 1)

    def rescan_window(self, texts: Sequence[bytes], conv_slot: Sequence[int], role: Sequence[int],
                      ts_us: Optional[Sequence[int]] = None) -> BatchResult:
        """Window re-scan (a12): row i's result = its conversation's redacted "\\n".join(last N
        utterances ending at row i); spans are window offsets; ctx_info = the window's context group."""
        n = max(1, self.window_n)
        return self._host_call(self.lib.pii_rescan_window, "pii_rescan_window", texts, conv_slot, role, ts_us, n)

    def window_enable(self, window_n: int = 5, slot_bytes: int = 8192, full: bool = False) -> None:
        """full=True forces the full re-scan of the joined windows (rule sets the incremental path
        cannot take get it anyway: window_mode() tells which one runs)"""
        rc = self.lib.pii_window_enable_ex(self.h, window_n, slot_bytes, PII_WINDOW_FULL if full else 0)
        if rc != PII_OK:
            raise self._err(rc, "pii_window_enable_ex")
        self.window_n = window_n

    def window_mode(self) -> str:
        rc = self.lib.pii_window_mode(self.h)
        if rc < 0:
            raise self._err(rc, "pii_window_mode")
        return "full" if rc == PII_WINDOW_FULL else "incremental"

    def window_reset(self, slot: int) -> None:
        rc = self.lib.pii_window_reset(self.h, slot)
        if rc != PII_OK:
            raise self._err(rc, "pii_window_reset")

    def window_count(self, slot: int) -> int:
        n = ctypes.c_uint32()
        rc = self.lib.pii_window_count(self.h, slot, ctypes.byref(n))
        if rc != PII_OK:
            raise self._err(rc, "pii_window_count")
        return int(n.value)

    def rescan_window_device(self, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out, out_cap, d_out_offsets,
                             d_spans, span_cap, d_ctx=None, stream=None) -> None:
        rc = self.lib.pii_rescan_window_device(self.h, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out,
                                               out_cap, d_out_offsets, d_spans, span_cap, d_ctx, stream)
        if rc != PII_OK:
            raise self._err(rc, "pii_rescan_window_device")

    def rescan_window_device_ex(self, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot, d_role, d_ts,
                                d_out, out_cap, d_out_offsets, d_spans, span_cap, d_ctx=None, stream=None) -> None:
        """rescan_window_device with offsets[0] and the batch size stated by the caller (no device-to-host
        read before the launch; pii_rescan_window_device_ex)"""
        rc = self.lib.pii_rescan_window_device_ex(self.h, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot,
                                                  d_role, d_ts, d_out, out_cap, d_out_offsets, d_spans, span_cap,
                                                  d_ctx, stream)
        if rc != PII_OK:
            raise self._err(rc, "pii_rescan_window_device_ex")

    def _host_call(self, fn, name, texts, conv_slot, role, ts_us, mult) -> BatchResult:
        data, offs = pack(texts)
        n = len(texts)
        slot = np.ascontiguousarray(conv_slot, dtype=np.uint32)
        rl = np.ascontiguousarray(role, dtype=np.uint8)
        ts = None if ts_us is None else np.ascontiguousarray(ts_us, dtype=np.int64)
        out_cap = mult * (int(offs[-1]) + 48 * max(1, n)) + 64
        span_cap = max(16, mult * (int(offs[-1]) // 3 + n))
        for _ in range(2):
            out = np.empty(out_cap, dtype=np.uint8)
            out_offs = np.zeros(n + 1, dtype=np.uint64)
            spans = np.empty(span_cap, dtype=SPAN_DTYPE)
            ns = ctypes.c_uint32(0)
            ctx = np.empty(n, dtype=np.int16)
            rc = fn(self.h, _ptr(data) if len(data) else None, _ptr(offs), n, _ptr(slot), _ptr(rl), _ptr(ts),
                    _ptr(out), out_cap, _ptr(out_offs), _ptr(spans), span_cap, ctypes.byref(ns), _ptr(ctx))
            if rc == PII_E_CAPACITY:
                out_cap = int(out_offs[-1]) + 64
                span_cap = int(ns.value) + 16
                continue
            if rc != PII_OK:
                raise self._err(rc, name)
            return BatchResult(out[:int(out_offs[-1])], out_offs, spans[:ns.value].copy(), ctx)
        raise self._err(PII_E_CAPACITY, name)

    # ------------------------------------------------------------------ device-buffer API (torch)
    def scan_redact_device(self, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out, out_cap, d_out_offsets,
                           d_spans, span_cap, d_ctx=None, stream=None) -> None:
        """All arguments are device pointers (ints, e.g. tensor.data_ptr()); asynchronous."""
        rc = self.lib.pii_scan_redact_device(self.h, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out,
                                             out_cap, d_out_offsets, d_spans, span_cap, d_ctx, stream)
        if rc != PII_OK:
            raise self._err(rc, "pii_scan_redact_device")

    def scan_redact_device_ex(self, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot, d_role, d_ts, d_out,
                              out_cap, d_out_offsets, d_spans, span_cap, d_ctx=None, stream=None) -> None:
        """scan_redact_device with offsets[0] and the batch size stated by the caller: enqueues without
        any device-to-host read (pii_scan_redact_device_ex)."""
        rc = self.lib.pii_scan_redact_device_ex(self.h, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot,
                                                d_role, d_ts, d_out, out_cap, d_out_offsets, d_spans, span_cap, d_ctx,
                                                stream)
        if rc != PII_OK:
            raise self._err(rc, "pii_scan_redact_device_ex")

    def scan_redact_device_ext(self, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot, d_role, d_ts, d_out,
                               out_cap, d_out_offsets, d_spans, span_cap, d_ctx, d_ext, d_ext_n, ext_stride,
                               stream=None) -> None:
        """scan_redact_device_ex plus external candidates in device memory (pii_scan_redact_device_ext):
        d_ext[row * ext_stride + k] for k < d_ext_n[row]."""
        rc = self.lib.pii_scan_redact_device_ext(self.h, d_bytes, d_offsets, n_utt, batch_base, batch_bytes, d_slot,
                                                 d_role, d_ts, d_out, out_cap, d_out_offsets, d_spans, span_cap, d_ctx,
                                                 d_ext, d_ext_n, ext_stride, stream)
        if rc != PII_OK:
            raise self._err(rc, "pii_scan_redact_device_ext")

    def reserve(self, max_utt: int, max_bytes: int, max_out: int, max_spans: int) -> None:
        """pre-size the work buffers so calls within these bounds allocate nothing (pii_reserve)"""
        rc = self.lib.pii_reserve(self.h, max_utt, max_bytes, max_out, max_spans)
        if rc != PII_OK:
            raise self._err(rc, "pii_reserve")

    def set_scratch_limit(self, n_bytes: int) -> None:
        """bound the work buffers' device memory (0 = none): calls that need more fail with PII_E_NOMEM"""
        rc = self.lib.pii_set_scratch_limit(self.h, int(n_bytes))
        if rc != PII_OK:
            raise self._err(rc, "pii_set_scratch_limit")

    def scratch_bytes(self) -> int:
        v = ctypes.c_uint64()
        rc = self.lib.pii_scratch_bytes(self.h, ctypes.byref(v))
        if rc != PII_OK:
            raise self._err(rc, "pii_scratch_bytes")
        return int(v.value)

    def sync(self) -> Tuple[int, int, int]:
        tot = (ctypes.c_uint64 * 3)()
        rc = self.lib.pii_sync(self.h, tot)
        if rc != PII_OK:
            raise self._err(rc, "pii_sync")
        return int(tot[0]), int(tot[1]), int(tot[2])

    def set_timing(self, level: int) -> None:
        """HIP events a call records: 0 completion only, 1 (default) + start and the roofline kernels,
        2 + the stage boundaries (pii_set_timing; each event costs the stream a few microseconds)."""
        rc = self.lib.pii_set_timing(self.h, int(level))
        if rc:
            raise self._err(rc, "pii_set_timing")

    def timings(self) -> List[float]:
        ms = (ctypes.c_float * 6)()
        self.lib.pii_last_timings(self.h, ms)
        return list(ms)

    def kernel_timings(self) -> dict:
        """Device time of the last call's roofline kernels alone (HIP events on the engine stream), ms."""
        ms = (ctypes.c_float * 8)()
        n = self.lib.pii_last_timings_ex(self.h, ms, 8)
        if n < 0:
            raise self._err(n, "pii_last_timings_ex")
        return {"k_scan": float(ms[6]), "k_redact": float(ms[7])}

    def queue_sizes(self) -> Tuple[int, int]:
        """(candidate pairs, scan events) of the last call."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.pii_last_queue_sizes(self.h, ctypes.byref(a), ctypes.byref(b))
        return int(a.value), int(b.value)

    def stats(self) -> dict:
        """work sizes of the last call (pii_last_stats)"""
        a = (ctypes.c_uint64 * 6)()
        n = self.lib.pii_last_stats(self.h, a, 6)
        if n < 0:
            raise self._err(n, "pii_last_stats")
        keys = ["pairs", "events", "lanes", "lane_bytes", "window_findings_arena", "spans"]
        return {k: int(a[i]) for i, k in enumerate(keys[:n])}

    # ------------------------------------------------------------------ context + histogram
    def context_get(self, slot: int) -> Tuple[int, int]:
        g, t = ctypes.c_int32(), ctypes.c_int64()
        rc = self.lib.pii_context_get(self.h, slot, ctypes.byref(g), ctypes.byref(t))
        if rc != PII_OK:
            raise self._err(rc, "pii_context_get")
        return g.value, t.value

    def context_set(self, slot: int, group: int, ts_us: int) -> None:
        rc = self.lib.pii_context_set(self.h, slot, group, ts_us)
        if rc != PII_OK:
            raise self._err(rc, "pii_context_set")

    def context_resize(self, n_slots: int) -> None:
        """grow the conversation table to n_slots (pii_context_resize): live records and window
        histories are kept, the new slots start empty"""
        rc = self.lib.pii_context_resize(self.h, int(n_slots))
        if rc != PII_OK:
            raise self._err(rc, "pii_context_resize")
        self.n_slots = int(n_slots)

    def context_update(self, texts: Sequence[bytes], conv_slot: Sequence[int], role: Sequence[int],
                       ts_us: Optional[Sequence[int]] = None) -> np.ndarray:
        """The context half of scan_redact alone (pii_context_update): AGENT rows' keyword hits are
        committed as scan_redact would; returns ctx_info (int16 per row)."""
        data, offs = pack(texts)
        n = len(texts)
        slot = np.ascontiguousarray(conv_slot, dtype=np.uint32)
        rl = np.ascontiguousarray(role, dtype=np.uint8)
        ts = None if ts_us is None else np.ascontiguousarray(ts_us, dtype=np.int64)
        ctx = np.empty(n, dtype=np.int16)
        rc = self.lib.pii_context_update(self.h, _ptr(data) if len(data) else None, _ptr(offs), n, _ptr(slot),
                                         _ptr(rl), _ptr(ts), _ptr(ctx))
        if rc != PII_OK:
            raise self._err(rc, "pii_context_update")
        return ctx

    def histogram(self) -> np.ndarray:
        n = len(self.type_names)
        out = np.zeros(n, dtype=np.uint64)
        rc = self.lib.pii_histogram(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n)
        if rc != PII_OK:
            raise self._err(rc, "pii_histogram")
        return out

    def histogram_reset(self) -> None:
        self.lib.pii_histogram_reset(self.h)
