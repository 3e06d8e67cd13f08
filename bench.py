"""Headline benchmark: transcript MB/s scanned+redacted per node, and % of the HBM roofline.

Workload (BASELINE.json configs[1], "config 2"): per GPU, 100k synthetic conversations x 100
utterances = 10M utterances (~120 B, lognormal), one scan+redact pass with per-conversation
expected_pii_type context.  A "step" = one pii_scan_redact_device call over the whole resident batch
(+ the RCCL all-reduce of the per-infoType histogram, the only collective).  Inputs are resident in
HBM before timing; outputs are written to HBM.  Multi-GPU: conversations are sharded by
conversation id (each rank owns its own 100k conversations, weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import importlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
synth = importlib.import_module("context-based-pii_amd.synth")
compiler = importlib.import_module("context-based-pii_amd.compiler")
distributed = importlib.import_module("context-based-pii_amd.distributed")

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s measured copy ceiling
LANE_BYTES = 1024        # BYTES_PER_LANE of csrc/pii_engine.hip (k_scan lane = utterances starting in 1 KiB)
SOURCES = ["context-based-pii_amd/csrc/pii_engine.hip", "context-based-pii_amd/csrc/pii_device.h"]
CFG2_MEAN_LEN = 120.8    # bytes per utterance of the config-2 corpus (1.208 GB / 10M)
METRIC = "transcript MB/s scanned+redacted per node (1/2/4/8 GPU) and % HBM roofline"

# --------------------------------------------------------------------------- CPU baseline (oracle)
_CPU = {}


def _cpu_init(data, offs, role, conv, ts):
    _CPU.update(data=data, offs=offs, role=role, conv=conv, ts=ts)


def _cpu_work(rng):
    from oracle import pii_oracle as O
    cfg = O.RuleConfig.load(_CPU.get("cfg_path"))
    d, o, r, c, t = _CPU["data"], _CPU["offs"], _CPU["role"], _CPU["conv"], _CPU["ts"]
    lo, hi = rng
    rows = [(int(c[i]), int(r[i]), d[int(o[i]):int(o[i + 1])].tobytes(), int(t[i])) for i in range(lo, hi)]
    t0 = time.perf_counter()
    O.process_rows(rows, cfg)
    return time.perf_counter() - t0, int(o[hi] - o[lo])


def cpu_share() -> int:
    """Host cores this process may use: the cgroup CPU quota (the GPU box gives each GPU a share of
    the host), else OMP_NUM_THREADS as the box sets it, else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(n, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(n, int(env))
    return n


def host_cpu_model() -> str:
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(bank, min_bytes: float = 1e9, cfg_path=None, what="config-2"):
    """The oracle (Python re + validators), multi-process over whole conversations on this host's CPU
    share, timed over at least `min_bytes` of the same synthetic distribution (SURVEY §8(d) /
    BASELINE.md §2: the full 1.2 GB config would take minutes, so >= 1 GB is timed and reported as a
    rate)."""
    cores = cpu_share()
    n_conv = int(min_bytes / (100 * CFG2_MEAN_LEN)) + 1
    meta = synth.corpus_meta(n_conv, 100, bank, seed=synth.SEED + 7)
    data = synth.gather_bytes(meta, bank)
    offs = meta.offsets.astype(np.int64)
    blocks = [(c * 100, min(c + 50, n_conv) * 100) for c in range(0, n_conv, 50)]   # 50 conversations each
    ctx = mp.get_context("fork")
    _CPU["cfg_path"] = cfg_path
    t0 = time.perf_counter()
    with ctx.Pool(cores, initializer=_cpu_init, initargs=(data, offs, meta.role, meta.conv_slot, meta.ts_us)) as pool:
        res = pool.map(_cpu_work, blocks, chunksize=1)
    wall = time.perf_counter() - t0
    nbytes = sum(b for _, b in res)
    return {"value": round(nbytes / wall / 1e6, 3), "unit": "MB/s", "cores": cores, "kind": "port",
            "host_cpu": host_cpu_model(), "host_logical_cpus": os.cpu_count(),
            "sample": f"{n_conv} conversations x 100 utterances ({nbytes / 1e9:.3f} GB) of the {what} synthetic "
                      f"distribution, oracle/pii_oracle.py process_rows over whole conversations, multiprocessing "
                      f"fork pool of {cores} (this host's CPU share), wall {wall:.1f}s; the 1.208 GB config-2 batch "
                      f"extrapolates to {1.208e9 / (nbytes / wall):.1f}s"}


def source_digest() -> str:
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    return h.hexdigest()[:16]


N_CU = 256                 # MI355X compute units
CLOCK_HZ = 2.4e9           # engine clock under load (MI355X_MICROARCH.md)


def _pmc_entry(workload: str, n_bytes: int):
    """the committed PMC passes of `workload` (tools/pmc_traffic.py -> profiles/traffic.json), only when
    measured on exactly these kernel sources and this workload size; else None"""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    e = t.get("workloads", {}).get(workload)
    if not e or e.get("source_digest") != source_digest() or e.get("bytes_per_gpu") != n_bytes:
        return None
    return e


def measured_traffic(kernel: str, n_bytes: int, workload: str = "scan"):
    """HBM bytes per launch of `kernel` (a name prefix: k_scan covers every SCAN-group instantiation,
    summed) from the workload's own PMC passes, or None"""
    e = _pmc_entry(workload, n_bytes)
    if e is None:
        return None
    ks = [v for k, v in e.get("kernels", {}).items() if k == kernel or k.startswith(kernel + "<")]
    if not ks or any(v.get("hbm_bytes") is None for v in ks):
        return None
    return int(sum(v["hbm_bytes"] for v in ks))


def measured_pipeline_traffic(n_bytes: int, workload: str = "scan"):
    """HBM bytes of all engine kernels of one call (sum of their per-dispatch means), or None"""
    e = _pmc_entry(workload, n_bytes)
    if e is None:
        return None
    ks = [v.get("hbm_bytes") for v in e.get("kernels", {}).values() if v.get("hbm_bytes") is not None]
    return int(sum(ks)) if ks else None


def roofline_compute(n_bytes: int, scan_ms: float, workload: str = "scan"):
    """k_scan's compute ceiling: the DFA step is bound by LDS-array cycles (three table reads per byte,
    bank conflicts), not by HBM.  LDS-array cycles per launch come from the workload's PMC pass
    (SQ_LDS_IDX_ACTIVE, converted with the tools/micro/lds_calib factor); all N_CU LDS arrays busy
    every CLOCK_HZ cycle is the ceiling."""
    e = _pmc_entry(workload, n_bytes)
    if e is None or not e.get("lds_counter_per_cycle"):
        return None
    ks = [v for k, v in e["kernels"].items() if k.startswith("k_scan<") and v.get("lds_array_cycles")]
    if not ks:
        return None
    cyc = sum(v["lds_array_cycles"] for v in ks)
    conf = sum(v.get("lds_bank_conflict", 0) for v in ks) / max(1, sum(v.get("lds_idx_active", 0) for v in ks))
    t_min = cyc / (N_CU * CLOCK_HZ)
    ceiling = n_bytes / t_min / 1e9
    achieved = n_bytes / (scan_ms / 1e3) / 1e9
    return {"bound": "lds", "kernel": "k_scan", "achieved": round(achieved, 1), "peak": round(ceiling, 1),
            "unit": "GB/s of input", "frac": round(achieved / ceiling, 4),
            "lds_cycles_per_byte": round(cyc / n_bytes, 4), "bank_conflict_share": round(conf, 4),
            "lds_cycles_per_launch": int(cyc),
            "note": f"ceiling = input bytes / (LDS-array cycles / ({N_CU} CUs x {CLOCK_HZ / 1e9:g} GHz)); "
                    "cycles from SQ_LDS_IDX_ACTIVE / tools/micro/lds_calib factor"}


# --------------------------------------------------------------------------- GPU corpus assembly
def gpu_corpus(meta, bank, dev):
    import torch
    bank_data = torch.from_numpy(bank.data).to(dev)
    bank_off = torch.from_numpy(bank.offsets).to(dev)
    bid = torch.from_numpy(meta.bank_id.astype(np.int64)).to(dev)
    offs = torch.from_numpy(meta.offsets.view(np.int64)).to(dev)
    total = int(meta.offsets[-1])
    text = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    n = meta.n
    step = 1 << 20
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        b = bid[lo:hi]
        lens = bank_off[b + 1] - bank_off[b]
        o0 = offs[lo:hi]
        nb = int(offs[hi] - offs[lo])
        rep = torch.repeat_interleave(bank_off[b] - o0, lens)
        idx = torch.arange(int(offs[lo]), int(offs[lo]) + nb, device=dev, dtype=torch.int64) + rep
        text[int(offs[lo]):int(offs[lo]) + nb] = bank_data[idx]
    return text, offs


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class DeviceBatch:
    """One rank's resident config-2 shard, staged into device memory once, plus the output buffers.
    The node's conversations have dense global ids and are sharded as everywhere else
    (distributed.shard_of, SURVEY §8(e): rank = id % world): rank r owns ids r, r + world, ...,
    r + (C - 1) world, kept in its context slots 0..C-1 (slot k = id // world).  Their text is the
    synthetic corpus generated for that rank (seed offset rank * C), so ranks hold different data."""

    def __init__(self, C, U, bank, conv_base, dev, join: int = 1, rank: int = 0, world: int = 1):
        import torch
        self.meta = synth.corpus_meta(C, U, bank, seed=synth.SEED, conv_base=conv_base)
        local = (self.meta.conv_slot - conv_base).astype(np.int64)
        self.conversation_ids = rank + world * np.arange(C, dtype=np.int64)     # global ids this rank owns
        assert all(distributed.shard_of(int(i), world) == rank for i in self.conversation_ids[:64])
        assert (self.conversation_ids[local] // world == local).all()
        self.text, self.offs = gpu_corpus(self.meta, bank, dev)
        self.n = self.meta.n
        self.n_bytes = int(self.meta.offsets[-1])
        self.slot = torch.from_numpy((self.meta.conv_slot - conv_base).view(np.int32)).to(dev)
        self.role = torch.from_numpy(self.meta.role).to(dev)
        self.ts = torch.from_numpy(self.meta.ts_us).to(dev)
        n_utt = self.n                     # capacities follow the utterance count, also for long rows
        if join > 1:
            # long rows (whole transcripts, ccai_insights_function/main.py:47-50): every `join`
            # consecutive utterances form one row, redacted without role context (ROLE_OTHER)
            idx = np.unique(np.append(np.arange(0, self.n + 1, join), self.n))
            self.offs = self.offs[torch.from_numpy(idx).to(dev)].contiguous()
            self.n = len(idx) - 1
            self.slot = torch.arange(self.n, dtype=torch.int32, device=dev) % max(C, 1)
            self.role = torch.full((self.n,), 2, dtype=torch.uint8, device=dev)
            self.ts = self.ts[:self.n].contiguous()
        self.out_cap = self.n_bytes + 48 * n_utt
        self.span_cap = n_utt * 2
        self.out = torch.empty(self.out_cap, dtype=torch.uint8, device=dev)
        self.out_offs = torch.empty(self.n + 1, dtype=torch.int64, device=dev)
        self.spans = torch.empty(self.span_cap * 16, dtype=torch.uint8, device=dev)
        self.ctx = torch.empty(self.n, dtype=torch.int16, device=dev)

    def run(self, eng):
        # the batch is resident and its size known: the declared-size entry point enqueues without a
        # device-to-host read of the offsets (pii_scan_redact_device_ex)
        eng.scan_redact_device_ex(self.text.data_ptr(), self.offs.data_ptr(), self.n, 0, self.n_bytes,
                                  self.slot.data_ptr(), self.role.data_ptr(), self.ts.data_ptr(), self.out.data_ptr(),
                                  self.out_cap, self.out_offs.data_ptr(), self.spans.data_ptr(), self.span_cap,
                                  self.ctx.data_ptr())


def reduce_over_ranks(dist, dev, elapsed: float, local_hist: np.ndarray, sums=()):
    """The timed region's cross-rank bookkeeping (the one data collective is the
    histogram all_reduce): max-over-ranks wall time, the SUM of each per-rank quantity in `sums`, the
    reduced u64[T+1] histogram (last slot = span total), and its check against an all_gather of every
    rank's own counts.  One rank (dist None): the local values.  Returns (elapsed, sums, reduced,
    verified)."""
    import torch
    T = len(local_hist) - 1
    sums = [float(x) for x in sums]
    if dist is None:
        return elapsed, sums, local_hist.copy(), bool(local_hist[T] == local_hist[:T].sum())
    world = dist.get_world_size()
    t = torch.tensor([elapsed] + sums, dtype=torch.float64, device=dev)
    dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
    if sums:
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    # (clone: on a CPU device .to() would alias the caller's array, and all_reduce works in place)
    h = torch.from_numpy(np.array(local_hist, dtype=np.int64)).to(dev).clone()
    dist.all_reduce(h)                                    # RCCL over xGMI under nccl: per-infoType counts
    reduced = h.cpu().numpy()
    parts = [torch.zeros(T + 1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(np.array(local_hist, dtype=np.int64)).to(dev).clone())
    want = np.sum([p.cpu().numpy() for p in parts], axis=0)
    verified = bool((want == reduced).all() and reduced[T] == reduced[:T].sum())
    return float(t[0].item()), [float(x) for x in t[1:].tolist()], reduced, verified


STAGES_NOTE = ("stages_ms: stage boundaries from HIP events (timing level 2) on 3 steps after the timed region "
               "(in the timed steps the engine records only the call's start / end and the events around "
               "k_scan and k_redact: each event between kernels costs the stream ~6 us); pipeline.GBps uses the "
               "timed steps' start-to-completion time")


def stage_probe(eng, step, n: int = 3):
    """per-stage device times (pii_last_timings [0..5] at timing level 2) averaged over n further
    calls of `step`; the engine is left at level 1"""
    eng.set_timing(2)
    acc = np.zeros(6)
    try:
        for i in range(n):
            step(i)
            acc += np.array(eng.timings())
    finally:
        eng.set_timing(1)
    return acc / n


def one_stream_scan_ms(B, make_engine, C, steps: int = 3) -> float:
    """k_scan device time per step with every SCAN group's pass on ONE stream (PII_SCAN_STREAMS=1,
    read at engine creation): the passes then run back to back, so the span between the events around
    the scan stage is the sum of the per-pass kernel times.  (With the passes on three streams the
    span is a wall-clock interval in which passes overlap: not a per-kernel time -- VERDICT r5.)"""
    old = os.environ.get("PII_SCAN_STREAMS")
    os.environ["PII_SCAN_STREAMS"] = "1"
    try:
        eng = make_engine(B, None, C)
    finally:
        if old is None:
            del os.environ["PII_SCAN_STREAMS"]
        else:
            os.environ["PII_SCAN_STREAMS"] = old
    tot = 0.0
    try:
        for i in range(steps + 1):
            B.run(eng)
            _, _, fl = eng.sync()
            if fl:
                raise RuntimeError(f"engine error flags {fl}")
            if i:                                  # (the first call sizes the work buffers)
                tot += eng.kernel_timings()["k_scan"]
    finally:
        eng.close()
    return tot / steps


def run_rank(args, rank: int, world: int, dev, make_engine, cpu=None, dist=None, bank=None,
             one_stream_probe: bool = False):
    """One rank of the config-2 benchmark: shard -> W warmup steps -> K timed steps between barriers
    + device syncs -> max-over-ranks time.  A step = one scan+redact pass over the rank's resident
    shard + the all-reduce of the u64[T+1] per-infoType histogram (the only collective; reset every
    step).  After timing, the reduced histogram of the last step is checked against an all-gather
    of every rank's own counts.  Returns the JSON line on rank 0 (None elsewhere)."""
    import torch
    if bank is None:
        bank = synth.build_bank(args.bank, args.bank, seed=synth.SEED)
    C, U = args.conversations, args.utt_per_conv
    join = max(1, int(getattr(args, "row_kb", 0) * 1024 / CFG2_MEAN_LEN)) if getattr(args, "workload", "") == "long" else 1
    B = DeviceBatch(C, U, bank, rank * C, dev, join=join, rank=rank, world=world)
    eng = make_engine(B, bank, C)
    T = len(eng.type_names)
    hist = torch.zeros(T + 1, dtype=torch.int64, device=dev)
    local = np.zeros(T + 1, dtype=np.int64)
    _sync(dev)

    def launch():
        eng.histogram_reset()                               # (deferred to the call's first kernel)
        B.run(eng)

    def finish():
        ob, ns, fl = eng.sync()
        if fl:
            raise RuntimeError(f"engine error flags {fl}")
        local[:T] = eng.histogram().astype(np.int64)
        local[T] = ns
        return ob, ns

    def reduce():
        if world > 1:
            hist.copy_(torch.from_numpy(local))
            dist.all_reduce(hist)                           # RCCL over xGMI: per-infoType counts

    def step():
        launch()
        ob, ns = finish()
        reduce()
        return ob, ns

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    _sync(dev)
    per_stage = np.zeros(6)
    k_ms = {"k_scan": 0.0, "k_redact": 0.0}
    t0 = time.perf_counter()
    # step i+1 is enqueued as soon as step i's counts are read, so the host work of step i (its
    # all-reduce, the bookkeeping) overlaps the device's work on step i+1; every step is still one
    # engine call and one all-reduce inside the timed region
    launch()
    for i in range(args.steps):
        ob, ns = finish()
        if i + 1 < args.steps:
            launch()
        reduce()
        per_stage += np.array(eng.timings())
        for k, v in eng.kernel_timings().items():
            k_ms[k] += v
    if world > 1:
        dist.barrier()
    _sync(dev)
    elapsed = time.perf_counter() - t0
    elapsed, _, reduced, verified = reduce_over_ranks(dist if world > 1 else None, dev, elapsed, local)
    if world > 1:        # the last step's in-loop all_reduce agrees with the one after timing
        verified = verified and bool((hist.cpu().numpy() == reduced).all())
    per_stage /= args.steps
    k_ms = {k: v / args.steps for k, v in k_ms.items()}
    stages = stage_probe(eng, lambda i: step())
    n_pairs, n_events = eng.queue_sizes()
    names = list(eng.type_names)
    eng.close()
    if rank != 0:
        return None
    scan_wall_ms = None
    if one_stream_probe:         # (after the timed region: per-pass k_scan time for the roofline)
        scan_wall_ms = k_ms["k_scan"]
        k_ms["k_scan"] = one_stream_scan_ms(B, make_engine, C)
    n, n_bytes = B.n, B.n_bytes
    n_lanes = (n_bytes + LANE_BYTES - 1) // LANE_BYTES
    ms_step = elapsed / args.steps * 1e3
    total_bytes = n_bytes * world * args.steps
    mbps = total_bytes / elapsed / 1e6
    # SURVEY 8(d) whole-path algorithmic bytes: in + out + in/out offsets + slot/role + spans
    Bw = n_bytes + ob + 8 * (n + 1) * 2 + 5 * n + 16 * ns
    t_pipe = max(per_stage[5], 1e-9) / 1e3
    # dominant kernel k_scan, algorithmic bytes per launch (DESIGN.md "Roofline accounting"):
    # every utterance byte once + the utterance-start bitmap (1 bit per byte) + per lane its
    # first_utt pair, offsets pair, event count (24 B) + 8 B per event written
    scan_B = n_bytes + (n_bytes + 63) // 64 * 8 + 24 * n_lanes + 8 * n_events
    scan_GBps = scan_B / max(k_ms["k_scan"] / 1e3, 1e-12) / 1e9
    # k_redact: what it moves -- the input bytes, the output bytes, one 16-B RSpan per kept span and
    # the 4-B first-span index per 64 KiB output tile (no offsets / counts, it reads none)
    red_B = n_bytes + ob + 16 * ns + 4 * ((ob >> 16) + 2)
    red_GBps = red_B / max(k_ms["k_redact"] / 1e3, 1e-12) / 1e9
    wl = getattr(args, "workload", "scan")
    traffic = measured_traffic("k_scan", n_bytes, wl)
    pipe_traffic = measured_pipeline_traffic(n_bytes, wl)
    rc = roofline_compute(n_bytes, k_ms["k_scan"], wl)
    return {
        "metric": METRIC, "value": round(mbps, 1), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": getattr(args, "workload_desc", None) or
                   "config2: per GPU 100k conversations x 100 utterances (10M utterances, "
                   "~120 B lognormal) single-utterance scan+redact with expected_pii_type context"
                   if join == 1 else
                   f"long rows: the config-2 bytes as {n} rows of ~{args.row_kb} KiB (whole transcripts, {join} "
                   f"utterances each, no role context), cut into halo-scanned lanes",
                   "utterances_per_gpu": n, "bytes_per_gpu": n_bytes, "parallelism": f"conversation-sharded x{world}",
                   "rules": getattr(args, "rules_desc", None) or
                   "main_service/dlp_config.yaml + rules/builtin_infotypes.yaml"},
        "utt_per_s": round(n * world * args.steps / elapsed, 1),
        "spans_per_step_per_gpu": int(ns),
        "queues_per_step_per_gpu": {"scan_events": n_events, "candidate_pairs": n_pairs},
        "stages_ms": {k: round(float(v), 4) for k, v in zip(
            ["scan+pairs", "context", "resolve", "offsets", "redact", "pipeline"], stages)},
        "stages_note": STAGES_NOTE,
        "kernels_ms": {k: round(v, 4) for k, v in k_ms.items()},
        **({"scan_stage_wall_ms": round(scan_wall_ms, 4),
            "scan_stage_note": "kernels_ms.k_scan and roofline.launch_ms: the SCAN passes' kernel time, from "
                               "an engine with the passes on one stream (PII_SCAN_STREAMS=1, after the timed "
                               "region); scan_stage_wall_ms: the wall span of the overlapped passes in the "
                               "timed steps (three streams)"} if scan_wall_ms is not None else {}),
        "pipeline": {"algorithmic_bytes": int(Bw), "GBps": round(Bw / t_pipe / 1e9, 1),
                     "frac": round(Bw / t_pipe / 1e9 / HBM_PEAK_GBPS, 4), "traffic": pipe_traffic},
        "roofline": {"bound": "hbm", "kernel": "k_scan", "achieved": round(scan_GBps, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(scan_GBps / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "algorithmic_bytes": int(scan_B), "launch_ms": round(k_ms["k_scan"], 4),
                     "input_frac": round(n_bytes / (k_ms["k_scan"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "roofline_compute": rc,
        "roofline_redact": {"bound": "hbm", "kernel": "k_redact", "achieved": round(red_GBps, 1),
                            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(red_GBps / HBM_PEAK_GBPS, 4),
                            "traffic": measured_traffic("k_redact", n_bytes, wl),
                            "algorithmic_bytes": int(red_B), "launch_ms": round(k_ms["k_redact"], 4)},
        "histogram": {"collective": "all_reduce u64[T+1] (RCCL)" if world > 1 else "none (1 rank)",
                      "total_spans_last_step": int(reduced[T]), "verified": verified,
                      "per_type": {names[t]: int(reduced[t]) for t in range(T) if reduced[t]}},
        "cpu_baseline": cpu,
    }


def _spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) without a launcher: start N rank processes with
    torch.distributed.run from this GPU-free parent (no HIP call has happened here) and exit with
    their status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--conversations", type=int, default=100_000, help="per GPU")
    ap.add_argument("--utt-per-conv", type=int, default=100)
    ap.add_argument("--bank", type=int, default=16384, help="agent / customer utterance bank size")
    ap.add_argument("--cpu-gb", type=float, default=1.0, help="bytes the CPU baseline times (>= 1 GB, BASELINE.md)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="(config 3 baseline) CPU seconds")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["scan", "window", "stream", "long", "config5", "ner", "ner-redact",
                                           "service"],
                    default="scan",
                    help="scan = config 2 (headline); window = config 3 multi-turn re-scan; "
                         "stream = config 4 PCIe-inclusive batch stream; long = config-2 bytes as long rows; "
                         "config5 = 500+ custom regex / dictionary infoTypes; ner = the BERT forward alone; "
                         "ner-redact = NER detector + scan+redact with its PERSON_NAME spans in one step")
    ap.add_argument("--row-kb", type=int, default=1024, help="(long) row size, KiB")
    ap.add_argument("--ner-batch", type=int, default=64, help="(ner) sequences per step")
    ap.add_argument("--ner-seq", type=int, default=128, help="(ner) tokens per sequence")
    ap.add_argument("--ner-rows", type=int, default=8192, help="(ner-redact) utterances per step")
    ap.add_argument("--clients", type=int, default=64, help="(service) concurrent HTTP clients")
    ap.add_argument("--requests", type=int, default=200, help="(service) requests per client")
    ap.add_argument("--batch-wait-ms", type=float, default=0.5, help="(service) MicroBatcher max_wait")
    ap.add_argument("--window-n", type=int, default=5)
    ap.add_argument("--window-full", action="store_true", help="(window) force the full re-scan of the joined windows")
    ap.add_argument("--window-rules", choices=["shipped", "config5"], default="shipped",
                    help="(window) the shipped rules, or config 5's 542-type rule set (7 SCAN groups)")
    ap.add_argument("--stream-gb", type=float, default=100.0, help="(config 4) stream size per node, GB")
    ap.add_argument("--stream-weak", action="store_true", help="(config 4) --stream-gb per GPU instead of per node")
    ap.add_argument("--shard-gb", type=float, default=1.0, help="(config 4) host shard each rank replays, GB")
    args = ap.parse_args()
    if args.workload == "window":
        return window_main(args)
    if args.workload == "stream":
        return stream_main(args)
    if args.workload == "config5":
        return config5_main(args)
    if args.workload == "ner":
        return ner_main(args)
    if args.workload == "ner-redact":
        return ner_redact_main(args)
    if args.workload == "service":
        return service_main(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        bank = synth.build_bank(args.bank, args.bank, seed=synth.SEED)
        cpu = cpu_baseline(bank, args.cpu_gb * 1e9)           # before any HIP initialisation (fork pool)

    import torch
    import torch.distributed as dist
    eng_mod = importlib.import_module("context-based-pii_amd.engine")
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comp = compiler.compile_default()

    def make_engine(batch, bank, C):
        return eng_mod.Engine(comp.blob, device=local, n_conv_slots=C)
    line = run_rank(args, rank, world, dev, make_engine, cpu=cpu, dist=dist if world > 1 else None)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- config 5: NER on MFMA
MFMA_BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 (MI355X_MICROARCH.md; the 2:1-sparse figure is not used)


def ner_main(args):
    """BASELINE config 5's optional NER: bf16 BERT-base token classification (ner.py / csrc/ner.hip)
    over a batch of --ner-batch sequences x --ner-seq tokens.  value = tokens/s of the whole forward;
    roofline = the MFMA GEMM (k_gemm) alone, timed with HIP events on the stream it runs on, against
    the dense bf16 peak.  cpu_baseline = the same HF model in fp32 on the host's CPU share."""
    import torch
    N = importlib.import_module("context-based-pii_amd.ner")
    B, S = args.ner_batch, args.ner_seq
    cpu = None
    ref = N.reference_model(seed=0)
    rng = np.random.default_rng(1)
    ids = rng.integers(1000, 30522, size=(B, S)).astype(np.int32)
    ids[:, 0], ids[:, -1] = N.CLS, N.SEP
    mask = np.ones((B, S), dtype=np.int32)
    if not args.no_cpu_baseline:
        cores = cpu_share()
        torch.set_num_threads(cores)
        nb = max(1, min(B, 8))
        with torch.no_grad():
            ref(input_ids=torch.as_tensor(ids[:1], dtype=torch.long))
            t0 = time.perf_counter()
            ref(input_ids=torch.as_tensor(ids[:nb], dtype=torch.long),
                attention_mask=torch.as_tensor(mask[:nb], dtype=torch.long))
            dt = time.perf_counter() - t0
        cpu = {"value": round(nb * S / dt, 1), "unit": "tokens/s", "cores": cores, "kind": "reference",
               "host_cpu": host_cpu_model(),
               "sample": f"HF transformers BertForTokenClassification(BertConfig()) fp32 forward, {nb} x {S} tokens, "
                         f"torch.set_num_threads({cores}), wall {dt:.2f}s"}
    torch.cuda.set_device(0)
    m = N.BertNer(ref, device=0)
    dev = m.dev
    d_ids, d_mask = torch.as_tensor(ids).to(dev), torch.as_tensor(mask).to(dev)
    for _ in range(args.warmup):
        m.forward(d_ids, d_mask)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.forward(d_ids, d_mask)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tokens = B * S
    # k_gemm alone: one layer's four GEMMs, HIP events on the current stream (where the kernels run)
    Mp = (tokens + 127) // 128 * 128
    bu = m._buffers(Mp)
    Ly = m.layers[0]
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record(st)
    for _ in range(reps):
        m.gemm(bu["h"], Ly["wqkv"], Ly["bqkv"], bu["qkv"])
        m.gemm(bu["ctx"], Ly["wo"], Ly["bo"], bu["a"], N.EPI_RESID, resid=bu["h"])
        m.gemm(bu["h1"], Ly["wi"], Ly["bi"], bu["f"], N.EPI_GELU)
        m.gemm(bu["f"], Ly["wf"], Ly["bf"], bu["a"], N.EPI_RESID, resid=bu["h1"])
    e1.record(st)
    e1.synchronize()
    g_ms = e0.elapsed_time(e1) / reps
    H, I = m.H, m.inter
    g_flop = 2.0 * Mp * (H * 3 * H + H * H + 2 * H * I)
    g_tf = g_flop / (g_ms / 1e3) / 1e12
    flop = m.flops_per_token(S) * tokens
    line = {
        "metric": "config 5 NER: tokens/s of bf16 BERT-base token classification (MFMA)", "value": round(tokens * args.steps / el, 1),
        "unit": "tokens/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"BertConfig() (bert-base, 12 layers, hidden 768) seeded random weights, {B} x {S} tokens",
                   "model": "bert-base token classification (3 labels)", "global_batch": B, "seq_len": S},
        "tflops_forward": round(flop * args.steps / el / 1e12, 1),
        "roofline": {"bound": "mfma", "kernel": "k_gemm", "achieved": round(g_tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(g_tf / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None,
                     "algorithmic_flop": int(g_flop), "launch_ms": round(g_ms / 4, 4)},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def _name_rows(n_rows, seed=synth.SEED):
    """config-2-shaped conversations (16 utterances each, AGENT / END_USER alternating) whose customer
    rows say a name half of the time ("my name is Jane Kim. ...")"""
    import random
    r = random.Random(seed)
    bank = synth.build_bank(4096, 4096, seed=seed)
    texts, roles, convs = [], [], []
    for i in range(n_rows):
        agent = i % 2 == 0
        t = r.choice(bank.texts[:4096] if agent else bank.texts[4096:])
        if not agent and r.random() < 0.5:
            t = f"my name is {r.choice(synth.NAMES).capitalize()} {r.choice(synth.NAMES).capitalize()}. ".encode() + t
        texts.append(t)
        roles.append(1 if agent else 0)
        convs.append(i // 16)
    return texts, roles, convs


def ner_redact_main(args):
    """SURVEY §8(f)4 on the redaction path: one step = the NER detector on the GPU (k_tokenize ->
    bf16 BERT-base forward on MFMA -> k_ner_spans) over --ner-rows resident utterances, then the
    scan+redact call with its PERSON_NAME spans as external candidates (pii_scan_redact_device_ext),
    no host round trip in between.  value = transcript MB/s of the whole step; the NER and engine
    shares come from HIP events on the stream both run on.  cpu_baseline = HF fp32 NER + the oracle
    on a sample of the same rows, on the host's CPU share."""
    import torch
    N = importlib.import_module("context-based-pii_amd.ner")
    E = importlib.import_module("context-based-pii_amd.engine")
    n, S = args.ner_rows, 64
    texts, roles, convs = _name_rows(n)
    data, offs = E.pack(texts)
    ref = N.reference_model(seed=0)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import pii_oracle as O
        cores = cpu_share()
        torch.set_num_threads(cores)
        cfg = O.RuleConfig.load()
        P = cfg.type_id["PERSON_NAME"]
        nb = min(n, 256)
        tok = N.HashTokenizer(max_len=S)
        t0 = time.perf_counter()
        ids, mask, sp = tok.batch(texts[:nb])
        with torch.no_grad():
            lab = ref(input_ids=torch.as_tensor(ids, dtype=torch.long),
                      attention_mask=torch.as_tensor(mask, dtype=torch.long)).logits.argmax(-1).numpy()
        ext = [[(a, b, P, N.LIKELY) for a, b in N.decode_spans(lab[i], sp[i])] for i in range(nb)]
        O.process_rows([(convs[i], roles[i], texts[i], 0) for i in range(nb)], cfg, extra=ext)
        dt = time.perf_counter() - t0
        nbytes = int(offs[nb])
        cpu = {"value": round(nbytes / dt / 1e6, 4), "unit": "MB/s", "cores": cores, "kind": "port",
               "host_cpu": host_cpu_model(),
               "sample": f"{nb} of the step's utterances ({nbytes} B): HashTokenizer + HF BertForTokenClassification "
                         f"fp32 (torch.set_num_threads({cores})) + oracle/pii_oracle.py process_rows with the spans, "
                         f"wall {dt:.2f}s"}
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comp = compiler.compile_default()
    eng = E.Engine(comp.blob, device=0, n_conv_slots=n // 16 + 2)
    P = eng.type_names.index("PERSON_NAME")
    m = N.BertNer(ref, device=0)
    d_text = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_slot = torch.tensor(convs, dtype=torch.int32, device=dev)
    d_role = torch.tensor(roles, dtype=torch.uint8, device=dev)
    d_ts = torch.zeros(n, dtype=torch.int64, device=dev)
    out_cap = int(offs[-1]) * 4 + 64 * n
    span_cap = int(offs[-1]) + n
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, device=dev)
    d_ctx = torch.empty(n, dtype=torch.int16, device=dev)
    # one explicit stream for the detector and the engine: a NULL stream handle would select the
    # engine's own stream, which is not ordered after the detector's kernels
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.set_stream(st)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    acc = np.zeros(2)

    def step(timed):
        eng.histogram_reset()
        ev[0].record(st)
        ext, ext_n, stride = m.detect_device(d_text.data_ptr(), d_offs.data_ptr(), n, S=S, info_type=P)
        ev[1].record(st)
        eng.scan_redact_device_ext(d_text.data_ptr(), d_offs.data_ptr(), n, 0, int(offs[-1]), d_slot.data_ptr(),
                                   d_role.data_ptr(), d_ts.data_ptr(), d_out.data_ptr(), out_cap, d_oo.data_ptr(),
                                   d_sp.data_ptr(), span_cap, d_ctx.data_ptr(), ext.data_ptr(), ext_n.data_ptr(),
                                   stride, st.cuda_stream)
        ev[2].record(st)
        ob, ns, fl = eng.sync()
        if fl:
            raise RuntimeError(f"engine error flags {fl}")
        if timed:
            ev[2].synchronize()
            acc[0] += ev[0].elapsed_time(ev[1])
            acc[1] += ev[1].elapsed_time(ev[2])
        return ns
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ns = step(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    hist = eng.histogram()
    tokens = n * S
    flop = m.flops_per_token(S) * tokens
    ner_ms, eng_ms = acc / args.steps
    line = {
        "metric": "config 5 NER on the redaction path: transcript MB/s (NER + scan+redact per step)",
        "value": round(int(offs[-1]) * args.steps / el / 1e6, 3), "unit": "MB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"{n} config-2 utterances (16 per conversation, half the customer rows with a name), "
                               f"NER at {S} tokens per utterance (BertConfig() seeded random weights) -> PERSON_NAME "
                               f"external candidates -> scan+redact with context", "bytes_per_step": int(offs[-1])},
        "utt_per_s": round(n * args.steps / el, 1),
        "ner_ms": round(float(ner_ms), 3), "engine_ms": round(float(eng_ms), 3),
        "ner_tflops": round(flop / (ner_ms / 1e3) / 1e12, 1),
        "person_name_findings_last_step": int(hist[P]), "spans_last_step": int(ns),
        "roofline": {"bound": "mfma", "kernel": "NER forward (k_gemm + attention)", "achieved":
                     round(flop / (ner_ms / 1e3) / 1e12, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flop / (ner_ms / 1e3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None},
        "cpu_baseline": cpu,
    }
    eng.close()
    print(json.dumps(line), flush=True)


# --------------------------------------------------------------------------- the drop-in service
def _service_client(port, k0, n_threads, n, texts_a, texts_c, out_q):
    """one client PROCESS (spawned: it never touches the GPU): n_threads keep-alive connections, each
    replaying its own conversation; reports (latencies, bytes, errors)"""
    import http.client
    import random
    import threading
    lat, nb, err = [], [0], [0]
    lock = threading.Lock()

    def one(k):
        r = random.Random(k)
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
        mine = []
        b = e = 0
        for j in range(n):
            agent = j % 2 == 0
            text = r.choice(texts_a if agent else texts_c)
            body = json.dumps({"conversation_id": f"c{k}", "transcript": text})
            t0 = time.perf_counter()
            conn.request("POST", "/handle-agent-utterance" if agent else "/handle-customer-utterance", body,
                         {"Content-Type": "application/json"})
            resp = conn.getresponse()
            resp.read()
            mine.append(time.perf_counter() - t0)
            b += len(text.encode())
            e += resp.status != 200
        conn.close()
        with lock:
            lat.extend(mine)
            nb[0] += b
            err[0] += e
    ts = [threading.Thread(target=one, args=(k0 + i,)) for i in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    out_q.put((lat, nb[0], err[0]))


def service_main(args):
    """The Flask drop-in (app.py) on the engine, over real HTTP on 127.0.0.1: --clients connections
    spread over spawned client processes (so the clients do not share the server's interpreter), each
    replaying its own conversation (agent question / customer answer alternating,
    /handle-agent-utterance and /handle-customer-utterance), --requests each.  Reports requests/s and
    latency percentiles, and the micro-batch sizes the batcher formed.  The reference's deployment
    serves these routes with 1 gunicorn worker x 8 threads, one blocking DLP RPC per request
    (main_service/Dockerfile:29): at most 8 requests in flight; its DLP latency is not published, so
    no reference rate is quoted."""
    import threading
    import logging
    from werkzeug.serving import make_server
    bank = synth.build_bank(4096, 4096, seed=synth.SEED)
    texts_a = [t.decode() for t in bank.texts[:4096]]
    texts_c = [t.decode() for t in bank.texts[4096:]]
    C, R = args.clients, args.requests
    n_proc = max(1, min(C, cpu_share() // 2))
    ctx = mp.get_context("spawn")
    import torch
    A = importlib.import_module("context-based-pii_amd.app")
    S = importlib.import_module("context-based-pii_amd.service")
    torch.cuda.set_device(0)
    svc = S.PiiService(n_slots=1 << 14)
    app = A.create_app(svc, max_batch=1024, max_wait_s=args.batch_wait_ms / 1e3)
    logging.getLogger("werkzeug").setLevel(logging.ERROR)
    srv = make_server("127.0.0.1", 0, app, threaded=True)
    port = srv.server_port
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    batcher = app.config["PII_BATCHER"]

    def run(n):
        q = ctx.Queue()
        per = [C // n_proc + (1 if i < C % n_proc else 0) for i in range(n_proc)]
        ps, k0 = [], 0
        for i in range(n_proc):
            ps.append(ctx.Process(target=_service_client, args=(port, k0, per[i], n, texts_a, texts_c, q)))
            k0 += per[i]
        t0 = time.perf_counter()
        for p in ps:
            p.start()
        res = [q.get() for _ in ps]
        el = time.perf_counter() - t0
        for p in ps:
            p.join()
        return el, res
    run(max(2, R // 10))                           # warmup: engine buffers, connections, interpreters
    batcher.batches.clear()
    el, res = run(R)
    srv.shutdown()
    all_lat = np.sort(np.concatenate([np.array(r[0]) for r in res])) * 1e3
    n_req = len(all_lat)
    nbytes = sum(r[1] for r in res)
    errors = sum(r[2] for r in res)
    sizes = np.array(batcher.batches)
    # the same kind of requests through PiiService.process_requests directly (no HTTP, no batcher),
    # in micro-batches of 1024: the rate the engine path itself sustains
    import random
    r = random.Random(0)
    reqs = []
    for j in range(R):
        for k in range(C):
            agent = j % 2 == 0
            reqs.append(("agent" if agent else "customer",
                         {"conversation_id": f"d{k}", "transcript": r.choice(texts_a if agent else texts_c)}))
    svc.process_requests(reqs[:C * 2])
    t0 = time.perf_counter()
    for i in range(0, len(reqs), 1024):
        svc.process_requests(reqs[i:i + 1024])
    direct = len(reqs) / (time.perf_counter() - t0)
    batcher.close()
    line = {
        "metric": "drop-in service: requests/s through the Flask shim (app.py) on one MI355X, with latency",
        "value": round(n_req / el, 1), "unit": "requests/s", "n_gpus": 1, "steps": R, "warmup": max(2, R // 10),
        "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"{C} HTTP/1.1 keep-alive clients in {n_proc} spawned processes on 127.0.0.1 x {R} "
                               f"requests, each client one conversation alternating /handle-agent-utterance and "
                               f"/handle-customer-utterance (config-2 utterances), werkzeug threaded server, "
                               f"MicroBatcher(max_batch=1024, max_wait={args.batch_wait_ms:g} ms)", "clients": C,
                   "batch_wait_ms": args.batch_wait_ms},
        "latency_ms": {"p50": round(float(np.percentile(all_lat, 50)), 3),
                       "p90": round(float(np.percentile(all_lat, 90)), 3),
                       "p99": round(float(np.percentile(all_lat, 99)), 3), "max": round(float(all_lat[-1]), 3)},
        "transcript_MBps": round(nbytes / el / 1e6, 3),
        "errors": int(errors),
        "micro_batches": {"count": int(len(sizes)), "mean_size": round(float(sizes.mean()), 2) if len(sizes) else 0,
                          "max_size": int(sizes.max()) if len(sizes) else 0},
        "process_requests_direct_per_s": round(direct, 1),
        "reference_concurrency": "1 gunicorn worker x 8 threads = at most 8 DLP RPCs in flight "
                                 "(main_service/Dockerfile:29); the DLP latency is not published",
    }
    svc.engine.close()
    print(json.dumps(line), flush=True)


# --------------------------------------------------------------------------- config 5: 500+ types
def config5_main(args):
    """BASELINE config 5: the config-2 shape (conversations x 100 utterances, one scan+redact pass per
    step) over a seeded rule set of 520 custom regex / dictionary infoTypes + the shipped ones
    (rulegen.Config5), text drawn from a bank of config-5 utterances.  The rule set is split over
    several SCAN groups (one k_scan pass each) and its FIRST automata are read from global memory
    (L2-resident); the L2 hit rate of those kernels comes from a committed PMC pass (profiles/)."""
    import tempfile
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))
    rulegen = importlib.import_module("context-based-pii_amd.rulegen")
    c5 = rulegen.Config5()
    path = os.path.join(tempfile.gettempdir(), f"config5_{os.getpid()}.json")
    c5.save(path)
    bank = c5.build_bank()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(bank, args.cpu_gb * 1e9, cfg_path=path, what="config-5")
    import torch
    import torch.distributed as dist
    eng_mod = importlib.import_module("context-based-pii_amd.engine")
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comp = compiler.compile_rules(compiler.Rules.load(path))
    args.workload_desc = (f"config5: per GPU {args.conversations} conversations x {args.utt_per_conv} utterances "
                          f"of config-5 text, scan+redact over {len(comp.rules.type_names)} infoTypes "
                          f"({len(comp.rules.patterns)} detector patterns in {len(comp.scan_groups)} SCAN groups)")
    args.rules_desc = "rules/dlp_config.json + rulegen.Config5(n_regex=320, n_dict=200, seed=5)"

    def make_engine(batch, bank_, C):
        return eng_mod.Engine(comp.blob, device=local, n_conv_slots=C)
    line = run_rank(args, rank, world, dev, make_engine, cpu=cpu, dist=dist if world > 1 else None, bank=bank,
                    one_stream_probe=len(comp.scan_groups) > 1)
    if rank == 0:
        line["metric"] = "config 5: transcript MB/s scanned+redacted per node with 500+ custom infoTypes"
        line["l2"] = measured_l2()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    os.unlink(path)


def measured_l2():
    """TCC hit rate of the config-5 kernels from the committed PMC pass (tools/pmc_l2.py), if it was
    measured on these kernel sources"""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "config5_l2.json")))
    except (OSError, ValueError):
        return None
    return t if t.get("source_digest") == source_digest() else None


# --------------------------------------------------------------------------- config 4: batch stream
STREAM_BATCH = 256 << 20      # per-GPU double-buffered batches of 256 MB


def _host_ring(args, rank, bank, dev):
    """One rank's 1 GB host shard (SURVEY config 4: generated in 1 GB shards): conversations
    [rank*C, (rank+1)*C) in stream order (every conversation's k-th utterance, then the (k+1)-th: a
    conversation's rows spread over all batches), assembled on the GPU from the utterance bank and
    copied into pinned host memory, cut into 256 MB batches (HostBatch views of the pinned shard)."""
    import torch
    S = importlib.import_module("context-based-pii_amd.stream")
    U = 100
    C = max(1, int(args.shard_gb * 1e9 / (U * CFG2_MEAN_LEN)))
    steps = max(1, int(STREAM_BATCH / (C * CFG2_MEAN_LEN * 1.02)))      # steps of every conversation per batch
    perm, ranges = synth.stream_order(C, U, steps)
    meta = synth.reorder(synth.corpus_meta(C, U, bank, seed=synth.SEED + 11, conv_base=rank * C), bank, perm)
    text, _ = gpu_corpus(meta, bank, dev)
    n_bytes = int(meta.offsets[-1])
    h_text = torch.empty(n_bytes + 64, dtype=torch.uint8, pin_memory=True)
    h_text.copy_(text[:n_bytes + 64])              # device -> pinned host
    del text
    offs = meta.offsets.astype(np.int64)
    slot = (meta.conv_slot - np.uint32(rank * C)).astype(np.int32)
    batches = []
    for lo, hi in ranges:
        b0, b1 = int(offs[lo]), int(offs[hi])
        pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory()  # noqa: E731
        batches.append(S.HostBatch(h_text[b0:b1], pin(offs[lo:hi + 1] - b0), pin(slot[lo:hi]), pin(meta.role[lo:hi]),
                                   pin(meta.ts_us[lo:hi]), hi - lo, b1 - b0))
    return batches, C, n_bytes


def _copy_rate(nbytes, dev, h2d: bool):
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for _ in range(2):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize(dev)
    return 5 * nbytes / (time.perf_counter() - t0) / 1e9


def stream_rank(args, rank, world, dev, eng, dist=None, cpu=None):
    """BASELINE config 4 on one rank: a --stream-gb stream (whole node) sharded by conversation, each
    rank streaming its share as 256 MB batches from pinned host memory through StreamIngest (H2D of
    batch i+1 and D2H of batch i-1 overlapped with the scan of batch i).  value = input bytes of all
    ranks / max-over-ranks wall time, PCIe-inclusive (host buffers in, host buffers out)."""
    import torch
    S = importlib.import_module("context-based-pii_amd.stream")
    bank = synth.build_bank(args.bank, args.bank, seed=synth.SEED)
    ring, C, ring_bytes = _host_ring(args, rank, bank, dev)
    per_rank = args.stream_gb * 1e9 / world
    K = max(1, int(round(per_rank / (ring_bytes / len(ring)))))
    ing = S.StreamIngest(eng, max_bytes=max(b.n_bytes for b in ring), max_rows=max(b.n for b in ring))
    h2d = _copy_rate(STREAM_BATCH, dev, True)
    d2h = _copy_rate(STREAM_BATCH, dev, False)
    duplex = h2d + d2h                  # PCIe is full duplex: the two one-way copy rates, summed
    T = len(eng.type_names)
    gpu_ms = []

    def consume(i, res):
        gpu_ms.append(eng.timings()[5])
    ing.run((ring[i % len(ring)] for i in range(args.warmup)), None)
    eng.histogram_reset()
    ing.stats.update(batches=0, bytes_in=0, bytes_out=0, spans=0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    st = ing.run((ring[i % len(ring)] for i in range(K)), consume)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    local = np.zeros(T + 1, dtype=np.int64)
    local[:T] = eng.histogram().astype(np.int64)
    local[T] = st["spans"]
    elapsed, (tot_in,), reduced, verified = reduce_over_ranks(dist if world > 1 else None, dev, elapsed, local,
                                                              [st["bytes_in"]])
    tot_in = int(tot_in)
    names = list(eng.type_names)
    if rank != 0:
        return None
    mean_b = st["bytes_in"] / max(st["batches"], 1)
    gpu_s = float(np.mean(gpu_ms)) / 1e3 if gpu_ms else 0.0
    serial = mean_b / (h2d * 1e9) + gpu_s + (st["bytes_out"] / max(st["batches"], 1)) / (d2h * 1e9)
    per_batch = elapsed / max(st["batches"], 1)
    rows_total = sum(ring[i % len(ring)].n for i in range(K))
    # over PCIe per row: in offsets 8 + slot 4 + role 1 + ts 8; out offsets 8 + ctx 2; + 16 B per span
    pcie_GBps = (st["bytes_in"] + st["bytes_out"] + 31 * rows_total + 16 * st["spans"]) / elapsed / 1e9
    return {
        "metric": "config 4 stream: transcript MB/s scanned+redacted per node, PCIe-inclusive (host in, host out)",
        "value": round(tot_in / elapsed / 1e6, 1), "unit": "MB/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(per_batch * 1e3, 3), "higher_is_better": True,
        "scaling": "weak" if args.stream_weak else "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"config4: {args.stream_gb:g} GB stream per node sharded by conversation, 256 MB "
                               f"double-buffered batches from pinned host memory (each rank replays its 1 GB shard, "
                               f"{C} conversations x 100 utterances in stream order)",
                   "batch_bytes": int(mean_b), "batches_per_gpu": K, "bytes_per_gpu": int(st["bytes_in"]),
                   "parallelism": f"conversation-sharded x{world}"},
        "overlap": {"h2d_GBps_alone": round(h2d, 2), "d2h_GBps_alone": round(d2h, 2),
                    "gpu_ms_per_batch": round(gpu_s * 1e3, 3), "wall_ms_per_batch": round(per_batch * 1e3, 3),
                    "serial_ms_per_batch": round(serial * 1e3, 3),
                    "overlap_factor": round(serial / max(per_batch, 1e-12), 3),
                    "bound": "pcie h2d" if mean_b / (h2d * 1e9) >= gpu_s else "gpu"},
        "roofline": {"bound": "pcie", "achieved": round(pcie_GBps, 2), "peak": round(duplex, 2),
                     "unit": "GB/s", "frac": round(pcie_GBps / duplex, 4), "traffic": None,
                     "note": "(input + output + per-row arrays) bytes over PCIe / wall, vs the sum of the measured "
                             "one-way pinned copy rates of a 256 MB batch (H2D + D2H, full duplex)"},
        "capacity_reruns": st["capacity_reruns"],
        "histogram": {"collective": "all_reduce u64[T+1] (RCCL)" if world > 1 else "none (1 rank)",
                      "total_spans": int(reduced[T]), "verified": verified,
                      "per_type": {names[t]: int(reduced[t]) for t in range(T) if reduced[t]}},
        "cpu_baseline": cpu,
    }


def stream_main(args):
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stream_weak:
        args.stream_gb = args.stream_gb * world
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        bank = synth.build_bank(args.bank, args.bank, seed=synth.SEED)
        cpu = cpu_baseline(bank, args.cpu_gb * 1e9)
    import torch
    import torch.distributed as dist
    eng_mod = importlib.import_module("context-based-pii_amd.engine")
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comp = compiler.compile_default()
    C = max(1, int(args.shard_gb * 1e9 / (100 * CFG2_MEAN_LEN)))
    eng = eng_mod.Engine(comp.blob, device=local, n_conv_slots=C)
    line = stream_rank(args, rank, world, dev, eng, dist=dist if world > 1 else None, cpu=cpu)
    eng.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- config 3: window re-scan
def _cpu_window_work(rng):
    from oracle import pii_oracle as O
    cfg = O.RuleConfig.load()
    d, o, r, c, t = _CPU["data"], _CPU["offs"], _CPU["role"], _CPU["conv"], _CPU["ts"]
    lo, hi = rng
    rows = [(int(c[i]), int(r[i]), d[int(o[i]):int(o[i + 1])].tobytes(), int(t[i])) for i in range(lo, hi)]
    n = _CPU["win_n"]
    t0 = time.perf_counter()
    O.process_window_rows(rows, cfg, n=n)
    return time.perf_counter() - t0, int(o[hi] - o[lo])


def cpu_window_baseline(bank, n_win: int, seconds: float = 15.0):
    """oracle.process_window_rows (full re-scan of every joined window: what the reference does per
    utterance) over whole conversations, multi-process on the host; MB/s of NEW utterance bytes."""
    cores = cpu_share()
    probe = synth.corpus_meta(4, 100, bank, seed=synth.SEED + 7)
    pdata = synth.gather_bytes(probe, bank)
    _cpu_init(pdata, probe.offsets.astype(np.int64), probe.role, probe.conv_slot, probe.ts_us)
    _CPU["win_n"] = n_win
    dt, nb = _cpu_window_work((0, probe.n))
    conv_rate = 4 / max(dt, 1e-6)
    n_conv = int(min(20000, max(cores * 4, conv_rate * cores * seconds * 0.5)))
    meta = synth.corpus_meta(n_conv, 100, bank, seed=synth.SEED + 7)
    data = synth.gather_bytes(meta, bank)
    chunks = [(i * 100, (i + 1) * 100) for i in range(n_conv)]
    _cpu_init(data, meta.offsets.astype(np.int64), meta.role, meta.conv_slot, meta.ts_us)
    _CPU["win_n"] = n_win
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_window_work, chunks, chunksize=max(1, len(chunks) // (cores * 8)))
    wall = time.perf_counter() - t0
    nbytes = sum(b for _, b in res)
    return {"value": round(nbytes / wall / 1e6, 3), "unit": "MB/s", "cores": cores, "kind": "port",
            "sample": f"{n_conv} conversations x 100 utterances ({nbytes / 1e6:.1f} MB new bytes), every utterance "
                      f"followed by a full oracle re-scan of its window of {n_win} (process_window_rows), "
                      f"multiprocessing fork pool of {cores}, wall {wall:.1f}s"}


def window_main(args):
    """BASELINE config 3: multi-turn sliding-window re-scan, N = --window-n, over --conversations
    concurrent conversations on one GPU.  A step = one pii_rescan_window_device call carrying the next
    utterance of every conversation (the aggregator's stream); each row yields its redacted window."""
    import torch
    eng_mod = importlib.import_module("context-based-pii_amd.engine")
    C, U, N = args.conversations, args.utt_per_conv, args.window_n
    c5path = None
    if args.window_rules == "config5":          # the re-scan under config 5's 542-type rule set
        import tempfile
        c5 = importlib.import_module("context-based-pii_amd.rulegen").Config5()
        c5path = os.path.join(tempfile.gettempdir(), f"config5_w_{os.getpid()}.json")
        c5.save(c5path)
        bank = c5.build_bank()
    else:
        bank = synth.build_bank(16384, 16384, seed=synth.SEED)
    cpu = None
    if not args.no_cpu_baseline and c5path is None:
        cpu = cpu_window_baseline(bank, N, args.cpu_seconds)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    meta = synth.step_major(synth.corpus_meta(C, U, bank, seed=synth.SEED), bank, C, U)
    text, offs = gpu_corpus(meta, bank, dev)
    slot = torch.from_numpy(meta.conv_slot.view(np.int32)).to(dev)
    role = torch.from_numpy(meta.role).to(dev)
    ts = torch.from_numpy(meta.ts_us).to(dev)
    step_bytes = [int(meta.offsets[(k + 1) * C] - meta.offsets[k * C]) for k in range(U)]
    out_cap = (N + 1) * max(step_bytes) + 64 * N * C
    span_cap = 8 * N * C
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(C + 1, dtype=torch.int64, device=dev)
    d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, device=dev)
    d_ctx = torch.empty(C, dtype=torch.int16, device=dev)
    comp = compiler.compile_rules(compiler.Rules.load(c5path)) if c5path else compiler.compile_default()
    if c5path:
        os.unlink(c5path)
    eng = eng_mod.Engine(comp.blob, device=0, n_conv_slots=C)
    eng.window_enable(N, 8192 if c5path is None else 16384, full=args.window_full)
    torch.cuda.synchronize()

    def launch(k):
        o = offs.data_ptr() + 8 * k * C
        # the step's rows are resident and their span known: no device-to-host read before the launch
        eng.rescan_window_device_ex(text.data_ptr(), o, C, int(meta.offsets[k * C]), step_bytes[k],
                                    slot.data_ptr() + 4 * k * C, role.data_ptr() + k * C, ts.data_ptr() + 8 * k * C,
                                    d_out.data_ptr(), out_cap, d_oo.data_ptr(), d_sp.data_ptr(), span_cap,
                                    d_ctx.data_ptr())

    def finish():
        ob, ns, fl = eng.sync()
        if fl:
            raise RuntimeError(f"engine error flags {fl}")
        return ob, ns

    def step(k):
        launch(k)
        return finish()

    warm = max(args.warmup, N)                 # windows are full from step N-1 on
    if warm + args.steps > U:
        raise SystemExit(f"--warmup + --steps must be <= --utt-per-conv ({U})")
    for k in range(warm):
        step(k)
    torch.cuda.synchronize()
    per_stage = np.zeros(6)
    k_red = 0.0
    new_b = out_b = spans = 0
    t0 = time.perf_counter()
    launch(warm)
    for k in range(warm, warm + args.steps):
        ob, ns = finish()
        # the next call is enqueued before this one's bookkeeping (its timings stay the engine's last
        # ones until the next sync), so the host work between calls overlaps the device's
        if k + 1 < warm + args.steps:
            launch(k + 1)
        per_stage += np.array(eng.timings())
        k_red += eng.kernel_timings()["k_redact"]
        new_b += step_bytes[k]
        out_b += ob
        spans += ns
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    K = args.steps
    per_stage /= K
    k_red /= K
    stages = stage_probe(eng, lambda i: step(warm + K + i)) if warm + K + 3 <= U else per_stage
    wkey = "window_config5" if c5path else "window"          # (profiles/traffic.json: its own PMC passes)
    # window bytes read to write the outputs: every window's utterances and separators
    lens = (meta.offsets[1:] - meta.offsets[:-1]).astype(np.int64).reshape(U, C)
    win_in = 0
    for k in range(warm, warm + K):
        lo = max(0, k - N + 1)
        win_in += int(lens[lo:k + 1].sum()) + (k - lo) * C
    t_pipe = per_stage[5] / 1e3 * K
    # algorithmic bytes: new bytes + window bytes re-read for the output copy +
    # window output written + ring commit of the new bytes + offsets/state (8+8+4+1+8 B per row)
    B = new_b + win_in + out_b + new_b + K * C * (8 + 8 + 4 + 1 + 8) + 16 * spans
    red_B = win_in + out_b + K * C * 24 + 32 * spans
    line = {
        "metric": "multi-turn window re-scan: new transcript MB/s (each utterance -> its redacted window of N)",
        "value": round(new_b / elapsed / 1e6, 1), "unit": "MB/s", "n_gpus": 1, "steps": K, "warmup": warm,
        "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"config3: {C} concurrent conversations, window N={N}, one new utterance per "
                               f"conversation per step (pii_rescan_window_device, {eng.window_mode()} mode), "
                               f"expected_pii_type context" + (", config-5 rules (542 types, 7 SCAN groups)"
                                                               if c5path else ""),
                   "rules": args.window_rules, "mode": eng.window_mode(),
                   "rows_per_step": C, "parallelism": "conversation-sharded x1",
                   # a step processes one new utterance per conversation: its bytes are the per-step
                   # workload; the whole U-step stream stays resident in HBM beside it
                   "bytes_per_gpu": int(new_b / K), "resident_stream_bytes": int(meta.offsets[-1])},
        "windows_per_s": round(K * C / elapsed, 1),
        "window_output_MBps": round(out_b / elapsed / 1e6, 1),
        "naive_equivalent_bytes_rescanned_per_step": int(win_in / K),
        "new_bytes_per_step": int(new_b / K),
        "stages_ms": {k: round(float(v), 4) for k, v in zip(
            ["scan+pairs", "context", "first+cands", "select+offsets", "redact+commit", "pipeline"], stages)},
        "stages_note": STAGES_NOTE,
        "probe_steps": 3 if warm + K + 3 <= U else 0,
        "pipeline": {"algorithmic_bytes": int(B / K), "GBps": round(B / t_pipe / 1e9, 1),
                     "frac": round(B / t_pipe / 1e9 / HBM_PEAK_GBPS, 4),
                     "traffic": measured_pipeline_traffic(int(meta.offsets[-1]), wkey)},
        "roofline": {"bound": "hbm", "kernel": "k_win_redact", "achieved": round(red_B / K / (k_red / 1e3) / 1e9, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(red_B / K / (k_red / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "traffic": measured_traffic("k_win_redact", int(meta.offsets[-1]), wkey),
                     "algorithmic_bytes": int(red_B / K), "launch_ms": round(k_red, 4)},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
