"""bench.py's multi-rank path on CPU (gloo, world size 2): each rank builds its own conversation
shard, runs warmup + timed steps with the per-step histogram reset, all-reduces the u64[T+1]
per-infoType histogram (the only collective), takes the max-over-ranks time and verifies the reduced
histogram against an all-gather of the ranks' own counts.  The per-rank engine is an oracle-backed
double (this tests the rank logic, not the kernels; the kernels' histogram is tested on the GPU in
test_gpu_parity.py::test_histogram_matches_spans)."""
import argparse
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as tmp

from conftest import ROOT, pkg


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ARGS = dict(conversations=6, utt_per_conv=10, bank=200, steps=2, warmup=1)


def _shard_rows(rank, C, U, bank_n):
    synth = pkg("synth")
    bank = synth.build_bank(bank_n, bank_n, seed=synth.SEED)
    meta = synth.corpus_meta(C, U, bank, seed=synth.SEED, conv_base=rank * C)
    data = synth.gather_bytes(meta, bank)
    o = meta.offsets
    return [(int(meta.conv_slot[i]), int(meta.role[i]), data[int(o[i]):int(o[i + 1])].tobytes(), int(meta.ts_us[i]))
            for i in range(meta.n)]


class OracleBenchEngine:
    """The engine surface bench.run_rank uses, with the oracle's results for the rank's shard."""

    def __init__(self, rows, cfg):
        from oracle import pii_oracle as O
        self.type_names = list(cfg.type_names)
        self.counts = np.zeros(len(self.type_names), dtype=np.uint64)
        self.h = np.zeros_like(self.counts)
        self.ob = self.ns = 0
        for red, fs, _, _ in O.process_rows(rows, cfg):
            self.ob += len(red)
            self.ns += len(fs)
            for f in fs:
                self.counts[f.type_id] += 1

    def histogram_reset(self):
        self.h[:] = 0

    def scan_redact_device(self, *a):
        self.h += self.counts

    scan_redact_device_ex = scan_redact_device

    def sync(self):
        return self.ob, self.ns, 0

    def histogram(self):
        return self.h.copy()

    def set_timing(self, level):
        self.timing = level

    def timings(self):
        return [0.1] * 5 + [0.5]

    def kernel_timings(self):
        return {"k_scan": 0.1, "k_redact": 0.1}

    def queue_sizes(self):
        return 0, 0

    def close(self):
        pass


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    from oracle import pii_oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = O.RuleConfig.load()
    args = argparse.Namespace(**ARGS)

    def make_engine(batch, bank, C):
        return OracleBenchEngine(_shard_rows(rank, C, args.utt_per_conv, args.bank), cfg)
    line = bench.run_rank(args, rank, world, torch.device("cpu"), make_engine, dist=dist)
    out[rank] = line
    dist.destroy_process_group()


def test_bench_rank_function_gloo_world2():
    from oracle import pii_oracle as O
    world = 2
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    line = out[0]
    assert out[1] is None
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["steps"] == ARGS["steps"]
    cfg = O.RuleConfig.load()
    want = np.zeros(len(cfg.type_names), dtype=np.int64)
    for rank in range(world):
        for _, fs, _, _ in O.process_rows(_shard_rows(rank, ARGS["conversations"], ARGS["utt_per_conv"],
                                                      ARGS["bank"]), cfg):
            for f in fs:
                want[f.type_id] += 1
    h = line["histogram"]
    assert h["verified"] is True and h["total_spans_last_step"] == int(want.sum())
    assert h["per_type"] == {cfg.type_names[t]: int(want[t]) for t in range(len(want)) if want[t]}
    # the two shards are different conversations: value counts both ranks' bytes
    assert line["config"]["bytes_per_gpu"] > 0 and line["value"] > 0


# ---------------------------------------------------------------- the cross-rank bookkeeping helper
def _reduce_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = 5
    local = np.zeros(T + 1, dtype=np.int64)
    local[:T] = np.arange(T) * (rank + 1)
    local[T] = local[:T].sum()
    # (config 4 stream_rank: per-rank input bytes are SUMMED, the wall time is the MAX over ranks)
    el, sums, red, ok = bench.reduce_over_ranks(dist, torch.device("cpu"), 1.0 + rank, local, [1000 * (rank + 1), 7])
    out[rank] = (el, sums, red.tolist(), ok)
    dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    """stream_rank / run_rank / config5 all end with bench.reduce_over_ranks: max-over-ranks time,
    summed per-rank totals (config 4's input bytes), the histogram all_reduce and its all_gather
    check."""
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_reduce_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        el, sums, red, ok = out[r]
        assert el == 2.0 and sums == [3000.0, 14.0] and ok
        assert red[:5] == [0, 3, 6, 9, 12] and red[5] == 30
    import bench
    el, sums, red, ok = bench.reduce_over_ranks(None, torch.device("cpu"), 3.0, np.array([1, 2, 3]), [5])
    assert el == 3.0 and sums == [5.0] and red.tolist() == [1, 2, 3] and ok


# ---------------------------------------------------------------- config 5's rank path
C5_ARGS = dict(conversations=4, utt_per_conv=6, bank=64, steps=1, warmup=1)


def _c5_worker(rank, world, port, path, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    from oracle import pii_oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rulegen, synth = pkg("rulegen"), pkg("synth")
    bank = rulegen.Config5().build_bank()
    cfg = O.RuleConfig.load(path)
    args = argparse.Namespace(**C5_ARGS)

    def make_engine(batch, bank_, C):
        meta = synth.corpus_meta(C, args.utt_per_conv, bank, seed=synth.SEED, conv_base=rank * C)
        data = synth.gather_bytes(meta, bank)
        o = meta.offsets
        rows = [(int(meta.conv_slot[i]), int(meta.role[i]), data[int(o[i]):int(o[i + 1])].tobytes(),
                 int(meta.ts_us[i])) for i in range(meta.n)]
        out[("rows", rank)] = rows
        return OracleBenchEngine(rows, cfg)
    out[rank] = bench.run_rank(args, rank, world, torch.device("cpu"), make_engine, dist=dist, bank=bank)
    dist.destroy_process_group()


def test_config5_rank_function_gloo_world2(tmp_path):
    """config5_main's rank path: bench.run_rank over the config-5 rule set (542 types) and config-5
    text at world size 2 -- shards, histogram all_reduce over all types, verification."""
    from oracle import pii_oracle as O
    rulegen = pkg("rulegen")
    path = str(tmp_path / "c5.json")
    rulegen.Config5().save(path)
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_c5_worker, args=(2, _free_port(), path, out), nprocs=2, join=True)
    line = out[0]
    assert out[1] is None and line["n_gpus"] == 2
    cfg = O.RuleConfig.load(path)
    want = np.zeros(len(cfg.type_names), dtype=np.int64)
    for rank in range(2):
        for _, fs, _, _ in O.process_rows(out[("rows", rank)], cfg):
            for f in fs:
                want[f.type_id] += 1
    h = line["histogram"]
    assert h["verified"] is True and h["total_spans_last_step"] == int(want.sum()) > 0
    assert h["per_type"] == {cfg.type_names[t]: int(want[t]) for t in range(len(want)) if want[t]}
