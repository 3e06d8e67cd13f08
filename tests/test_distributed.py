"""Conversation-sharded multi-rank path on CPU (gloo, world size 2): each rank owns the conversations
shard_of() assigns it, computes its per-infoType counts, and the one collective (an all-reduce of the
histogram) reproduces the single-process totals.  The per-rank engine is stood in for by the oracle
(this is a CPU test of the sharding and the reduction, not of the kernels)."""
import os
import socket

import numpy as np
import torch.multiprocessing as tmp

from conftest import ROOT, pkg


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hist(rows, cfg):
    from oracle import pii_oracle as O
    h = np.zeros(len(cfg.type_names) + 1, dtype=np.int64)
    for red, fs, _, _ in O.process_rows(rows, cfg):
        for f in fs:
            h[f.type_id] += 1
        h[-1] += len(fs)
    return h


def _rows():
    synth = pkg("synth")
    bank = synth.build_bank(200, 300, seed=4)
    corp = synth.make_corpus(24, 10, bank, seed=8)
    return [(int(corp.conv_slot[i]), int(corp.role[i]),
             corp.data[int(corp.offsets[i]):int(corp.offsets[i + 1])].tobytes(), int(corp.ts_us[i]))
            for i in range(corp.n)]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = pkg("distributed")
    from oracle import pii_oracle as O
    cfg = O.RuleConfig.load()
    rows = _rows()
    mine = D.shard_rows([r[0] for r in rows], rank, world)
    local = _hist([rows[i] for i in mine], cfg)
    total = D.reduce_histogram(local)
    out[rank] = (len(mine), total.tolist())
    dist.destroy_process_group()


def test_sharded_histogram_allreduce_gloo():
    from oracle import pii_oracle as O
    world = 2
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rows = _rows()
    full = _hist(rows, O.RuleConfig.load())
    assert out[0][0] + out[1][0] == len(rows) and out[0][0] > 0 and out[1][0] > 0
    assert out[0][1] == out[1][1] == full.tolist()


def test_shard_of_is_stable_and_balanced():
    D = pkg("distributed")
    ids = [f"sess_{i:05d}" for i in range(4000)]
    for world in (2, 4, 8):
        counts = np.bincount([D.shard_of(c, world) for c in ids], minlength=world)
        assert counts.min() > 0.8 * len(ids) / world
        assert [D.shard_of(c, world) for c in ids[:50]] == [D.shard_of(c, world) for c in ids[:50]]
