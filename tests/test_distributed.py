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


# ---------------------------------------------------------------- string conversation ids, service level
def _svc_worker(rank, world, port, payloads, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from test_service import Clock, OracleEngine
    from oracle import pii_oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D, S = pkg("distributed"), pkg("service")
    cfg = O.RuleConfig.load()
    mine = [p for p in payloads if D.shard_of(p["conversation_id"], world) == rank]
    svc = S.PiiService(engine=OracleEngine(cfg, n_slots=8), clock=Clock(), time_base="payload")
    res = svc.process_pubsub_batch(mine)
    h = np.zeros(len(cfg.type_names) + 1, dtype=np.int64)
    for r in res:
        red, fs = O.redact(r["original_text"].encode(), cfg, None)
        h[-1] += 1
    out[rank] = (res, D.reduce_histogram(h).tolist())
    dist.destroy_process_group()


def test_string_conversation_ids_shard_and_match_one_process():
    """Config 4's sharding with the reference's string conversation ids (UUID-like, e2e_test.py): every
    rank serves the conversations shard_of() gives it with its own service and context table; the
    union of the ranks' redacted payloads equals one process serving everything, and the all_reduce
    sees every row exactly once."""
    import json
    import random
    from oracle import pii_oracle as O
    S = pkg("service")
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "transcripts.json")))
    pay = []
    for k in range(6):
        for name, t in tr.items():
            cid = f"conv-{k:02d}-{t['conversation_id']}"
            for e in t["entries"]:
                pay.append({"conversation_id": cid, "original_entry_index": e["i"], "participant_role": e["role"],
                            "text": e["text"], "user_id": "u", "start_timestamp_usec": e["ts"]})
    random.Random(3).shuffle(pay)
    D = pkg("distributed")
    assert {D.shard_of(p["conversation_id"], 2) for p in pay} == {0, 1}
    mgr = tmp.Manager()
    out = mgr.dict()
    tmp.spawn(_svc_worker, args=(2, _free_port(), pay, out), nprocs=2, join=True)
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_service import Clock, OracleEngine
    one = S.PiiService(engine=OracleEngine(O.RuleConfig.load(), n_slots=8), clock=Clock(), time_base="payload")
    want = {(r["conversation_id"], r["original_entry_index"]): r for r in one.process_pubsub_batch(pay)}
    got = {}
    for rank in range(2):
        res, h = out[rank]
        assert h[-1] == len(pay)
        for r in res:
            got[(r["conversation_id"], r["original_entry_index"])] = r
    assert got == want
