"""The multi-GPU path's collective code, executed on the real device under RCCL.

The 8-GPU scaling run belongs to the driver; what one GPU box can run is the RCCL backend itself:
``init_process_group("nccl")`` at world size 1 on ``cuda:0`` and every collective the bench and the
service issue (``bench.reduce_over_ranks``: max / sum ``all_reduce`` + histogram ``all_reduce`` +
``all_gather`` check; ``distributed.reduce_histogram``) on DEVICE tensors, against the engine's own
histogram of a batch checked against the oracle.  It runs in a fresh spawned child (its own HIP
context and RCCL communicator), so nothing of the pytest process's GPU state is shared.
"""
import multiprocessing as mp
import os
import socket

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(port: int, q) -> None:
    try:
        import sys

        for p in (ROOT, os.path.join(ROOT, "tests")):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        import importlib

        import numpy as np
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        dev = torch.device("cuda", 0)
        E = importlib.import_module("context-based-pii_amd.engine")
        C = importlib.import_module("context-based-pii_amd.compiler")
        D = importlib.import_module("context-based-pii_amd.distributed")
        import bench
        from oracle import pii_oracle as O

        comp = C.compile_default()
        eng = E.Engine(comp.blob, device=0, n_conv_slots=64)
        rc = O.RuleConfig.load()
        rows = [(0, O.ROLE_AGENT, b"Can I get the credit card number on file?", 0),
                (0, O.ROLE_CUSTOMER, b"Sure, it is 4141-1212-2323-5009 and my email is jane.doe@example.com", 1),
                (1, O.ROLE_AGENT, b"What is your phone number?", 2),
                (1, O.ROLE_CUSTOMER, b"Call me at (415) 555-0100 or 555-867-5309, ssn 123-45-6789", 3)] * 50
        rows = sorted(rows, key=lambda r: r[0])
        eng.histogram_reset()
        res = eng.scan_redact([t for _, _, t, _ in rows], [c for c, _, _, _ in rows], [r for _, r, _, _ in rows],
                              [s for _, _, _, s in rows])
        exp = O.process_rows(rows, rc)
        for i, (red, _, _, _) in enumerate(exp):
            assert res.text(i) == red, i
        T = len(eng.type_names)
        want = np.zeros(T + 1, dtype=np.int64)
        for _, fs, _, _ in exp:
            for f in fs:
                want[f.type_id] += 1
        want[T] = want[:T].sum()
        h = np.asarray(eng.histogram(), dtype=np.int64)
        hist = np.append(h, h.sum())                   # bench's u64[T+1] layout: last slot = span total
        assert (hist == want).all(), (hist.tolist(), want.tolist())
        el, sums, red_h, ok = bench.reduce_over_ranks(dist, dev, 1.25, hist, sums=(3.0, 4.0))
        assert ok and el == 1.25 and sums == [3.0, 4.0] and (red_h == want).all()
        r2 = D.reduce_histogram(hist)
        assert (np.asarray(r2) == want).all()
        t = torch.arange(8, dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert t.cpu().tolist() == list(range(8))
        backend = dist.get_backend()
        eng.close()
        dist.destroy_process_group()
        q.put(("ok", backend, int(want[T])))
    except BaseException as e:      # noqa: BLE001 - reported to the parent
        import traceback
        q.put(("err", repr(e), traceback.format_exc()))


def test_rccl_world1_device_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    p.join(150)
    if p.is_alive():
        p.kill()
        p.join()
        pytest.fail("RCCL child timed out")
    assert not q.empty(), f"RCCL child exited {p.exitcode} without a result"
    r = q.get()
    assert r[0] == "ok", r
    assert r[1] == "nccl"
    assert r[2] > 0
    print(f"RCCL world-1 collectives ok on cuda:0 ({r[2]} spans in the histogram)")
