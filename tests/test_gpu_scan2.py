"""The two-chain SCAN (k_scan2, PII_SCAN2=1: each lane split at one of its own utterance starts,
two interleaved DFA chains per thread; measured slower than k_scan and off by default)
against the oracle, at a size that takes its path (1 KiB lanes: a batch of >= 64 MiB).

6,000 conversations x 100 utterances of the config-2 distribution (~72 MB) run once through the device
API with PII_SCAN2=1; every conversation's redacted bytes, spans and per-row context are digested and
compared with oracle.process_rows on a pool of spawned workers (test_gpu_fullsize's harness)."""
import os
import shutil

import numpy as np
import pytest

from conftest import ROOT, pkg
from test_gpu_fullsize import _digest, _oracle_block, _spawn_pool

pytestmark = pytest.mark.gpu


def test_scan2_split_lanes_vs_oracle(monkeypatch):
    import sys
    import torch
    sys.path.insert(0, ROOT)
    import bench
    synth, E, C_ = pkg("synth"), pkg("engine"), pkg("compiler")
    monkeypatch.setenv("PII_SCAN2", "1")            # read by pii_engine_create
    dev = torch.device("cuda", 0)
    C, U = 6000, 100
    bank = synth.build_bank(16384, 16384, seed=synth.SEED)
    B = bench.DeviceBatch(C, U, bank, 0, dev)
    assert B.n_bytes >= 64 << 20                    # 1 KiB lanes (pick_lane_shift): the split path
    eng = E.Engine(C_.compile_default().blob, device=0, n_conv_slots=C)
    B.run(eng)
    ob, ns, fl = eng.sync()
    assert fl == 0
    out = B.out[:ob].cpu().numpy()
    oo = B.out_offs.cpu().numpy()
    sp = B.spans[:ns * 16].cpu().numpy().view(E.SPAN_DTYPE)
    ctx = B.ctx.cpu().numpy()
    eng.close()
    starts = np.searchsorted(sp["utt"], np.arange(0, C * U + 1, U))
    got = [_digest(out[int(oo[c * U]):int(oo[(c + 1) * U])].tobytes(),
                   sp[int(starts[c]):int(starts[c + 1])].tobytes(), ctx[c * U:(c + 1) * U].tobytes())
           for c in range(C)]
    cores = bench.cpu_share()
    blocks = [(c, min(c + 100, C)) for c in range(0, C, 100)]
    want = [None] * C
    pool, tmp = _spawn_pool(dict(data=B.text[:B.n_bytes].cpu().numpy(), offs=B.meta.offsets.astype(np.int64),
                                 role=B.meta.role, conv=B.meta.conv_slot, ts=B.meta.ts_us, U=U), cores)
    try:
        with pool:
            for c0, digs in pool.imap_unordered(_oracle_block, blocks):
                want[c0:c0 + len(digs)] = digs
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    bad = [c for c in range(C) if got[c] != want[c]]
    assert not bad, (len(bad), bad[:10])
    assert ns > 50_000
