"""Config 2 at full size: the 10M-utterance, 1.21 GB batch the headline bench times, every row checked
against the oracle (the bench only checked error flags at this size).

The engine runs the batch once through the device API (exactly bench.DeviceBatch.run); the oracle
replays all 100k conversations (oracle.process_rows, the reference's two handlers in order) on a
pool of the host's CPU share.  The pool's workers are SPAWNED (fresh interpreters that never touched
HIP: this pytest process has initialised the GPU by the time these tests run) and read the corpus
through memory-mapped .npy files.  Both sides reduce each conversation to one digest over its
redacted bytes, its spans (16-byte pii_span records, utt = batch row) and its per-row context
(ctx_info), so 10M rows are compared without holding the oracle's output."""
import hashlib
import multiprocessing as mp
import os

import numpy as np
import pytest

from conftest import ROOT, pkg

pytestmark = pytest.mark.gpu

_W = {}


def _init_worker(paths):
    """spawned pool worker: the corpus arrays, memory-mapped (no copy per worker)"""
    for k, path in paths.items():
        _W[k] = np.load(path, mmap_mode="r") if path.endswith(".npy") else int(open(path).read())


def _spawn_pool(arrays, cores):
    """a pool of fresh interpreters over `arrays` (saved once as .npy files); returns (pool, tmpdir)"""
    import tempfile
    d = tempfile.mkdtemp(prefix="pii_fullsize_")
    paths = {}
    for k, v in arrays.items():
        if isinstance(v, int):
            paths[k] = os.path.join(d, k + ".int")
            open(paths[k], "w").write(str(v))
        else:
            paths[k] = os.path.join(d, k + ".npy")
            np.save(paths[k], np.ascontiguousarray(v))
    return mp.get_context("spawn").Pool(cores, initializer=_init_worker, initargs=(paths,)), d


def _digest(out: bytes, spans: bytes, ctx: bytes) -> bytes:
    h = hashlib.blake2b(digest_size=16)
    for part in (out, spans, ctx):
        h.update(len(part).to_bytes(8, "little"))
        h.update(part)
    return h.digest()


def _oracle_block(rng):
    from oracle import pii_oracle as O
    cfg = O.RuleConfig.load()
    groups = list(cfg.context_keywords.keys())
    d, o, role, conv, ts, U = (_W[k] for k in ("data", "offs", "role", "conv", "ts", "U"))
    E = pkg("engine")
    out = []
    for c in range(*rng):
        lo, hi = c * U, (c + 1) * U
        rows = [(int(conv[i]), int(role[i]), d[int(o[i]):int(o[i + 1])].tobytes(), int(ts[i])) for i in range(lo, hi)]
        res = O.process_rows(rows, cfg)
        red = b"".join(r[0] for r in res)
        recs = [(lo + k, f.start, f.end, f.type_id, f.likelihood, 0) for k, r in enumerate(res) for f in r[1]]
        sp = np.array(recs, dtype=E.SPAN_DTYPE).tobytes() if recs else b""
        ctx = np.array([groups.index(r[3]) if rows[k][1] == O.ROLE_AGENT and r[3] else
                        groups.index(r[2]) if rows[k][1] == O.ROLE_CUSTOMER and r[2] else -1
                        for k, r in enumerate(res)], dtype=np.int16).tobytes()
        out.append(_digest(red, sp, ctx))
    return rng[0], out


def test_config2_full_batch_every_row_vs_oracle():
    import sys
    import torch
    sys.path.insert(0, ROOT)
    import bench
    synth, E, C_ = pkg("synth"), pkg("engine"), pkg("compiler")
    dev = torch.device("cuda", 0)
    C, U = 100_000, 100
    bank = synth.build_bank(16384, 16384, seed=synth.SEED)
    B = bench.DeviceBatch(C, U, bank, 0, dev)
    eng = E.Engine(C_.compile_default().blob, device=0, n_conv_slots=C)
    B.run(eng)
    ob, ns, fl = eng.sync()
    assert fl == 0 and B.n == C * U
    out = B.out[:ob].cpu().numpy()
    oo = B.out_offs.cpu().numpy()
    sp = B.spans[:ns * 16].cpu().numpy().view(E.SPAN_DTYPE)
    ctx = B.ctx.cpu().numpy()
    eng.close()
    starts = np.searchsorted(sp["utt"], np.arange(0, C * U + 1, U))
    got = [_digest(out[int(oo[c * U]):int(oo[(c + 1) * U])].tobytes(),
                   sp[int(starts[c]):int(starts[c + 1])].tobytes(), ctx[c * U:(c + 1) * U].tobytes())
           for c in range(C)]
    # oracle: all conversations on a pool of spawned workers (see the module docstring)
    import shutil
    cores = bench.cpu_share()
    blocks = [(c, min(c + 250, C)) for c in range(0, C, 250)]
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
    assert ns > 1_000_000


def _oracle_window_block(rng):
    from oracle import pii_oracle as O
    cfg = O.RuleConfig.load()
    groups = list(cfg.context_keywords.keys())
    d, o, role, ts, U, N = (_W[k] for k in ("wdata", "woffs", "wrole", "wts", "wU", "wN"))
    out = []
    for c in range(*rng):
        rows = [(c, int(role[c * U + k]), d[int(o[c * U + k]):int(o[c * U + k + 1])].tobytes(), int(ts[c * U + k]))
                for k in range(U)]
        h = hashlib.blake2b(digest_size=16)
        for red, fs, et in O.process_window_rows(rows, cfg, n=N):
            h.update(len(red).to_bytes(8, "little") + red)
            h.update(repr([(f.start, f.end, f.type_id, f.likelihood) for f in fs]).encode())
            h.update(str(groups.index(et) if et else -1).encode())
        out.append(h.digest())
    return rng[0], out


def test_config3_window_rescan_100k_conversations_vs_oracle():
    """Config 3 at its full width: 100k concurrent conversations, one new utterance each per call,
    N = 5, 12 steps (the windows fill at step 5) -- every redacted window, its spans and context vs
    the oracle's full re-scan of each joined window (oracle.process_window_rows)."""
    import sys
    import torch  # noqa: F401
    sys.path.insert(0, ROOT)
    import bench
    synth, E, C_ = pkg("synth"), pkg("engine"), pkg("compiler")
    C, U, N = 100_000, 12, 5
    bank = synth.build_bank(16384, 16384, seed=synth.SEED)
    meta = synth.corpus_meta(C, U, bank, seed=synth.SEED + 3)        # conversation-major
    data = synth.gather_bytes(meta, bank)
    o = meta.offsets.astype(np.int64)
    eng = E.Engine(C_.compile_default().blob, device=0, n_conv_slots=C)
    eng.window_enable(N, 8192)
    hs = [hashlib.blake2b(digest_size=16) for _ in range(C)]
    for k in range(U):                                             # step k: utterance k of every conversation
        idx = np.arange(C) * U + k
        texts = [data[int(o[i]):int(o[i + 1])].tobytes() for i in idx]
        res = eng.rescan_window(texts, list(range(C)), meta.role[idx].tolist(), meta.ts_us[idx].tolist())
        su = res.spans["utt"].astype(np.int64)
        starts = np.searchsorted(su, np.arange(C + 1))
        for c in range(C):
            red = res.text(c)
            hs[c].update(len(red).to_bytes(8, "little") + red)
            s = res.spans[int(starts[c]):int(starts[c + 1])]
            hs[c].update(repr([(int(x["start"]), int(x["end"]), int(x["info_type"]), int(x["likelihood"]))
                               for x in s]).encode())
            hs[c].update(str(int(res.ctx_info[c])).encode())
    eng.close()
    got = [h.digest() for h in hs]
    import shutil
    blocks = [(c, min(c + 500, C)) for c in range(0, C, 500)]
    want = [None] * C
    pool, tmp = _spawn_pool(dict(wdata=data, woffs=o, wrole=meta.role, wts=meta.ts_us, wU=U, wN=N), bench.cpu_share())
    try:
        with pool:
            for c0, digs in pool.imap_unordered(_oracle_window_block, blocks):
                want[c0:c0 + len(digs)] = digs
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    bad = [c for c in range(C) if got[c] != want[c]]
    assert not bad, (len(bad), bad[:10])
