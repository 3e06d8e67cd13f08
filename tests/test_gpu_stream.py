"""Config 4 ingest (stream.py): batches streamed through one engine with overlapped H2D / scan / D2H
give the same rows, spans and context as one big call and as the oracle; conversation-sharded
streams (one engine per shard, as one per GPU) reduce to the oracle's per-infoType histogram; the
declared-size entry point rejects a wrong declaration without committing anything."""
import numpy as np
import pytest

from conftest import pkg


def _stream_rows(n_conv, per, seed, conv_base=0):
    """step-major rows (every conversation's k-th utterance, then the (k+1)-th ...): a conversation's
    rows fall into many batches, so its context has to carry from batch to batch"""
    synth = pkg("synth")
    bank = synth.build_bank(2048, 2048, seed=seed)
    meta = synth.step_major(synth.corpus_meta(n_conv, per, bank, seed=seed, conv_base=conv_base), bank, n_conv, per)
    data = synth.gather_bytes(meta, bank)
    o = meta.offsets
    return [(int(meta.conv_slot[i]), int(meta.role[i]), data[int(o[i]):int(o[i + 1])].tobytes(), int(meta.ts_us[i]))
            for i in range(meta.n)]


def _batches(rows, batch_bytes, pin=False):
    S = pkg("stream")
    lens = np.array([len(r[2]) for r in rows], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [S.HostBatch.from_rows(rows[lo:hi], pin=pin) for lo, hi in S.split_batches(offs, batch_bytes)]


def test_split_batches_cpu():
    S = pkg("stream")
    offs = np.array([0, 10, 30, 31, 100, 101, 102], dtype=np.int64)
    b = S.split_batches(offs, 30)
    assert b == [(0, 2), (2, 3), (3, 4), (4, 6)]
    assert S.split_batches(offs, 1000, max_rows=4) == [(0, 4), (4, 6)]
    rows = [(1, 0, b"abc", 5), (2, 1, b"", 6), (3, 2, b"xy", 7)]
    hb = S.HostBatch.from_rows(rows)
    assert hb.n == 3 and hb.n_bytes == 5 and hb.rows() == rows
    rows = [(4, 1, b"a", 1), (2, 1, b"b", 2), (4, 0, b"c", 3), (2, 0, b"d", 4), (9, 2, b"e", 5)]
    hb = S.HostBatch.from_rows(rows)
    assert [r[2] for r in hb.rows()] == [b"b", b"d", b"a", b"c", b"e"]
    assert [rows[int(k)] for k in hb.perm] == hb.rows()


def _collect(ing, batches):
    """results in arrival order (each batch's rows were grouped by conversation: undo with perm)"""
    got = [None] * sum(b.n for b in batches)
    starts = np.concatenate([[0], np.cumsum([b.n for b in batches])])

    def consume(i, res):
        perm = batches[i].perm
        for k in range(len(res.out_offsets) - 1):
            m = res.spans["utt"] == k
            got[int(starts[i]) + (int(perm[k]) if perm is not None else k)] = (
                res.text(k), [(int(s["start"]), int(s["end"]), int(s["info_type"]), int(s["likelihood"]))
                              for s in res.spans[m]], int(res.ctx_info[k]))
    stats = ing.run(batches, consume)
    return got, stats


@pytest.fixture(scope="module")
def blob(compiled):
    return compiled.blob


@pytest.mark.gpu
@pytest.mark.parametrize("pin", [False, True])
def test_stream_equals_one_call_and_oracle(blob, oracle_cfg, pin):
    from oracle import pii_oracle as O
    E, S = pkg("engine"), pkg("stream")
    rows = _stream_rows(600, 24, 3)                     # 14.4k rows, ~1.7 MB
    batches = _batches(rows, 96 << 10, pin=pin)         # ~18 batches
    assert len(batches) > 8
    eng = E.Engine(blob, device=0, n_conv_slots=1 << 12)
    ing = S.StreamIngest(eng, max_bytes=max(b.n_bytes for b in batches), max_rows=max(b.n for b in batches))
    got, stats = _collect(ing, batches)
    assert stats["batches"] == len(batches) and stats["capacity_reruns"] == 0
    eng.close()
    # one call over the whole stream (grouped by conversation, as the batch contract wants)
    perm = np.argsort(np.array([r[0] for r in rows]), kind="stable")
    srows = [rows[int(k)] for k in perm]
    one = E.Engine(blob, device=0, n_conv_slots=1 << 12)
    res = one.scan_redact([r[2] for r in srows], [r[0] for r in srows], [r[1] for r in srows], [r[3] for r in srows])
    one.close()
    one_text, one_ctx = [None] * len(rows), [None] * len(rows)
    for j, k in enumerate(perm):
        one_text[int(k)], one_ctx[int(k)] = res.text(j), int(res.ctx_info[j])
    groups = list(oracle_cfg.context_keywords.keys())
    exp = O.process_rows(rows, oracle_cfg)
    for i, (red, fs, used, stored) in enumerate(exp):
        assert got[i][0] == one_text[i] == red, i
        assert got[i][1] == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i
        want_ctx = stored if rows[i][1] == O.ROLE_AGENT else used if rows[i][1] == O.ROLE_CUSTOMER else None
        assert got[i][2] == (groups.index(want_ctx) if want_ctx is not None else -1), i
        assert got[i][2] == one_ctx[i]


@pytest.mark.gpu
def test_stream_capacity_rerun(blob, oracle_cfg):
    """An output buffer too small for some batches: those are re-run with exact capacities (nothing
    was committed by the failed run), results unchanged."""
    from oracle import pii_oracle as O
    E, S = pkg("engine"), pkg("stream")
    rows = _stream_rows(200, 20, 5)
    batches = _batches(rows, 32 << 10)
    eng = E.Engine(blob, device=0, n_conv_slots=1 << 12)
    mb = max(b.n_bytes for b in batches)
    ing = S.StreamIngest(eng, max_bytes=mb, max_rows=max(b.n for b in batches), out_cap=mb - 4096, span_cap=64)
    got, stats = _collect(ing, batches)
    eng.close()
    assert stats["capacity_reruns"] > 0
    exp = O.process_rows(rows, oracle_cfg)
    for i, (red, fs, _, _) in enumerate(exp):
        assert got[i][0] == red and got[i][1] == [(f.start, f.end, f.type_id, f.likelihood) for f in fs], i


@pytest.mark.gpu
def test_sharded_streams_histogram(blob, oracle_cfg):
    """Two conversation shards streamed by two engines (one per GPU in config 4); the sum of their
    per-infoType histograms (what bench.py all-reduces over RCCL) equals the oracle's counts."""
    from oracle import pii_oracle as O
    E, S = pkg("engine"), pkg("stream")
    T = len(oracle_cfg.type_names)
    total = np.zeros(T, dtype=np.int64)
    want = np.zeros(T, dtype=np.int64)
    for rank in range(2):
        rows = _stream_rows(150, 20, 11 + rank, conv_base=rank * 150)
        eng = E.Engine(blob, device=0, n_conv_slots=1 << 10)
        eng.histogram_reset()
        batches = _batches(rows, 40 << 10)
        ing = S.StreamIngest(eng, max_bytes=max(b.n_bytes for b in batches), max_rows=max(b.n for b in batches))
        got, _ = _collect(ing, batches)
        total += eng.histogram().astype(np.int64)
        eng.close()
        for i, (red, fs, _, _) in enumerate(O.process_rows(rows, oracle_cfg)):
            assert got[i][0] == red, (rank, i)
            for f in fs:
                want[f.type_id] += 1
    assert (total == want).all() and want.sum() > 100


@pytest.mark.gpu
def test_declared_size_mismatch_is_rejected(blob):
    """pii_scan_redact_device_ex with a wrong batch size: pii_sync -> PII_E_ARG, the agent row's
    context is not stored; the same call declared correctly then stores it."""
    import torch
    E = pkg("engine")
    eng = E.Engine(blob, device=0, n_conv_slots=64)
    texts = [b"what is your date of birth?", b"sure"]
    data, offs = E.pack(texts)
    dev = torch.device("cuda", 0)
    d_text = torch.from_numpy(data.copy()).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_slot = torch.tensor([7, 7], dtype=torch.int32, device=dev)
    d_role = torch.tensor([E.ROLE_AGENT, E.ROLE_CUSTOMER], dtype=torch.uint8, device=dev)
    d_ts = torch.tensor([1_000_000, 2_000_000], dtype=torch.int64, device=dev)
    d_out = torch.empty(4096, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(3, dtype=torch.int64, device=dev)
    d_sp = torch.empty(64 * 16, dtype=torch.uint8, device=dev)
    d_ctx = torch.empty(2, dtype=torch.int16, device=dev)
    args = lambda nb: (d_text.data_ptr(), d_offs.data_ptr(), 2, 0, nb, d_slot.data_ptr(), d_role.data_ptr(),  # noqa
                       d_ts.data_ptr(), d_out.data_ptr(), 4096, d_oo.data_ptr(), d_sp.data_ptr(), 64, d_ctx.data_ptr())
    eng.scan_redact_device_ex(*args(int(offs[-1]) - 3))
    with pytest.raises(E.PiiError) as ei:
        eng.sync()
    assert ei.value.code == E.PII_E_ARG
    assert eng.context_get(7)[0] == -1
    eng.scan_redact_device_ex(*args(int(offs[-1])))
    ob, ns, fl = eng.sync()
    assert fl == 0 and ob == int(offs[-1])
    assert eng.group_types[eng.context_get(7)[0]] == "DATE_OF_BIRTH"
    eng.close()
