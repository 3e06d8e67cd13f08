"""Device-API calls whose per-row arrays are NOT 16-byte aligned (views one element into a tensor) and
whose row counts are not multiples of the kernels' row groups: the context kernels take their
scalar path, k_chunk_index its tail path.  Results must equal the aligned call's and the oracle's.
Also: the declared-size entry point, and the histogram copied with the call's totals after a
stream-ordered reset.  Needs an MI355X: pytest -m gpu."""
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu


def _run(compiled, corp, shift, declared):
    import torch
    E = pkg("engine")
    eng = E.Engine(compiled.blob, device=0, n_conv_slots=1 << 12)
    dev = torch.device("cuda:0")
    n = corp.n

    def place(arr, dtype):
        # the array `shift` elements into a larger device tensor: misaligned for shift > 0
        t = torch.zeros(len(arr) + shift + 8, dtype=dtype, device=dev)
        t[shift:shift + len(arr)] = torch.from_numpy(arr).to(dev)
        return t, t[shift:]

    _, d_text = place(corp.data, torch.uint8)
    _, d_offs = place(corp.offsets.view(np.int64), torch.int64)
    _, d_slot = place(corp.conv_slot.view(np.int32), torch.int32)
    _, d_role = place(corp.role, torch.uint8)
    _, d_ts = place(corp.ts_us, torch.int64)
    out_cap = int(corp.offsets[-1]) * 2 + 64 * n
    span_cap = n * 4
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sp = torch.empty(span_cap * 16, dtype=torch.uint8, device=dev)
    _, d_ctx = place(np.zeros(n, np.int16), torch.int16)
    eng.histogram_reset()
    args = (d_slot.data_ptr(), d_role.data_ptr(), d_ts.data_ptr(), d_out.data_ptr(), out_cap, d_oo.data_ptr(),
            d_sp.data_ptr(), span_cap, d_ctx.data_ptr())
    if declared:
        eng.scan_redact_device_ex(d_text.data_ptr(), d_offs.data_ptr(), n, int(corp.offsets[0]),
                                  int(corp.offsets[-1] - corp.offsets[0]), *args)
    else:
        eng.scan_redact_device(d_text.data_ptr(), d_offs.data_ptr(), n, *args)
    ob, ns, flags = eng.sync()
    assert flags == 0
    hist = eng.histogram()
    res = (d_out[:ob].cpu().numpy().tobytes(), d_oo.cpu().numpy(), d_sp[:ns * 16].cpu().numpy().tobytes(),
           d_ctx[:n].cpu().numpy(), hist)
    eng.close()
    return res


def test_misaligned_rows_match_aligned_and_oracle(compiled, oracle_cfg):
    from oracle import pii_oracle as O
    synth = pkg("synth")
    bank = synth.build_bank(600, 600, seed=7)
    corp = synth.make_corpus(263, 37, bank, seed=3)          # 9731 rows: not a multiple of 4 or 8
    a = _run(compiled, corp, 0, declared=True)
    b = _run(compiled, corp, 1, declared=False)
    assert a[0] == b[0]
    assert (a[1] == b[1]).all() and a[2] == b[2] and (a[3] == b[3]).all()
    assert (a[4] == b[4]).all()
    spans = np.frombuffer(b[2], dtype=pkg("engine").SPAN_DTYPE)
    want = np.bincount(spans["info_type"].astype(np.int64), minlength=len(b[4]))
    assert (b[4] == want[:len(b[4])]).all()                 # histogram copied with the totals
    rows = [(int(corp.conv_slot[i]), int(corp.role[i]),
             corp.data[int(corp.offsets[i]):int(corp.offsets[i + 1])].tobytes(), int(corp.ts_us[i]))
            for i in range(corp.n)]
    exp = O.process_rows(rows, oracle_cfg)
    oo = b[1]
    for i in range(0, corp.n, 7):
        assert b[0][int(oo[i]):int(oo[i + 1])] == exp[i][0], i
