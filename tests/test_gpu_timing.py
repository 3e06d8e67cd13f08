"""Timing levels (pii_set_timing): what a call records with HIP events, and that the level changes
nothing but the timings.

Level 2 records the stage boundaries (pii_last_timings [0..4], their sum as [5]); level 1 (the
default) only the call's start and end ([5]) and the events around the scan and redaction kernels
(pii_last_timings_ex); level 0 only the completion.  The redacted rows, spans and context must be the
same bytes at every level, and a level outside 0..2 is refused with PII_E_ARG."""
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu


def _rows():
    synth = pkg("synth")
    bank = synth.build_bank(400, 900, seed=41)
    corp = synth.make_corpus(300, 12, bank, seed=42)
    texts, slots, roles, ts = [], [], [], []
    for i in range(corp.n):
        a, b = int(corp.offsets[i]), int(corp.offsets[i + 1])
        texts.append(corp.data[a:b].tobytes())
        slots.append(int(corp.conv_slot[i]))
        roles.append(int(corp.role[i]))
        ts.append(int(corp.ts_us[i]))
    return texts, slots, roles, ts


def test_timing_levels_record_only_their_events(compiled):
    E = pkg("engine")
    texts, slots, roles, ts = _rows()
    got = {}
    for level in (2, 1, 0):
        eng = E.Engine(compiled.blob, device=0, n_conv_slots=4096)     # fresh context per level
        try:
            eng.set_timing(level)
            res = eng.scan_redact(texts, slots, roles, ts)
            got[level] = (res.out[:int(res.out_offsets[-1])].tobytes(), res.spans.tobytes(), res.ctx_info.tobytes(),
                          eng.timings(), eng.kernel_timings())
            with pytest.raises(E.PiiError):
                eng.set_timing(3)
        finally:
            eng.close()
    assert got[2][:3] == got[1][:3] == got[0][:3]
    st2, k2 = got[2][3], got[2][4]
    assert min(st2[:5]) >= 0 and sum(st2[:5]) > 0
    assert st2[5] == pytest.approx(sum(st2[:5]), rel=1e-4, abs=1e-4)
    assert k2["k_scan"] > 0 and k2["k_redact"] > 0
    st1, k1 = got[1][3], got[1][4]
    assert st1[:5] == [0.0] * 5 and st1[5] > 0
    assert k1["k_scan"] > 0 and k1["k_redact"] > 0
    st0, k0 = got[0][3], got[0][4]
    assert st0 == [0.0] * 6 and k0 == {"k_scan": 0.0, "k_redact": 0.0}
    assert np.isfinite(st1[5])
