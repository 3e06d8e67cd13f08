"""The C ABI boundary (include/pii_engine.h) without a GPU: every declared symbol is exported by the
in-tree libpii.so, and the product path fails loudly (no CPU fallback) when no device is usable."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, pkg

HEADER = os.path.join(ROOT, "include", "pii_engine.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pii_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("pii_engine_create", "pii_scan_redact", "pii_scan_redact_device", "pii_context_get",
                 "pii_context_set", "pii_histogram"):
        assert must in names


def test_library_exports_every_declared_symbol():
    E = pkg("engine")
    lib = E.load_library()
    for name in declared():
        assert hasattr(lib, name), name
    assert set(declared()) <= set(E.EXPORTS)


def test_rejects_malformed_blob():
    E = pkg("engine")
    lib = E.load_library()
    h = ctypes.c_void_p()
    assert lib.pii_engine_create(b"not a blob", 10, 0, 4, 0, ctypes.byref(h)) == E.PII_E_RULES


def test_no_cpu_fallback_without_gpu(compiled):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    E = pkg("engine")
    with pytest.raises(E.PiiError) as ei:
        E.Engine(compiled.blob, device=0, n_conv_slots=4)
    assert ei.value.code == E.PII_E_DEVICE
