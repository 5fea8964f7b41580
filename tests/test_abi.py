"""CPU-only checks of the C-ABI library: it loads, exports every symbol include/crdt_gpu.h and
include/crdt_trace.h declare,
and refuses to run without a gfx950 device (no silent CPU fallback)."""
import ctypes
import os
import re

import pytest

import crdt_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    h = "".join(open(os.path.join(ROOT, "include", f)).read() for f in ("crdt_gpu.h", "crdt_trace.h"))
    return sorted(set(re.findall(r"\b(crdt_[a-z_0-9]+)\s*\(", h)))


def test_header_matches_binding_list():
    assert sorted(crdt_amd.EXPORTED_SYMBOLS) == declared_symbols()


def test_library_exports_all_symbols():
    crdt_amd.build()
    lib = ctypes.CDLL(crdt_amd.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(crdt_amd.CrdtError):
        crdt_amd.Engine(1)
