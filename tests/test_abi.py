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


def test_codegen_guard_holds_for_the_built_library():
    # build() refuses a library whose replay kernel leaves the 8-waves/SIMD register budget
    # (<= 64 VGPRs, no spill written inside the replay loop): the built one passes, at both leaf
    # layouts and for every stream-shape instance (crdt_types.h SHAPE_*: all, remote, generated, local)
    crdt_amd.build()
    seen = crdt_amd.check_codegen(crdt_amd.LIB_PATH)
    replay = [r for n, r in seen.items() if "8k_replayI" in n]
    assert len(replay) == 2 * 4
    for r in replay:
        assert r["vgpr_count"] <= 64 and r.get("private_segment_fixed_size", 0) <= 32
    # (at most one spill slot, written outside the replay loop)
    ss = crdt_amd.scratch_stores(crdt_amd.LIB_PATH)
    assert all(n <= 4 for k, n in ss.items() if "8k_replayI" in k), ss


def test_codegen_guard_rejects_a_bloated_kernel(monkeypatch):
    res = crdt_amd.kernel_resources(crdt_amd.LIB_PATH)
    name = next(n for n in res if "8k_replayILi32E" in n)
    bad = dict(res)
    bad[name] = dict(res[name], vgpr_count=97)
    monkeypatch.setattr(crdt_amd, "kernel_resources", lambda p: bad)
    with pytest.raises(crdt_amd.CrdtError, match="vgpr_count = 97"):
        crdt_amd.check_codegen(crdt_amd.LIB_PATH)
    bad[name] = dict(res[name], private_segment_fixed_size=64)
    with pytest.raises(crdt_amd.CrdtError, match="private_segment_fixed_size"):
        crdt_amd.check_codegen(crdt_amd.LIB_PATH)
