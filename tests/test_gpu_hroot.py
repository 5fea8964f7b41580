"""The two-level directory root (wave_gpu.h HR: an LDS top level over HBM rows of root groups),
which documents past the LDS root's capacity replay with.  CRDT_FORCE_HBM_ROOT=1 puts every
document of an engine laid out while it is set on it, so parity cases run through it at small
sizes (row splits, inserts at row boundaries, the flat <-> two-level conversion at every launch),
bit-exact against the oracle.  (Past the LDS root for real: test_gpu_parity.py
test_kevin_debug_layout_two_level_root.)"""
import os

import pytest

pytestmark = pytest.mark.gpu

import test_gpu_edge as E  # noqa: E402
import test_gpu_parity as P  # noqa: E402


@pytest.fixture
def hroot():
    os.environ["CRDT_FORCE_HBM_ROOT"] = "1"
    yield
    del os.environ["CRDT_FORCE_HBM_ROOT"]


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
def test_traces_on_the_two_level_root(hroot, name):
    P.test_trace_local_exact(name)
    P.test_trace_remote_exact(name)
    P.test_trace_debug_layout(name)


def test_histories_on_the_two_level_root(hroot):
    P.test_concurrent_histories()
    P.test_generated_config4()
    P.test_concurrent_config5()
    P.test_config1_every_op_probed(4)
    E.test_tables_grow_during_replay()
    E.test_fit_then_replay()
