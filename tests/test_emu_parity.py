"""CPU-only: the product's replay core (replay_core.h), run through the test-only CPU emulation
backend, must reproduce the oracle exactly (entry layout included)."""
import numpy as np
import pytest

from emu_lib import EmuDoc, diff_states
from oracle_lib import OracleDoc
from crdt_amd.traces import load_trace, load_remote_wire
from fuzz_gen import random_local_trace, concurrent_wire


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
@pytest.mark.parametrize("L", [32, 4])
def test_traces(name, L):
    if name == "automerge-paper" and L == 4:
        pytest.skip("debug layout of automerge-paper needs 25,855 leaves > root capacity (8,160)")
    t = load_trace(name)
    o = OracleDoc(L, 16 if L == 32 else 8)
    o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
    e = EmuDoc(L)
    assert e.run_local(e.agent("jeremy"), t.counts, t.patches, 48 if L == 32 else 4) == 0
    assert e.check() == ""
    assert diff_states(o.export(), e.export()) == []
    r = EmuDoc(L)
    assert r.run_wire(load_remote_wire(name), 64) == 0
    assert diff_states(o.export(), r.export()) == []


@pytest.mark.parametrize("seed", range(8))
def test_random_local(seed):
    c, p = random_local_trace(seed, 4000, ins_max=1 + seed % 4)
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_trace(o.agent("x"), c, p) == 0
        e = EmuDoc(L)
        assert e.run_local(e.agent("x"), c, p, 200) == 0  # tight leaf cap: exercises growth/resume
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("seed", range(12))
def test_concurrent(seed):
    w, n = concurrent_wire(seed, n_agents=2 + seed % 3, rounds=4 + seed % 3)
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        so = o.apply_remote_wire(w)
        e = EmuDoc(L)
        se = e.run_wire(w, 48)
        assert so == se, (so, se)
        if so == 0:
            assert e.check() == ""
            assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("seed", range(6))
def test_generated_config4(seed):
    # BASELINE config 4 generator (make_random_change, doc.rs:544-569) expanded inside the replay
    # loop from one GEN record; the oracle draws the same ops (crdt_oracle.hpp random_change).
    n_ops = 3000 + 500 * seed
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_random(o.agent("gen"), n_ops, 0x9E3779B9 * (seed + 1)) == 0
        e = EmuDoc(L)
        assert e.run_random(e.agent("gen"), n_ops, 0x9E3779B9 * (seed + 1), 400) == 0  # tight caps: growth
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("seed", range(6))
def test_concurrent_config5(seed):
    # BASELINE config 5 shape (16 agents, deletion-heavy, hotspot ties, double deletes)
    from fuzz_gen import config5_wire
    w = config5_wire(seed, base_len=3000, rounds=6, ops=4)
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_remote_wire(w) == 0
        assert o.sizes()["dd"] > 0
        e = EmuDoc(L)
        assert e.run_wire(w, 48) == 0
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []
