"""CPU-only: the product's replay core (replay_core.h), run through the test-only CPU emulation
backend, must reproduce the oracle exactly (entry layout included)."""
import os

import numpy as np
import pytest

from emu_lib import EmuDoc, diff_states
from oracle_lib import OracleDoc
from crdt_amd.traces import load_trace, load_remote_wire
from fuzz_gen import random_local_trace, concurrent_wire


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
@pytest.mark.parametrize("L", [32, 4])
def test_traces(name, L):
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


@pytest.mark.parametrize("L", [32, 4])
def test_kevin_prepends(L):
    # the reference's "kevin" benchmark shape (benches/yjs.rs:51-62): single-char prepends at
    # position 0, one unmergeable entry each.  200k prepends at leaf 4 = 50,000 leaves, past the
    # round-1 directory limit (8,160 leaves); tests/test_gpu_parity.py runs 1M on the GPU.
    n = 200_000
    c = np.ones(n, np.uint32)
    p = np.zeros((n, 3), np.uint32)
    p[:, 2] = 1
    o = OracleDoc(L, 16 if L == 32 else 8)
    assert o.apply_trace(o.agent("seph"), c, p) == 0
    e = EmuDoc(L)
    assert e.run_local(e.agent("seph"), c, p, 48 if L == 32 else 4) == 0
    assert e.check() == ""
    assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("seed", range(4))
def test_front_runs_mixed(seed):
    # runs of inserts at position 0 (replay_core.h front_run: closed form, leaf splits at index 0)
    # of 1-3 chars, broken by deletes at the front (the next run's origin_right is then a deleted
    # item, Q1), typing elsewhere and runs longer than the record window; tight leaf capacity so
    # runs stop for growth and resume
    rng = np.random.default_rng(seed)
    counts, patches, ln = [], [], 0
    while len(counts) < 6000:
        k, w = int(rng.integers(1, 150)), int(rng.integers(1, 4))
        for _ in range(k):
            counts.append(1); patches.append((0, 0, w)); ln += w
        r = rng.random()
        if r < 0.4 and ln > 3:
            d = int(rng.integers(1, 4))
            counts.append(1); patches.append((0, d, 0)); ln -= d
        elif r < 0.7:
            pos = int(rng.integers(0, ln + 1))
            for j in range(int(rng.integers(1, 6))):
                counts.append(1); patches.append((pos + j, 0, 1)); ln += 1
    c = np.array(counts, np.uint32)
    p = np.array(patches, np.uint32).reshape(-1, 3)
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_trace(o.agent("seph"), c, p) == 0
        e = EmuDoc(L)
        assert e.run_local(e.agent("seph"), c, p, 24 if L == 32 else 4) == 0
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("L", [32, 4])
def test_config5_full_size(L):
    # BASELINE config 5 at its stated size: a 1M-char base, 16 agents x 64 rounds x 64 txns
    # (65,536 remote txns); the frontier grows past its first capacity (16 heads), the debug
    # layout needs ~23k leaves.
    from fuzz_gen import config5_wire
    w = config5_wire(7, base_len=1 << 20, n_agents=16, rounds=64, ops=64)
    o = OracleDoc(L, 16 if L == 32 else 8)
    assert o.apply_remote_wire(w) == 0
    e = EmuDoc(L)
    assert e.run_wire(w, 48) == 0
    assert e.check() == ""
    assert diff_states(o.export(), e.export()) == []
    assert e.sizes()["frontier"] == 16 and e.sizes()["grow_mask"] & 128


def test_config5_generator_histories():
    # the C++ config-5 generator (tests/gen, scripts/bench_config5.py --distinct): every seed gives
    # its own causally ordered history (the oracle replays it with status OK), seeds differ, a seed
    # repeats exactly, and the replay core equals the oracle on small histories at both layouts and
    # on one history of SURVEY's full shape (1 M-char base, 16 agents x 64 rounds x 64 txns)
    from fuzz_gen import config5_wires
    ws = config5_wires([11, 12, 11], base_len=4096, n_agents=16, rounds=6, ops=4)
    assert ws[0] == ws[2] and ws[0] != ws[1]
    for w in ws[:2]:
        for L in (32, 4):
            o = OracleDoc(L, 16 if L == 32 else 8)
            assert o.apply_remote_wire(w) == 0
            e = EmuDoc(L)
            assert e.run_wire(w, 48) == 0
            assert e.check() == ""
            assert diff_states(o.export(), e.export()) == []
    w = config5_wires([5])[0]
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(w) == 0
    assert o.sizes()["dd"] > 0  # overlapping deletes made double deletes
    e = EmuDoc(32)
    assert e.run_wire(w, 48) == 0
    assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("name", ["sveltecomponent", "automerge-paper"])
@pytest.mark.parametrize("L", [32, 4])
def test_config1_probes(name, L):
    # BASELINE config 1: every txn of the trace followed by a pos->loc and a loc->pos query on the
    # live state (PROBE records), answered by the replay core like the oracle's count_pos
    from fuzz_gen import config1_probes
    t = load_trace(name)
    for seed in (None, 3):
        o = OracleDoc(L, 16 if L == 32 else 8)
        a = o.agent("jeremy")
        q = config1_probes(t.counts, t.patches, a, seed)
        so, oans = o.probe_trace(a, t.counts, t.patches, q)
        e = EmuDoc(L)
        se, eans = e.run_local_probed(e.agent("jeremy"), t.counts, t.patches, q, 48 if L == 32 else 4)
        assert so == se == 0
        bad = np.argwhere((eans != oans).any(1))
        assert bad.size == 0, (int(bad[0][0]), eans[bad[0][0]], oans[bad[0][0]])
        assert (oans[:, 3] != 2).any() and (oans[:, 3] == 2).any()


def test_config5_dd_top_level_threshold():
    # the double-delete directory's LDS top level covers 64 * DDT_LDS blocks; a document past that
    # searches the directory in HBM.  The emulator built with a one-word top level (64 blocks,
    # tests/emu/build/libemu_ddt1.so) replays a config-5 history whose directory crosses it
    # mid-replay: every top-level search is checked against the directory, and the state equals the
    # oracle's.
    import subprocess
    import sys
    import emu_lib
    emu_lib.build()
    code = (
        "import sys; sys.path[:0] = ['tests', 'text-crdt-rust_amd']\n"
        "from emu_lib import EmuDoc, diff_states\n"
        "from oracle_lib import OracleDoc\n"
        "from fuzz_gen import config5_wire\n"
        "w = config5_wire(3, base_len=1 << 16, n_agents=16, rounds=24, ops=32)\n"
        "o = OracleDoc(32, 16)\n"
        "assert o.apply_remote_wire(w) == 0\n"
        "e = EmuDoc(32)\n"
        "assert e.run_wire(w, 48) == 0\n"
        "assert e.check() == ''\n"
        "assert diff_states(o.export(), e.export()) == []\n"
        "print(o.sizes()['dd'])\n")
    env = dict(os.environ, CRDT_EMU_LIB=os.path.join(emu_lib.EMU_DIR, "build", "libemu_ddt1.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=emu_lib.ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert int(r.stdout.split()[-1]) > 64 * 64  # (more double-delete entries than 64 full blocks hold)


@pytest.mark.parametrize("L", [32, 4])
def test_local_txn_parts(L):
    # replace ops and multi-op local txns are encoded as single-op parts (host_plan.h
    # encode_local_txn): same state as the oracle's one txn, an empty op skipped, and a txn of only
    # empty ops keeps its empty-txn status
    cases = [
        ([1, 2, 1, 3], [[0, 0, 5], [2, 1, 0], [1, 0, 2], [0, 2, 1], [1, 0, 0], [3, 1, 2], [0, 0, 0]]),
        ([2, 1], [[0, 0, 4], [1, 2, 3], [2, 1, 1]]),
        ([1, 1], [[0, 0, 3], [0, 0, 0]]),
    ]
    for counts, patches in cases:
        c = np.array(counts, np.uint32)
        p = np.array(patches, np.uint32)
        o = OracleDoc(L, 16 if L == 32 else 8)
        so = o.apply_trace(o.agent("x"), c, p)
        e = EmuDoc(L)
        se = e.run_local(e.agent("x"), c, p, 48 if L == 32 else 4)
        assert se == so
        if so == 0:
            assert e.check() == ""
            assert diff_states(o.export(), e.export()) == []


@pytest.mark.parametrize("seed", range(4))
def test_wide_frontier(seed):
    # frontiers past the context lanes (replay_core.h FR_S0: heads 1..24 in lanes, more in HBM):
    # 40 concurrent agents grow the frontier to 41 heads and the round-start merges shrink it back,
    # so the heads cross between lanes and HBM both ways; local txns after the wire take the whole
    # frontier as their parents (heads -> parent pool); tight caps add capacity stops and resumes
    from fuzz_gen import config5_wire
    w = config5_wire(seed, base_len=4000, n_agents=40, rounds=5, ops=3)
    c = np.array([1, 1], np.uint32)
    pt = np.array([[5, 0, 3], [0, 2, 0]], np.uint32)
    for L in (32, 4):
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_remote_wire(w) == 0
        assert len(o.export()["frontier"]) > 25
        e = EmuDoc(L)
        assert e.run_wire(w, 48) == 0
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []
        assert o.apply_trace(o.agent("local-editor"), c, pt) == 0
        e = EmuDoc(L)
        assert e.run_wire_local(w, "local-editor", c, pt, 48) == 0
        assert e.check() == ""
        assert diff_states(o.export(), e.export()) == []
    # frontiers that stay within the lanes, then a local txn (config 5's 16 agents)
    w = config5_wire(seed, base_len=4000, n_agents=16, rounds=5, ops=3)
    o = OracleDoc()
    assert o.apply_remote_wire(w) == 0
    assert 2 <= len(o.export()["frontier"]) <= 25
    assert o.apply_trace(o.agent("local-editor"), c, pt) == 0
    e = EmuDoc(32)
    assert e.run_wire_local(w, "local-editor", c, pt, 48) == 0
    assert diff_states(o.export(), e.export()) == []
