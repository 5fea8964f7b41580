"""GPU edge cases (SURVEY §4 test strategy): empty and ragged batches, very long ops, many agents,
errors in the middle of a batch, documents that grow every table.  Each compares the HIP engine
(through the C ABI) with the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import crdt_amd  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402
from fuzz_gen import random_local_trace, concurrent_wire  # noqa: E402
from test_gpu_parity import assert_same, check_queries  # noqa: E402


def test_empty_and_ragged_batch():
    # documents with 0, 1, 2, 17, 3000 and 20000 ops in one launch (ragged work per wave)
    sizes = [0, 1, 2, 17, 3000, 20000]
    e = crdt_amd.Engine(len(sizes), 32)
    ag = e.agent_intern(list(range(len(sizes))), ["x"] * len(sizes))
    per_doc, oracles = [], []
    for i, n in enumerate(sizes):
        o = OracleDoc()
        a = o.agent("x")
        if n:
            c, p = random_local_trace(50 + i, n, ins_max=3)
            off = np.concatenate([[0], np.cumsum(c)]).astype(int)
            per_doc.append((i, [(int(ag[i]), p[off[k]:off[k + 1]]) for k in range(len(c))]))
            assert o.apply_trace(a, c, p) == 0
        oracles.append(o)
    st = e.apply_local(per_doc)
    assert (st == 0).all(), st
    dg = e.digests()
    for i, o in enumerate(oracles):
        assert int(dg[i]) == o.digest(), i
        assert int(e.lens()[i]) == len(o)
        assert_same(e.export(i), o.export())
    # a document that never saw an op answers queries like an empty ListCRDT
    ag_, sq = e.pos_to_loc(np.zeros(3, np.uint32), np.arange(3, dtype=np.uint32))
    assert (ag_ == 0xFFFF).all() and (sq == 0xFFFFFFFF).all()


def test_long_ops_take_the_general_path():
    # one 1,000,000-char insert, deletes of up to 70,000 chars, inserts of 65,536+ chars
    ops = [[(0, 0, 1_000_000)], [(123_456, 70_000, 0)], [(5, 0, 65_536)], [(900_000, 1, 70_001)],
           [(0, 500_000, 3)], [(10, 10, 10)]]
    e = crdt_amd.Engine(1, 32)
    a = int(e.agent_intern([0], ["big"])[0])
    st = e.apply_local([(0, [(a, o) for o in ops])])
    assert st[0] == 0
    o = OracleDoc()
    oa = o.agent("big")
    for op in ops:
        assert o.apply_local(oa, op) == 0
    assert_same(e.export(0), o.export())
    assert int(e.digests()[0]) == o.digest()


def test_many_agents_concurrent():
    # 40 concurrent agents: name ranks decide integrate ties (doc.rs:204-216)
    wires = [concurrent_wire(700 + s, n_agents=40, rounds=3, ops_per_round=2)[0] for s in range(3)]
    e = crdt_amd.Engine(len(wires), 32)
    st = e.apply_remote_wire(list(range(len(wires))), wires)
    for i, w in enumerate(wires):
        o = OracleDoc()
        so = o.apply_remote_wire(w)
        assert st[i] == so
        if so == 0:
            assert_same(e.export(i), o.export())
            check_queries(e, i, o)


def test_error_mid_batch_poisons_only_its_document():
    # doc 1's third txn deletes past the end (root.rs:160 panic in the reference): doc 1 stops
    # with POS_OOB; docs 0 and 2 finish and match the oracle; doc 1 skips its later txns
    good = [[(0, 0, 5)], [(2, 1, 0)], [(4, 0, 2)]]
    bad = [[(0, 0, 5)], [(2, 1, 0)], [(3, 5, 0)], [(0, 0, 1)]]
    e = crdt_amd.Engine(3, 32)
    ag = e.agent_intern([0, 1, 2], ["p"] * 3)
    st = e.apply_local([(0, [(int(ag[0]), o) for o in good]), (1, [(int(ag[1]), o) for o in bad]),
                        (2, [(int(ag[2]), o) for o in good])])
    assert list(st) == [0, -1, 0]
    o = OracleDoc()
    a = o.agent("p")
    for op in good:
        o.apply_local(a, op)
    dg = e.digests()
    assert int(dg[0]) == int(dg[2]) == o.digest()
    # the poisoned document accepts no further ops
    st2 = e.apply_local([(1, [(int(ag[1]), [(0, 0, 1)])])])
    assert st2[0] == -1


def test_tables_grow_during_replay():
    # 200 agents interleaving local txns on one document: every RLE table (client_with_order,
    # item_orders per agent, txns, deletes) outgrows its first capacity and resumes (ST_NEED_CAPACITY)
    rng = np.random.default_rng(3)
    e = crdt_amd.Engine(1, 32)
    names = [f"agent{i:03d}" for i in range(200)]
    ags = e.agent_intern([0] * len(names), names)
    o = OracleDoc()
    oags = [o.agent(n) for n in names]
    txns, n = [], 0
    for k in range(6000):
        i = int(rng.integers(len(names)))
        if n == 0 or rng.random() < 0.6:
            op = (int(rng.integers(n + 1)), 0, int(rng.integers(1, 4)))
            n += op[2]
        else:
            p = int(rng.integers(n))
            op = (p, int(rng.integers(1, min(6, n - p) + 1)), 0)
            n -= op[1]
        txns.append((int(ags[i]), [op]))
        assert o.apply_local(oags[i], [op]) == 0
    st = e.apply_local([(0, txns)])
    assert st[0] == 0
    assert_same(e.export(0), o.export())
    assert int(e.digests()[0]) == o.digest()


def test_republish_after_different_history():
    # k_publish writes span_of at item orders only; after a reset and a different history, the
    # entries it leaves at the new history's delete orders are stale and loc->pos must reject them
    import crdt_amd
    from crdt_amd.traces import load_trace
    from oracle_lib import OracleDoc
    A, B = load_trace("rustcode"), load_trace("sveltecomponent")
    cA, cB = A.counts[:6000], B.counts[:4000]
    pA, pB = A.patches[: int(cA.sum())], B.patches[: int(cB.sum())]
    e = crdt_amd.Engine(2, 32)
    ag = e.agent_intern([0, 1], ["jeremy"] * 2)
    assert (e.apply_trace([0, 1], int(ag[0]), cA, pA) == 0).all()
    nA = int(pA[:, 1].sum() + pA[:, 2].sum())
    e.loc_to_pos(np.zeros(nA, np.uint32), np.full(nA, ag[0], np.uint16), np.arange(nA, dtype=np.uint32))
    e.reset_async()
    assert (e.apply_trace([0, 1], int(ag[0]), cB, pB) == 0).all()
    o = OracleDoc(32, 16)
    oa = o.agent("jeremy")
    assert o.apply_trace(oa, cB, pB) == 0
    nB = int(pB[:, 1].sum() + pB[:, 2].sum())
    seqs = np.arange(nB + 64, dtype=np.uint32)
    op, odl = o.loc_to_pos(np.full(seqs.shape[0], oa, np.uint16), seqs)
    assert (odl == 2).any() and (odl == 1).any()        # delete-op seqs and deleted items both covered
    for d in (0, 1):
        gp, gdl = e.loc_to_pos(np.full(seqs.shape[0], d, np.uint32), np.full(seqs.shape[0], ag[d], np.uint16), seqs)
        assert np.array_equal(gdl, odl) and np.array_equal(gp, op)


def _wire_of_local(doc, agent, counts, patches):
    """the remote wire of `agent`'s local txns applied to oracle `doc` (and applies them)."""
    import ctypes as C
    from oracle_lib import lib, _p
    c = np.ascontiguousarray(counts, np.uint32)
    p = np.ascontiguousarray(patches, np.uint32)
    buf = C.create_string_buffer(64 << 20)
    n = lib().orc_local_trace_to_wire(doc.h, agent, c.shape[0], _p(c), _p(p), C.cast(buf, C.c_void_p), 64 << 20)
    assert n > 0
    return buf.raw[:n]


def test_local_document_starts_keeping_the_order_map():
    # Documents that only apply local txns keep no order -> leaf map (remote ops alone read it).
    # The first remote stream makes the engine rebuild it from the leaves: agent B's remote txns
    # then resolve their origins (A's items) through it.
    from crdt_amd.traces import load_trace
    sv = load_trace("sveltecomponent")
    cA, cB = sv.counts[:3000], sv.counts[3000:3600]
    pA = sv.patches[: int(cA.sum())]
    pB = sv.patches[int(cA.sum()): int(cA.sum()) + int(cB.sum())]
    o = OracleDoc()
    a = o.agent("A")
    assert o.apply_trace(a, cA, pA) == 0
    wB = _wire_of_local(o, o.agent("B"), cB, pB)
    e = crdt_amd.Engine(2, 32)
    ag = e.agent_intern([0, 1], ["A", "A"])
    assert (e.apply_trace([0, 1], int(ag[0]), cA, pA) == 0).all()
    st = e.apply_remote_wire([1], [wB])
    assert st[0] == 0
    assert_same(e.export(1), o.export())
    assert int(e.digests()[1]) == o.digest()
    check_queries(e, 1, o)
    # doc 0 stayed local-only and still matches its own history
    o0 = OracleDoc()
    o0.apply_trace(o0.agent("A"), cA, pA)
    assert int(e.digests()[0]) == o0.digest()


def test_fit_then_replay():
    # crdt_fit shrinks every capacity to the staged streams' use; a reset + replay of the same
    # streams then runs in exactly that room (no growth) and publishes the same state
    from crdt_amd.traces import load_trace, load_remote_wire
    w = load_remote_wire("sveltecomponent")
    t = load_trace("rustcode")
    e = crdt_amd.Engine(2, 32)
    assert e.apply_remote_wire([0], [w])[0] == 0
    dg0 = e.digests()
    b0 = e.mem_bytes()
    e.fit()
    assert e.mem_bytes() <= b0
    e.reset_async()
    e.run_async()
    e.sync()
    assert (e.status() == 0).all()
    assert (e.digests() == dg0).all()
    o = OracleDoc()
    o.apply_remote_wire(w)
    assert_same(e.export(0), o.export())
    check_queries(e, 0, o)
    # a new stream after a fit grows the capacities back
    ag = e.agent_intern([1], ["jeremy"])
    assert e.apply_trace([1], int(ag[0]), t.counts, t.patches)[0] == 0
    o2 = OracleDoc()
    o2.apply_trace(o2.agent("jeremy"), t.counts, t.patches)
    assert int(e.digests()[1]) == o2.digest()


def test_relayout_peak_memory():
    # layout() moves the pools one at a time (k_relayout_pool: allocate the new pool, move every
    # document's part, free the old one), so a growth relayout peaks at the old pools + the
    # largest new one -- below 1.3x the grown footprint -- and crdt_fit at the old pools + the
    # largest fitted one (both sets at once before)
    from crdt_amd.traces import load_trace
    t = load_trace("automerge-paper")
    n = 64
    e = crdt_amd.Engine(n, 32)
    ag = int(e.agent_intern(list(range(n)), ["jeremy"] * n)[0])
    half = t.counts.shape[0] // 2
    ph = int(t.counts[:half].sum())
    assert (e.apply_trace(list(range(n)), ag, t.counts[:half], t.patches[:ph]) == 0).all()
    crdt_amd.Engine.device_bytes(reset_peak=True)
    assert (e.apply_trace(list(range(n)), ag, t.counts[half:], t.patches[ph:]) == 0).all()
    grown, peak = crdt_amd.Engine.device_bytes()
    print(f"growth: footprint {grown / 1e6:.1f} MB, peak {peak / 1e6:.1f} MB ({peak / grown:.3f}x)")
    assert peak <= 1.3 * grown
    o = OracleDoc()
    o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
    assert (e.digests() == np.uint64(o.digest())).all()
    crdt_amd.Engine.device_bytes(reset_peak=True)
    e.fit()
    fitted, peak2 = crdt_amd.Engine.device_bytes()
    print(f"fit: footprint {grown / 1e6:.1f} -> {fitted / 1e6:.1f} MB, peak {peak2 / 1e6:.1f} MB ({peak2 / grown:.3f}x)")
    assert fitted <= grown and peak2 <= 1.5 * grown
    # the relocated state is the same state (a reset would replay only the last staged stream)
    assert (e.status() == 0).all() and (e.digests() == np.uint64(o.digest())).all()
    assert_same(e.export(n - 1), o.export())


def test_rejected_stage_leaves_agent_ids_unchanged():
    # a stage call that names a document twice is CRDT_E_ARG before any interning: the agent ids a
    # later valid call assigns follow the reference's get_or_create order (doc.rs:66-80) as if the
    # rejected call had not happened
    from crdt_amd.traces import load_remote_wire
    w = load_remote_wire("sveltecomponent")
    w2 = concurrent_wire(5, n_agents=4, rounds=3, ops_per_round=3)[0]
    e = crdt_amd.Engine(2, 32)
    with pytest.raises(crdt_amd.CrdtError):
        e.apply_remote_wire([1, 1], [w2, w])
    with pytest.raises(crdt_amd.CrdtError):
        e.stage_random([0, 0], "zz", 10, 1)
    assert e.apply_remote_wire([1], [w2])[0] == 0
    o = OracleDoc()
    assert o.apply_remote_wire(w2) == 0
    assert_same(e.export(1), o.export())
    assert int(e.digests()[1]) == o.digest()


def test_failed_relayout_poisons_the_engine():
    # a growth relayout that runs out of device memory after it began moving pools must
    # not leave a half-moved engine usable.  The k-th device allocation of a staging call that grows
    # every document is made to fail, for every k until the call no longer fails: either nothing
    # had moved yet (the engine keeps its state: same digests) or the engine is poisoned (every
    # later call but destroy / docs_alloc answers CRDT_E_NOMEM, and a fresh docs_alloc works).
    from crdt_amd.traces import load_trace
    t = load_trace("sveltecomponent")
    o = OracleDoc()
    o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
    L = crdt_amd.lib()
    h50 = int(t.counts[:50].sum())
    poisoned = intact = 0
    for k in range(64):
        e = crdt_amd.Engine(2, 32)
        ag = int(e.agent_intern([0, 1], ["jeremy"] * 2)[0])
        assert (e.apply_trace([0, 1], ag, t.counts[:50], t.patches[:h50]) == 0).all()
        d1 = e.digests()
        L.crdt_test_fail_alloc_after(k)
        try:
            e.apply_trace([0, 1], ag, t.counts[50:], t.patches[h50:], stage_only=True)
            failed = False
        except crdt_amd.CrdtError:
            failed = True
        finally:
            L.crdt_test_fail_alloc_after(-1)
        if not failed:
            e.close()
            break
        try:
            d = e.digests()
        except crdt_amd.CrdtError as x:
            assert "rc=-102" in str(x), x
            poisoned += 1
            with pytest.raises(crdt_amd.CrdtError, match="rc=-102"):
                e.run()
            with pytest.raises(crdt_amd.CrdtError, match="rc=-102"):
                e.pos_to_loc(np.zeros(1, np.uint32), np.zeros(1, np.uint32))
            # a fresh allocation of the documents makes the engine usable again
            assert L.crdt_docs_alloc(e.h, 1) == 0
            e.n_docs = 1
            ag = int(e.agent_intern([0], ["jeremy"])[0])
            assert e.apply_trace([0], ag, t.counts, t.patches)[0] == 0
            assert int(e.digests()[0]) == o.digest()
        else:
            intact += 1
            assert (d == d1).all(), k  # (failed before anything moved)
        e.close()
    else:
        raise AssertionError("every allocation of the staging call failed")
    assert poisoned >= 5, (poisoned, intact)  # (the relayout moves ~20 pools one at a time)


def test_config4_batches_reseed_and_fit_note():
    # bench.py --workload config4: one engine replays the batches of a larger corpus.  Documents
    # reseeded to corpus ids id_base + d replay exactly what stage_random gives those ids, the
    # capacities noted over every batch (fit_note) hold each batch without growth, and the
    # device digest copy equals crdt_digest.
    import torch
    n, ops, seed = 24, 3000, 0xC0FFEE
    big = crdt_amd.Engine(3 * n, 32)
    big.stage_random(list(range(3 * n)), "gen", ops, seed)
    assert (big.run() == 0).all()
    want = big.digests()
    e = crdt_amd.Engine(n, 32)
    e.stage_random(list(range(n)), "gen", ops, seed)
    for b in range(3):
        e.reseed_random_async(seed, b * n)
        e.reset_async()
        assert (e.run() == 0).all()
        e.publish_async()
        e.sync()
        assert (e.digests() == want[b * n:(b + 1) * n]).all(), b
        e.fit_note(False)
    e.fit_note(True)
    d = torch.zeros(n, dtype=torch.int64, device="cuda")
    for b in (2, 0, 1):
        e.reseed_random_async(seed, b * n)
        e.reset_async()
        e.run_async()
        e.publish_async()
        e.digests_dev_async(d.data_ptr())
        e.sync()
        assert (e.status() == 0).all()  # (no capacity stop: the noted maximum holds every batch)
        assert (d.cpu().numpy().view(np.uint64) == want[b * n:(b + 1) * n]).all(), b
    # the oracle agrees with a sampled corpus document (global id 2n + 5)
    o = OracleDoc(32, 16)
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import splitmix64
    assert o.apply_random(o.agent("gen"), ops, splitmix64(seed ^ (2 * n + 5)) & 0xFFFFFFFF) == 0
    assert int(want[2 * n + 5]) == o.digest()


def test_fitted_forward_delete_runs():
    # forward-delete runs (the delete key held down: data/micro/fd200, 200-delete runs at random
    # places of a 50,000-char document) replayed in fitted capacities (crdt_fit: the delete log's
    # room is the stream's own count) take the fast path's room check for one coalesced log run and
    # reach the same state as the oracle
    import gzip
    import os
    w = gzip.open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "micro", "fd200.rtx.gz"), "rb").read()
    o = OracleDoc()
    assert o.apply_remote_wire(w) == 0
    e = crdt_amd.Engine(4, 32)
    assert (e.apply_remote_wire([0, 1, 2, 3], [w] * 4) == 0).all()
    e.fit()
    e.reset_async()
    e.run_async()
    e.sync()
    assert (e.status() == 0).all()
    assert (e.digests() == np.uint64(o.digest())).all()
    assert_same(e.export(2), o.export())


def test_same_wire_staged_once_and_fit_keeps_exact_maps():
    # documents handed one wire buffer stage one host stream (crdt_stage_remote_wire), referenced
    # by one device copy with shared streams; crdt_fit sizes the order maps to next_order + 1 (a
    # replay from reset checks next_order + txn_len <= map_cap per txn), and a relayout leaves the
    # pools whose capacities did not change where they are.  Digests equal the oracle's before and
    # after the fit, and a replay of the fitted engine needs no growth.
    w, _ = concurrent_wire(11, n_agents=6, rounds=10, ops_per_round=6)
    o = OracleDoc()
    assert o.apply_remote_wire(w) == 0
    for share in (False, True):
        e = crdt_amd.Engine(6, 32)
        e.share_streams(share)
        assert (e.apply_remote_wire(list(range(6)), [w] * 6) == 0).all()
        assert (e.digests() == np.uint64(o.digest())).all()
        b0 = e.mem_bytes()
        e.fit()
        assert e.mem_bytes() <= b0
        for _ in range(2):
            e.reset_async()
            e.run_async()
            e.sync()
            assert (e.status() == 0).all()
            assert (e.digests() == np.uint64(o.digest())).all()
        assert_same(e.export(5), o.export())
        check_queries(e, 5, o)


def test_local_txn_parts():
    # replace ops and multi-op local txns replay as single-op parts on the fast paths: digests and
    # exports equal the oracle's one txn; a txn of only empty ops keeps its empty-txn status
    cases = [
        ([1, 2, 1, 3], [[0, 0, 5], [2, 1, 0], [1, 0, 2], [0, 2, 1], [1, 0, 0], [3, 1, 2], [0, 0, 0]]),
        ([2, 1], [[0, 0, 4], [1, 2, 3], [2, 1, 1]]),
        ([1, 1], [[0, 0, 3], [0, 0, 0]]),
    ]
    for counts, patches in cases:
        c = np.array(counts, np.uint32)
        p = np.array(patches, np.uint32)
        o = OracleDoc()
        so = o.apply_trace(o.agent("x"), c, p)
        e = crdt_amd.Engine(1, 32)
        ag = e.agent_intern([0], ["x"])
        st = e.apply_trace([0], int(ag[0]), c, p)
        assert int(st[0]) == so
        if so == 0:
            assert int(e.digests()[0]) == o.digest()
            assert_same(e.export(0), o.export())
