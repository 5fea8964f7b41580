"""GPU parity: the HIP engine (through the C ABI) against the oracle, bit-exact.

Compared per document: raw entry layout + leaf boundaries (the reference's release B-tree leaves),
canonical spans, client_with_order, deletes, double deletes, txns + parents, frontier, len,
the 64-bit digest, and every pos->loc / loc->pos answer.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire, load_trace  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402
from fuzz_gen import random_local_trace  # noqa: E402
import sys, os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # bench helpers

KEYS = ("raw", "leaf_sizes", "canon", "cwo", "deletes", "dd", "txns", "parents", "frontier", "len", "next_order")


def assert_same(g, o, keys=KEYS):
    for k in keys:
        x, y = g[k], o[k]
        if isinstance(x, np.ndarray):
            assert x.shape == y.shape, (k, x.shape, y.shape)
            if not np.array_equal(x, y):
                i = int(np.argwhere(x != y)[0][0])
                raise AssertionError(f"{k} differs at {i}: gpu {x[i]} oracle {y[i]}")
        else:
            assert x == y, (k, x, y)


def check_queries(e, doc, o):
    n = len(o)
    pos = np.arange(n + 2, dtype=np.uint32)
    ga, gs = e.pos_to_loc(np.full(pos.shape, doc, np.uint32), pos)
    oa, os_ = o.pos_to_loc(pos)
    assert np.array_equal(ga, oa) and np.array_equal(gs, os_)
    s = o.sizes()
    for a in range(s["agents"]):
        seq = np.arange(s["next_order"] + 1, dtype=np.uint32)
        ag = np.full(seq.shape, a, np.uint16)
        gp, gd = e.loc_to_pos(np.full(seq.shape, doc, np.uint32), ag, seq)
        op, od = o.loc_to_pos(ag, seq)
        assert np.array_equal(gd, od)
        assert np.array_equal(gp[od != 2], op[od != 2])


def check_queries_sampled(e, doc, o, n=1 << 18, seed=5):
    """check_queries for large documents: n random positions (plus both ends) and n random
    (agent, seq) pairs over every agent's seq range, against the oracle."""
    rng = np.random.default_rng(seed)
    ln = len(o)
    pos = np.concatenate([rng.integers(0, ln + 2, n), [0, max(ln - 1, 0), ln, ln + 1]]).astype(np.uint32)
    ga, gs = e.pos_to_loc(np.full(pos.shape, doc, np.uint32), pos)
    oa, os_ = o.pos_to_loc(pos)
    assert np.array_equal(ga, oa) and np.array_equal(gs, os_)
    s = o.sizes()
    ag = rng.integers(0, s["agents"], n).astype(np.uint16)
    seq = rng.integers(0, s["next_order"] + 1, n).astype(np.uint32)
    gp, gd = e.loc_to_pos(np.full(seq.shape, doc, np.uint32), ag, seq)
    op, od = o.loc_to_pos(ag, seq)
    assert np.array_equal(gd, od)
    assert np.array_equal(gp[od != 2], op[od != 2])


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
def test_trace_local_exact(name):
    t = load_trace(name)
    e = crdt_amd.Engine(1, 32)
    a = e.agent_intern([0], ["jeremy"])
    st = e.apply_trace([0], int(a[0]), t.counts, t.patches)
    assert st[0] == 0
    o = OracleDoc(32, 16)
    o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
    assert_same(e.export(0), o.export())
    assert int(e.digests()[0]) == o.digest()
    assert int(e.lens()[0]) == t.end_len
    check_queries(e, 0, o)


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
def test_trace_remote_exact(name):
    w = load_remote_wire(name)
    e = crdt_amd.Engine(2, 32)
    st = e.apply_remote_wire([0, 1], [w, w])
    assert (st == 0).all()
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(w) == 0
    for d in (0, 1):
        assert_same(e.export(d), o.export())
    assert (e.digests() == np.uint64(o.digest())).all()
    check_queries(e, 1, o)
    check_query_fixtures(e, 0, name)


def check_query_fixtures(e, doc, name):
    """The engine's pos -> loc and loc -> pos answers against the committed fixtures
    (tests/golden/make_queries.py; the oracle's answers, pinned in tests/test_oracle.py)."""
    from bench import golden_pos_seq, golden_seq_pos
    if name == "automerge-paper":
        gseq = golden_pos_seq(name)
        ga, gs = e.pos_to_loc(np.full(gseq.shape, doc, np.uint32), np.arange(gseq.shape[0], dtype=np.uint32))
        assert (ga == 0).all() and np.array_equal(gs, gseq)
        gp, gd = golden_seq_pos(name)
        seq = np.arange(gp.shape[0], dtype=np.uint32)
        p, d = e.loc_to_pos(np.full(seq.shape, doc, np.uint32), np.zeros(seq.shape, np.uint16), seq)
        assert np.array_equal(d, gd) and np.array_equal(p[d != 2], gp[d != 2])
        return
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"queries_{name}.npz"))
    a, s = e.pos_to_loc(np.full(z["pos"].shape, doc, np.uint32), z["pos"])
    assert np.array_equal(a, z["pos_agent"]) and np.array_equal(s, z["pos_seq"])
    p, d = e.loc_to_pos(np.full(z["loc_seq"].shape, doc, np.uint32), z["loc_agent"], z["loc_seq"])
    assert np.array_equal(d, z["loc_deleted"]) and np.array_equal(p[d != 2], z["loc_pos"][d != 2])


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
def test_trace_debug_layout(name):
    # automerge-paper at leaf 4 needs ~25,900 leaves: past round 1's 8,160-leaf directory
    t = load_trace(name)
    e = crdt_amd.Engine(1, 4)
    a = e.agent_intern([0], ["jeremy"])
    assert e.apply_trace([0], int(a[0]), t.counts, t.patches)[0] == 0
    o = OracleDoc(4, 8)
    o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
    assert_same(e.export(0), o.export())


def test_mixed_corpus_and_random():
    # documents with different traces and random edit streams in one launch (segmented work)
    names = ["sveltecomponent", "rustcode", "automerge-paper"]
    traces = [load_trace(n) for n in names]
    rnd = [random_local_trace(1000 + i, 3000) for i in range(5)]
    docs = [(t.counts, t.patches) for t in traces] + rnd
    e = crdt_amd.Engine(len(docs), 32)
    ag = e.agent_intern(list(range(len(docs))), ["jeremy"] * len(docs))
    per_doc = []
    for i, (c, p) in enumerate(docs):
        off = np.concatenate([[0], np.cumsum(c)]).astype(int)
        per_doc.append((i, [(int(ag[i]), p[off[k]:off[k + 1]]) for k in range(len(c))]))
    st = e.apply_local(per_doc)
    assert (st == 0).all(), st
    dg = e.digests()
    for i, (c, p) in enumerate(docs):
        o = OracleDoc()
        o.apply_trace(o.agent("jeremy"), c, p)
        assert int(dg[i]) == o.digest(), i
        if i >= 3:
            assert_same(e.export(i), o.export())


def test_reference_unit_cases():
    from test_oracle import wire, ROOT_ID
    # remote_txns (doc.rs:620-676)
    e = crdt_amd.Engine(2, 4)
    w1 = wire([("seph", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)])])
    w2 = wire([("seph", 2, [("seph", 1)], [("del", ("seph", 0), 2)])])
    assert e.apply_remote_wire([0], [w1])[0] == 0
    assert e.apply_remote_wire([0], [w2])[0] == 0
    o = OracleDoc(4, 8)
    o.apply_remote_wire(w1)
    o.apply_remote_wire(w2)
    assert_same(e.export(0), o.export())
    # smoke (doc.rs:522-532) + deletes_merged (doc.rs:589-601) on doc 1, several apply calls
    a = int(e.agent_intern([1], ["seph"])[0])
    for ops in ([(0, 0, 2)], [(1, 0, 4)], [(0, 3, 0)], [(0, 0, 3)], [(0, 1, 0)], [(0, 1, 0)], [(0, 1, 0)]):
        assert e.apply_local([(1, [(a, ops)])])[0] == 0
    o = OracleDoc(4, 8)
    oa = o.agent("seph")
    for ops in ([(0, 0, 2)], [(1, 0, 4)], [(0, 3, 0)], [(0, 0, 3)], [(0, 1, 0)], [(0, 1, 0)], [(0, 1, 0)]):
        o.apply_local(oa, ops)
    assert_same(e.export(1), o.export())


def test_error_statuses_match():
    from test_oracle import wire, ROOT_ID
    cases = [
        wire([("seph", 1, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 1)])]),                     # SEQ
        wire([("A", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)]),
              ("B", 0, [("A", 0)], [("ins", ("A", 0), ROOT_ID, 1)])]),                        # NONTERMINATING
        wire([("A", 0, [ROOT_ID], [("ins", ("Z", 0), ROOT_ID, 1)])]),                         # UNKNOWN_AGENT
        wire([("A", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)]),
              ("A", 2, [("A", 1)], [("del", ("A", 7), 1)])]),                                 # UNKNOWN_ID
    ]
    e = crdt_amd.Engine(len(cases), 32)
    st = e.apply_remote_wire(list(range(len(cases))), cases)
    exp = []
    for w in cases:
        o = OracleDoc()
        exp.append(o.apply_remote_wire(w))
    assert list(st) == exp, (list(st), exp)
    assert exp == [-2, -5, -3, -4]


def test_concurrent_histories():
    from fuzz_gen import concurrent_wire
    wires = [concurrent_wire(s, n_agents=3, rounds=5)[0] for s in range(6)]
    e = crdt_amd.Engine(len(wires), 32)
    st = e.apply_remote_wire(list(range(len(wires))), wires)
    dg = e.digests()
    for i, w in enumerate(wires):
        o = OracleDoc()
        so = o.apply_remote_wire(w)
        assert st[i] == so, (i, st[i], so)
        if so == 0:
            assert int(dg[i]) == o.digest()
            assert_same(e.export(i), o.export())


def _seed32(seed, doc):
    from bench import splitmix64
    return splitmix64(seed ^ doc) & 0xFFFFFFFF


def test_generated_config4():
    # BASELINE config 4 shape: every document's edit stream is generated on the device from one
    # GEN record (make_random_change semantics, doc.rs:544-569), 20,000 ops per document.
    n_docs, n_ops, seed = 96, 20000, 0xC0FFEE
    e = crdt_amd.Engine(n_docs, 32)
    st = e.apply_random(list(range(n_docs)), "gen", n_ops, seed)
    assert (st == 0).all(), st
    dg = e.digests()
    for d in range(n_docs):
        o = OracleDoc()
        assert o.apply_random(o.agent("gen"), n_ops, _seed32(seed, d)) == 0
        assert int(dg[d]) == o.digest(), d
        if d < 3:
            assert_same(e.export(d), o.export())
            check_queries(e, d, o)


def test_concurrent_config5():
    # BASELINE config 5 shape at reduced scale: per document a 64k-char base by agent "base",
    # then 16 agents x 12 rounds x 4 concurrent txns (60 % deletes of 1..64 base items ->
    # double deletes, 40 % inserts at 32 shared hotspots -> integrate ties), seeded delivery.
    from fuzz_gen import config5_wire
    wires = [config5_wire(100 + s, base_len=65536, rounds=12, ops=4) for s in range(12)]
    e = crdt_amd.Engine(len(wires), 32)
    st = e.apply_remote_wire(list(range(len(wires))), wires)
    assert (st == 0).all(), st
    dg = e.digests()
    for i, w in enumerate(wires):
        o = OracleDoc()
        assert o.apply_remote_wire(w) == 0
        assert int(dg[i]) == o.digest(), i
        if i < 2:
            assert_same(e.export(i), o.export())
            check_queries(e, i, o)


def test_mixed_corpus_config3():
    # BASELINE config 3 shape: doc d replays [AP, RC, SV][splitmix64(d) % 3] (local txns), from
    # shared streams; every digest must equal the committed oracle golden digest of its trace.
    import json
    import os
    from bench import splitmix64
    names = ["automerge-paper", "rustcode", "sveltecomponent"]
    traces = [load_trace(n) for n in names]
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_golden.json")))
    n = 48
    which = [splitmix64(d) % 3 for d in range(n)]
    e = crdt_amd.Engine(n, 32)
    ag = e.agent_intern(list(range(n)), ["jeremy"] * n)
    e.stage_local_shared(list(range(n)), which, int(ag[0]), traces)
    st = e.run()
    assert (st == 0).all(), st
    dg = e.digests()
    for d in range(n):
        assert int(dg[d]) == int(gold[f"{names[which[d]]}/L32"]["digest"], 16), d


def test_kevin_prepends():
    # the reference's "kevin" benchmark shape (benches/yjs.rs:51-62), 1M single-char prepends at
    # position 0: 31,250 leaves at the release layout, 250,000 at the debug layout (an LDS root
    # class of its own, one wave per workgroup).  A small document in the same engine takes the
    # default root class: two replay launches from one run, with document lists.
    n = 1_000_000
    c = np.ones(n, np.uint32)
    p = np.zeros((n, 3), np.uint32)
    p[:, 2] = 1
    sv = load_trace("sveltecomponent")
    for L in (32, 4):
        e = crdt_amd.Engine(2, L)
        ag = e.agent_intern([0, 1], ["seph", "jeremy"])
        tx = np.concatenate([np.stack([np.full(n, ag[0]), c], 1),
                             np.stack([np.full(len(sv.counts), ag[1]), sv.counts], 1)]).astype(np.uint32)
        st = e.apply_local_arrays([0, 1], [0, n, n + len(sv.counts)], tx, np.concatenate([p, sv.patches]))
        assert (st == 0).all(), st
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_trace(o.agent("seph"), c, p) == 0
        assert_same(e.export(0), o.export())
        assert int(e.digests()[0]) == o.digest()
        o2 = OracleDoc(L, 16 if L == 32 else 8)
        assert o2.apply_trace(o2.agent("jeremy"), sv.counts, sv.patches) == 0
        assert int(e.digests()[1]) == o2.digest()
        check_queries_sampled(e, 0, o)


def test_config5_full_size():
    # BASELINE config 5 at its stated size: per document a 1M-char base by agent
    # "base", then 16 agents x 64 rounds x 64 concurrent txns = 65,536 remote txns (60 % deletes
    # of 1..64 base items -> double deletes, 40 % inserts at 32 shared hotspots -> integrate ties),
    # seeded delivery order.  Bit-exact against the oracle, at both layouts.
    from fuzz_gen import config5_wire
    wires = [config5_wire(900 + s, base_len=1 << 20, n_agents=16, rounds=64, ops=64) for s in range(4)]
    for L in (32, 4):
        e = crdt_amd.Engine(len(wires), L)
        st = e.apply_remote_wire(list(range(len(wires))), wires)
        assert (st == 0).all(), st
        dg = e.digests()
        for i, w in enumerate(wires):
            o = OracleDoc(L, 16 if L == 32 else 8)
            assert o.apply_remote_wire(w) == 0
            assert int(dg[i]) == o.digest(), (L, i)
            if i < 2:
                assert_same(e.export(i), o.export())
            if i == 0:
                check_queries_sampled(e, 0, o)


def test_config5_per_document_histories():
    # config 5's measured shape (scripts/bench_config5.py default): every document replays its own
    # seeded history (tests/gen/config5_gen.cpp: its own ops and delivery order) from its own record
    # copy, 96 documents in one launch at a reduced size; every digest against the oracle's replay
    # of that document's history, both layouts
    from fuzz_gen import config5_wires
    wires = config5_wires([0xC5100000 + s for s in range(96)], base_len=1 << 15, n_agents=16, rounds=8, ops=16,
                          threads=8)
    assert len({w for w in wires}) == len(wires)  # (distinct histories)
    odg = []
    for w in wires:
        o = OracleDoc(32, 16)
        assert o.apply_remote_wire(w) == 0
        odg.append(o.digest())
    for L in (32, 4):
        e = crdt_amd.Engine(len(wires), L)
        e.share_streams(False)
        st = e.apply_remote_wire(list(range(len(wires))), wires)
        assert (st == 0).all(), st
        dg = e.digests()
        if L == 32:
            assert [int(x) for x in dg] == odg
        else:
            for i in (0, 47, 95):
                o = OracleDoc(4, 8)
                assert o.apply_remote_wire(wires[i]) == 0
                assert int(dg[i]) == o.digest(), i
        e.close()


def test_wide_frontier_then_local():
    # frontier heads live in context lanes up to 25 heads (replay_core.h FR_S0), in HBM past that:
    # documents with 40 concurrent agents (frontiers to 41 heads, crossing both ways) and with 16
    # (always in the lanes), replayed as remote wires, then a second launch of local txns by a new
    # agent on every document (begin() reloads the heads; the local txn takes them as parents);
    # every digest and the first documents' whole state against the oracle, both layouts
    from fuzz_gen import config5_wire
    wires = [config5_wire(300 + s, base_len=4000, n_agents=40 if s % 2 else 16, rounds=5, ops=3) for s in range(8)]
    txs = [[5, 0, 3], [0, 2, 0]]
    for L in (32, 4):
        e = crdt_amd.Engine(len(wires), L)
        st = e.apply_remote_wire(list(range(len(wires))), wires)
        assert (st == 0).all(), st
        ids = e.agent_intern(list(range(len(wires))), ["local-editor"] * len(wires))
        st = e.apply_local([(d, [(int(ids[d]), [t]) for t in txs]) for d in range(len(wires))])
        assert (st == 0).all(), st
        dg = e.digests()
        for d, w in enumerate(wires):
            o = OracleDoc(L, 16 if L == 32 else 8)
            assert o.apply_remote_wire(w) == 0
            if d % 2:
                assert len(o.export()["frontier"]) > 25
            a = o.agent("local-editor")
            assert a == int(ids[d])
            for t in txs:
                assert o.apply_local(a, [t]) == 0
            assert int(dg[d]) == o.digest(), (L, d)
            if d < 2:
                assert_same(e.export(d), o.export())
        e.close()


@pytest.mark.parametrize("L", [32, 4])
def test_config1_every_op_probed(L):
    # BASELINE config 1 ("checking every position <-> CRDT-location lookup"): after EVERY txn of
    # automerge-paper (and rustcode), pos_to_loc(the op's position) and loc_to_pos(the txn's first
    # item) on the live state, in the replay kernel (PROBE records), against the oracle after the
    # same txn; a second pass probes random positions / earlier items instead
    from fuzz_gen import config1_probes
    names = ["automerge-paper", "rustcode"]
    traces = [load_trace(n) for n in names]
    for seed in (None, 11):
        e = crdt_amd.Engine(len(traces), L)
        ag = e.agent_intern(list(range(len(traces))), ["jeremy"] * len(traces))
        tx, ops, pr, off = [], [], [], [0]
        oans = []
        for d, t in enumerate(traces):
            tx.append(np.stack([np.full(len(t.counts), ag[d]), t.counts], 1))
            ops.append(t.patches)
            q = config1_probes(t.counts, t.patches, int(ag[d]), seed)
            pr.append(q)
            off.append(off[-1] + len(t.counts))
            o = OracleDoc(L, 16 if L == 32 else 8)
            so, a = o.probe_trace(o.agent("jeremy"), t.counts, t.patches, q)
            assert so == 0
            oans.append(a)
        st, ans = e.apply_local_probed(list(range(len(traces))), off, np.concatenate(tx), np.concatenate(ops),
                                       np.concatenate(pr))
        assert (st == 0).all(), st
        oans = np.concatenate(oans)
        bad = np.argwhere((ans != oans).any(1))
        assert bad.size == 0, (int(bad[0][0]), ans[bad[0][0]], oans[bad[0][0]])


def test_long_document_publish_chains():
    # Documents with >= 2048 leaves publish with a workgroup each (k_publish_big): the leaf
    # sequence is cut into 16 ranges and canonical spans crossing range boundaries are joined.
    # Forward-deleting a typed run leaves one deleted entry per item (split over thousands of
    # leaves) that all coalesce into ONE canonical span crossing every range; a second document
    # keeps a visible head and tail around the deleted middle.
    n = 200_000
    full = [(0, 0, n)] + [(0, 1, 0)] * n
    part = [(0, 0, n)] + [(1000, 1, 0)] * (n // 2) + [(n // 2, 0, 7)]
    for L in (32, 4):
        e = crdt_amd.Engine(2, L)
        ag = e.agent_intern([0, 1], ["f", "f"])
        per = [full, part]
        tx = np.concatenate([np.stack([np.full(len(t), ag[i]), np.ones(len(t))], 1) for i, t in enumerate(per)])
        st = e.apply_local_arrays([0, 1], [0, len(full), len(full) + len(part)], tx, np.concatenate([np.array(t) for t in per]))
        assert (st == 0).all(), st
        for i, ops in enumerate(per):
            o = OracleDoc(L, 16 if L == 32 else 8)
            a = o.agent("f")
            c = np.ones(len(ops), np.uint32)
            assert o.apply_trace(a, c, np.array(ops, np.uint32)) == 0
            assert o.sizes()["leaves"] >= 2048
            assert_same(e.export(i), o.export())
            assert int(e.digests()[i]) == o.digest()
            check_queries_sampled(e, i, o, n=1 << 14)
        assert e.export(0)["canon"].shape[0] <= 2


@pytest.mark.parametrize("mode", ["lds", "per_thread", "merge"])
def test_pos_to_loc_chunks_staged_and_mixed(mode):
    """pos -> loc answers of every query kernel family against the oracle (lds: k_pos_to_loc_blk,
    4,096-query chunks; a chunk of one document searches its visible prefix staged in LDS, any other
    chunk per thread in HBM; merge: k_pos_to_loc_merge, a sorted chunk merges against the visible
    prefix, others per thread): uniform chunks (sorted and unsorted), a chunk straddling two
    documents, interleaved documents and out-of-range positions / documents in one batch."""
    names = ["sveltecomponent", "rustcode", "automerge-paper"]
    e = crdt_amd.Engine(len(names), 32)
    e.query_kernel(mode)
    orc = []
    for d, name in enumerate(names):
        t = load_trace(name)
        a = e.agent_intern([d], ["jeremy"])
        assert e.apply_trace([d], int(a[0]), t.counts, t.patches)[0] == 0
        o = OracleDoc(32, 16)
        o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
        orc.append(o)
    rng = np.random.default_rng(11)
    lens = [len(o) for o in orc]
    # 2.5 uniform chunks of document 2, 1.5 of document 0 (a chunk straddles them), then mixed
    d_u = np.concatenate([np.full(10240, 2), np.full(6144, 0)])
    d_m = rng.integers(0, 4, 9000)  # document 3 does not exist
    docs = np.concatenate([d_u, d_m]).astype(np.uint32)
    pos = np.array([rng.integers(0, (lens[d] if d < 3 else 10) + 3) for d in docs], np.uint32)
    pos[:8192] = np.sort(pos[:8192])       # two sorted uniform chunks (the merge path), the
    pos[4096:8192] = np.sort(pos[4096:8192])  # second starting at its own minimum; then unsorted
    pos[100:110] = pos[100]  # (equal positions in a sorted chunk)
    ga, gs = e.pos_to_loc(docs, pos)
    for d in range(4):
        m = docs == d
        if d == 3:
            assert (ga[m] == 0xFFFF).all() and (gs[m] == 0xFFFFFFFF).all()
            continue
        oa, os_ = orc[d].pos_to_loc(pos[m])
        assert np.array_equal(ga[m], oa) and np.array_equal(gs[m], os_), d
    # loc -> pos through the same chunking (k_loc_to_pos_blk): staged and mixed chunks, unknown
    # agents / seqs / documents
    ag = rng.integers(0, 3, docs.shape[0]).astype(np.uint16)  # agent 0 is the only real one
    sq = np.array([rng.integers(0, (orc[d].sizes()["next_order"] if d < 3 else 10) + 3) for d in docs], np.uint32)
    gp, gd = e.loc_to_pos(docs, ag, sq)
    for d in range(4):
        m = docs == d
        if d == 3:
            assert (gd[m] == 2).all()
            continue
        op, od = orc[d].loc_to_pos(ag[m], sq[m])
        assert np.array_equal(gd[m], od), d
        assert np.array_equal(gp[m][od != 2], op[od != 2]), d


def test_kevin_reference_size():
    # The reference's own "kevin" benchmark at its size (benches/yjs.rs:51-62): 5,000,000
    # single-char local_insert(agent, 0, " ") on one document at the release layout: 5M entries in
    # 156,250 leaves.  Bit-exact raw layout + leaf boundaries, digest, sampled queries.
    n = 5_000_000
    c = np.ones(n, np.uint32)
    p = np.zeros((n, 3), np.uint32)
    p[:, 2] = 1
    e = crdt_amd.Engine(1, 32)
    ag = e.agent_intern([0], ["seph"])
    st = e.apply_local_arrays([0], [0, n], np.stack([np.full(n, ag[0]), c], 1).astype(np.uint32), p)
    assert st[0] == 0, st
    o = OracleDoc(32, 16)
    assert o.apply_trace(o.agent("seph"), c, p) == 0
    assert int(e.lens([0])[0]) == n == len(o)
    g = e.export(0)
    assert g["leaf_sizes"].shape[0] == 156_250
    assert_same(g, o.export())
    assert int(e.digests()[0]) == o.digest()
    check_queries_sampled(e, 0, o)


def test_kevin_debug_layout_two_level_root():
    # kevin at the reference size on the debug layout (leaf 4 / node 8): 1.25M leaves in about
    # 39k directory blocks, past the LDS root's 13,632 groups, so the document replays with the
    # two-level root (LDS top level over HBM rows of groups).  Bit-exact against the oracle.
    n = 5_000_000
    c = np.ones(n, np.uint32)
    p = np.zeros((n, 3), np.uint32)
    p[:, 2] = 1
    e = crdt_amd.Engine(1, 4)
    ag = e.agent_intern([0], ["seph"])
    st = e.apply_local_arrays([0], [0, n], np.stack([np.full(n, ag[0]), c], 1).astype(np.uint32), p)
    assert st[0] == 0, st
    o = OracleDoc(4, 8)
    assert o.apply_trace(o.agent("seph"), c, p) == 0
    g = e.export(0)
    assert g["leaf_sizes"].shape[0] == 1_250_000
    assert_same(g, o.export())
    assert int(e.digests()[0]) == o.digest()
    check_queries_sampled(e, 0, o)


@pytest.mark.parametrize("seed", range(3))
def test_front_runs_mixed(seed):
    # runs of local inserts at position 0 (leaf_insert_front's closed form: the prepends that fit
    # the first leaf in one lane-parallel write; the one that finds it full splits at index 0) of
    # 1-3 chars, broken by deletes at the front (the next run's origin_right is then a deleted item),
    # typing elsewhere, and runs longer than the record window -- bit-exact vs the oracle at both
    # layouts, with queries (tests/test_emu_parity.py runs the same shapes on the CPU emulation)
    rng = np.random.default_rng(100 + seed)
    counts, patches, ln = [], [], 0
    while len(counts) < 20000:
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
        e = crdt_amd.Engine(1, L)
        a = e.agent_intern([0], ["seph"])
        assert e.apply_trace([0], int(a[0]), c, p)[0] == 0
        o = OracleDoc(L, 16 if L == 32 else 8)
        assert o.apply_trace(o.agent("seph"), c, p) == 0
        assert_same(e.export(0), o.export())
        assert int(e.digests()[0]) == o.digest()
        check_queries_sampled(e, 0, o, n=1 << 14)
