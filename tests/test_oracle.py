"""Pin the oracle (CPU restatement) against the reference's own tests and fixtures.

CPU-only.  Each test names the reference test / assertion it ports.
"""
import json
import os
import random

import numpy as np
import pytest

from oracle_lib import OracleDoc, DoubleDeletes, OK, ERR_POS_OOB, ERR_SEQ, ERR_NONTERMINATING
from crdt_amd.traces import TRACE_NAMES, load_trace, load_remote_wire

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "oracle_golden.json")))
ROOT_ID = ("ROOT", 0xFFFFFFFF)


def wire(txns, names=None):
    """Build a wire batch from [(agent, seq, [parents], [ops])]; op = ('ins', ol, or, len) | ('del', id, len)."""
    import struct
    names = list(names or [])

    def ni(n):
        if n not in names:
            names.append(n)
        return names.index(n)

    body = []
    for agent, seq, parents, ops in txns:
        body += [ni(agent), seq, len(parents), len(ops)]
        for p in parents:
            body += [ni(p[0]), p[1]]
        for op in ops:
            if op[0] == "ins":
                body += [0, ni(op[1][0]), op[1][1], ni(op[2][0]), op[2][1], op[3]]
            else:
                body += [1, ni(op[1][0]), op[1][1], 0, 0, op[2]]
    out = struct.pack("<II", 0x31585452, len(names))
    for n in names:
        b = n.encode()
        out += struct.pack("<I", len(b)) + b + b"\0" * ((4 - len(b) % 4) % 4)
    out += struct.pack("<I", len(txns)) + np.array(body, dtype=np.uint32).tobytes()
    return out


# --- double_delete.rs:114-139 inc_delete_range (exact golden vectors) -------------------------
def test_inc_delete_range():
    d = DoubleDeletes()
    d.increment(5, 3)
    assert d.get() == [(5, 3, 1)]
    d.increment(5, 3)
    assert d.get() == [(5, 3, 2)]
    d.increment(4, 2)
    assert d.get() == [(4, 1, 1), (5, 1, 3), (6, 2, 2)]
    d.increment(7, 3)
    assert d.get() == [(4, 1, 1), (5, 1, 3), (6, 1, 2), (7, 1, 3), (8, 2, 1)]


def test_inc_delete_range_adjacent_run_quirk():
    # Quirk Q9 (double_delete.rs:52 tests `self.0[idx].0 > base`): after incrementing (5,3) the
    # loop reaches the adjacent run at 8 (key 8 == next key > base 5) and takes the gap branch
    # with a zero-length remainder, which release builds insert as an entry of length 0
    # (rle/mod.rs:34's debug_assert is compiled out).  Release semantics, hand-derived.
    d = DoubleDeletes()
    d.increment(5, 3)
    d.increment(5, 3)
    d.increment(8, 2)
    assert d.get() == [(5, 3, 2), (8, 2, 1)]
    d.increment(5, 5)
    assert d.get() == [(5, 3, 3), (8, 0, 1), (8, 2, 2)]
    # zero-length entries are counted as entries of the run they precede and multiply
    d.increment(3, 6)
    assert d.get() == [(3, 2, 1), (5, 3, 4), (8, 0, 1), (8, 0, 2), (8, 0, 1), (8, 1, 3), (9, 1, 2)]


# --- benches/yjs.rs:39,46: final doc.len() == endContent.len() --------------------------------
@pytest.mark.parametrize("name", TRACE_NAMES)
@pytest.mark.parametrize("caps", [(32, 16), (4, 8)])
def test_trace_final_length(name, caps):
    t = load_trace(name)
    assert t.start_len == 0
    d = OracleDoc(*caps)
    assert d.apply_trace(d.agent("jeremy"), t.counts, t.patches) == OK
    assert len(d) == t.end_len
    g = GOLDEN[f"{name}/L{caps[0]}"]
    assert g["len"] == t.end_len
    assert hex(d.digest()) == g["digest"]
    assert d.sizes() == g["sizes"]


# --- doc.rs:620-676 remote_txns (remote == local for frontier/txns/deletes), whole traces ------
@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode"])
def test_remote_replay_equals_local(name):
    t = load_trace(name)
    loc = OracleDoc()
    loc.apply_trace(loc.agent("jeremy"), t.counts, t.patches)
    rem = OracleDoc()
    assert rem.apply_remote_wire(load_remote_wire(name)) == OK
    el, er = loc.export(), rem.export()
    for k in ("raw", "leaf_sizes", "cwo", "deletes", "txns", "parents", "frontier"):
        assert np.array_equal(el[k], er[k]), k
    assert loc.digest() == rem.digest() == int(GOLDEN[f"{name}/L32"]["remote_digest"], 16)


def test_remote_txns_unit():
    # The exact reference test: seph@0 Ins "hi" (ROOT, ROOT), then seph@2 Del(seph@0, 2).
    rem = OracleDoc(4, 8)
    assert rem.apply_remote_wire(wire([("seph", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)])])) == OK
    loc = OracleDoc(4, 8)
    loc.agent("seph")
    assert loc.local_insert(0, 0, 2) == OK
    a, b = rem.export(), loc.export()
    for k in ("frontier", "txns", "parents", "deletes"):
        assert np.array_equal(a[k], b[k]), k
    assert rem.apply_remote_wire(wire([("seph", 2, [("seph", 1)], [("del", ("seph", 0), 2)])])) == OK
    assert loc.local_delete(0, 0, 2) == OK
    a, b = rem.export(), loc.export()
    for k in ("frontier", "txns", "parents", "deletes"):
        assert np.array_equal(a[k], b[k]), k
    assert len(rem) == len(loc) == 0


# --- doc.rs:522-532 smoke ---------------------------------------------------------------------
def test_smoke():
    d = OracleDoc(4, 8)
    a = d.agent("seph")
    assert d.local_insert(a, 0, 2) == OK     # "hi"
    assert d.local_insert(a, 1, 4) == OK     # "hyoooi"
    assert d.local_delete(a, 0, 3) == OK     # "ooi"
    assert len(d) == 3


# --- doc.rs:589-601 deletes_merged --------------------------------------------------------------
def test_deletes_merged():
    d = OracleDoc(4, 8)
    a = d.agent("seph")
    d.local_insert(a, 0, 3)
    for _ in range(3):
        assert d.local_delete(a, 0, 1) == OK
    e = d.export()
    assert len(d) == 0
    assert e["deletes"].tolist() == [[3, 0, 3]]   # three single deletes coalesce (Rle::append)
    m = 0xFFFFFFFF
    assert e["raw"][:, 3].tolist() == [-1 & m] * 3        # the tree keeps three deleted entries
    assert e["canon"].tolist() == [[0, m, m, -3 & m]]     # which are one item-level run


# --- doc.rs:571-587 random_single_document (own RNG; SmallRng seed-7 stream is Rust-only) -----
def make_random_change(d, a, rng, shadow):
    n = len(d)
    w = 0.55 if n < 100 else 0.45
    if n == 0 or rng.random() < w:
        pos = rng.randint(0, n)
        assert d.local_insert(a, pos, 1) == OK
        shadow.insert(pos, "x")
    else:
        pos = rng.randint(0, n - 1)
        span = rng.randint(1, min(10, n - pos))
        assert d.local_delete(a, pos, span) == OK
        del shadow[pos:pos + span]


@pytest.mark.parametrize("caps", [(32, 16), (4, 8)])
def test_random_single_document(caps):
    rng = random.Random(7)
    d = OracleDoc(*caps)
    a = d.agent("seph")
    shadow = []
    for _ in range(1000):
        make_random_change(d, a, rng, shadow)
        assert len(d) == len(shadow)
    s = d.sizes()
    assert s["cwo"] == 1 and s["agents"] == 1      # client_with_order / item_orders: 1 entry
    assert s["txns"] == 1


# --- error paths mirror the reference's panics -----------------------------------------------
def test_errors():
    d = OracleDoc()
    a = d.agent("seph")
    assert d.local_insert(a, 1, 1) == ERR_POS_OOB           # root.rs:71/79 panic
    d = OracleDoc()
    a = d.agent("seph")
    d.local_insert(a, 0, 5)
    assert d.local_delete(a, 3, 3) == ERR_POS_OOB           # mutations.rs:573 panic
    r = OracleDoc()
    assert r.apply_remote_wire(wire([("seph", 1, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 1)])])) == ERR_SEQ


def test_concurrent_nontermination_detected():
    # A types "ab" (one entry); B inserts after 'a' concurrently (origin_right ROOT).  The
    # reference's integrate lands mid-entry in the last entry of the doc and next_entry() fails
    # without moving the cursor (cursor.rs:127-141) -> the loop never exits (doc.rs:183-221).
    d = OracleDoc()
    w = wire([("A", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)]),
              ("B", 0, [("A", 0)], [("ins", ("A", 0), ROOT_ID, 1)])])
    assert d.apply_remote_wire(w) == ERR_NONTERMINATING


def test_concurrent_at_doc_end_is_nonterminating():
    # Two agents insert at the start of a 1-item document concurrently: the scan reaches the last
    # entry of the document and next_entry() cannot advance -> the reference loops forever.
    w1 = [("A", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 1)]), ("B", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 1)])]
    d1, d2 = OracleDoc(), OracleDoc()
    assert d1.apply_remote_wire(wire(w1)) == ERR_NONTERMINATING
    assert d2.apply_remote_wire(wire(w1[::-1])) == OK   # A sorts before B: breaks on origin_right


def test_concurrent_tiebreak_converges():
    # base "xy" by X; A and B both insert between x and y concurrently.  Both delivery orders
    # give x A B y (doc.rs:204-216 name tie-break, incl. the end-of-entry first iteration).
    base = ("X", 0, [ROOT_ID], [("ins", ROOT_ID, ROOT_ID, 2)])
    ta = ("A", 0, [("X", 1)], [("ins", ("X", 0), ("X", 1), 1)])
    tb = ("B", 0, [("X", 1)], [("ins", ("X", 0), ("X", 1), 1)])
    res = []
    for order in ((base, ta, tb), (base, tb, ta)):
        d = OracleDoc()
        assert d.apply_remote_wire(wire(list(order))) == OK
        names = [t[0] for t in order]
        ag, sq = d.pos_to_loc(np.arange(4))
        res.append([(names[a], int(q)) for a, q in zip(ag, sq)])
    assert res[0] == res[1] == [("X", 0), ("A", 0), ("B", 0), ("X", 1)]


def test_queries_roundtrip():
    t = load_trace("sveltecomponent")
    d = OracleDoc()
    d.apply_trace(d.agent("jeremy"), t.counts, t.patches)
    pos = np.arange(len(d), dtype=np.uint32)
    ag, seq = d.pos_to_loc(pos)
    assert (ag == 0).all()
    p2, dl = d.loc_to_pos(ag, seq)
    assert np.array_equal(p2, pos) and (dl == 0).all()
    # every seq: deleted items map to the position of the next visible item
    allseq = np.arange(d.sizes()["next_order"], dtype=np.uint32)
    p3, dl3 = d.loc_to_pos(np.zeros_like(allseq, dtype=np.uint16), allseq)
    assert ((dl3 == 0) | (dl3 == 1) | (dl3 == 2)).all()
    assert (p3[dl3 != 2] <= len(d)).all()


# --- config 4 generator: doc.rs:571-587 random_single_document invariants + distribution ------
def test_generator_invariants():
    d = OracleDoc()
    a = d.agent("seph")
    assert d.apply_random(a, 20000, 12345) == 0
    s = d.sizes()
    assert s["cwo"] == 1 and s["agents"] == 1 and s["txns"] == 1 and s["frontier"] == 1
    # make_random_change keeps the document short (deletes of up to 10 chars outweigh inserts)
    assert len(d) <= 200
    assert s["next_order"] > 20000   # deletes of 1..10 chars consume several orders each


@pytest.mark.parametrize("name", ["automerge-paper", "rustcode", "sveltecomponent"])
@pytest.mark.parametrize("leaf,node", [(32, 16), (4, 8)])
def test_text_matches_end_content(name, leaf, node):
    # Text materialisation (to_string with the rope on, doc.rs:498-505) pinned by the reference's
    # own fixture: the visible items' content in document order is the trace's endContent.
    from crdt_amd.traces import content_by_order, fnv1a64, utf32_to_str
    t = load_trace(name)
    o = OracleDoc(leaf, node)
    assert o.apply_trace(o.agent("a"), t.counts, t.patches) == 0
    txt, _ = o.text(content_by_order(t))
    b = utf32_to_str(txt).encode()
    assert len(txt) == t.end_len and len(b) == t.end_bytes
    assert fnv1a64(b) == t.end_fnv


@pytest.mark.parametrize("name", ["sveltecomponent", "rustcode", "automerge-paper"])
def test_splitlist_index_same_state(name):
    # the CPU baseline's order index is the reference's SplitList (split_list/mod.rs, bucket 100,
    # delete orders padded with the last marker, doc.rs:337-339 / 402-404); it must give the same
    # document as the dense table, on the local and the remote (index-reading) path
    from crdt_amd.traces import load_remote_wire
    t = load_trace(name)
    a = OracleDoc(32, 16)
    b = OracleDoc(32, 16, split_index=True)
    assert a.apply_trace(a.agent("jeremy"), t.counts, t.patches) == 0
    assert b.apply_trace(b.agent("jeremy"), t.counts, t.patches) == 0
    assert a.digest() == b.digest()
    w = load_remote_wire(name)
    a, b = OracleDoc(32, 16), OracleDoc(32, 16, split_index=True)
    assert a.apply_remote_wire(w) == 0 and b.apply_remote_wire(w) == 0
    assert a.digest() == b.digest()


@pytest.mark.parametrize("seed", range(4))
def test_splitlist_index_concurrent(seed):
    from fuzz_gen import concurrent_wire, config5_wire
    for w in (concurrent_wire(seed, n_agents=3, rounds=5)[0], config5_wire(seed, base_len=2000, rounds=4, ops=4)):
        a, b = OracleDoc(4, 8), OracleDoc(4, 8, split_index=True)
        sa, sb = a.apply_remote_wire(w), b.apply_remote_wire(w)
        assert sa == sb
        if sa == 0:
            assert a.digest() == b.digest()


def test_query_fixture_matches_oracle():
    # tests/golden/ap_remote_pos_seq.delta.gz (bench.py checks every timed pos -> loc answer against
    # it) is the oracle's pos -> (agent 0, seq) for every position of automerge-paper's remote replay
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import golden_pos_seq
    from crdt_amd.traces import load_remote_wire
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(load_remote_wire("automerge-paper")) == 0
    gseq = golden_pos_seq("automerge-paper")
    assert gseq is not None and gseq.shape[0] == len(o)
    a, s = o.pos_to_loc(np.arange(len(o), dtype=np.uint32))
    assert (a == 0).all() and np.array_equal(s, gseq)


def test_loc_query_fixtures_match_oracle():
    # tests/golden/ap_remote_seq_pos.delta.gz (bench.py checks every timed loc -> pos answer against
    # it): the oracle's (agent 0, seq) -> (pos, deleted) (Cursor::count_pos, cursor.rs:147-190) for
    # every seq of automerge-paper's remote replay; queries_{rustcode,sveltecomponent}.npz: sampled
    # pos -> loc and loc -> pos answers of those traces' remote replays
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from bench import golden_seq_pos
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(load_remote_wire("automerge-paper")) == 0
    gp, gd = golden_seq_pos("automerge-paper")
    n = o.sizes()["next_order"]
    assert gp.shape[0] == n
    p, d = o.loc_to_pos(np.zeros(n, np.uint16), np.arange(n, dtype=np.uint32))
    assert np.array_equal(d, gd) and np.array_equal(p[d != 2], gp[d != 2])
    # every visible seq maps to its position and back (pos -> loc fixture)
    a, s = o.pos_to_loc(np.arange(len(o), dtype=np.uint32))
    assert np.array_equal(gp[s], np.arange(len(o))) and (gd[s] == 0).all()
    for tr in ("rustcode", "sveltecomponent"):
        z = np.load(os.path.join(HERE, "golden", f"queries_{tr}.npz"))
        o = OracleDoc(32, 16)
        assert o.apply_remote_wire(load_remote_wire(tr)) == 0
        a, s = o.pos_to_loc(z["pos"])
        assert np.array_equal(a, z["pos_agent"]) and np.array_equal(s, z["pos_seq"])
        p, d = o.loc_to_pos(z["loc_agent"], z["loc_seq"])
        assert np.array_equal(d, z["loc_deleted"]) and np.array_equal(p, z["loc_pos"])
