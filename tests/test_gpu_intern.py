"""Device agent-name interning (crdt_agent_intern_dev, kernels.h k_intern)
against the reference semantics of ListCRDT::get_or_create_agent_id (doc.rs:66-89): per document,
ids in order of first appearance, "ROOT" -> 0xFFFF and never stored; and each name's rank in
byte-lexicographic order (Rust `str` Ord, the order integrate's tie-break compares, doc.rs:207).
The expected values are restated here in Python (a dict per document) and cross-checked with the
host path crdt_agent_intern on the same calls."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = 0xFFFF
INVALID = 0xFFFFFFFF


def reference(calls):
    """calls: list of (docs, names) batches -> per batch (ids, ranks) by the reference rule."""
    tables, index = {}, {}
    out = []
    for docs, names in calls:
        ids = []
        for d, n in zip(docs, names):
            b = n.encode() if isinstance(n, str) else bytes(n)
            t = tables.setdefault(d, [])
            ix = index.setdefault(d, {})
            if b == b"ROOT":
                ids.append(ROOT)
            elif b in ix:
                ids.append(ix[b])
            else:
                t.append(b)
                ix[b] = len(t) - 1
                ids.append(len(t) - 1)
        rank_of = {d: {b: r for r, b in enumerate(sorted(t))} for d, t in tables.items()}
        ranks = [INVALID if i == ROOT else rank_of[d][tables[d][i]] for d, i in zip(docs, ids)]
        out.append((np.array(ids, np.uint16), np.array(ranks, np.uint32)))
    return out


def _engine(n):
    import crdt_amd
    return crdt_amd.Engine(n, 32)


def _random_names(rng, k):
    pool = ["ROOT", "", "a", "b", "ab", "aa", "seph", "jeremy", "Jeremy", "kevin", "ROOTS", "ROO",
            "z" * 40, "été", "日本", "user-%d" % 7, "user-%d" % 70]
    pool += ["n%05d" % int(x) for x in rng.integers(0, 300, 40)]
    return [pool[int(i)] for i in rng.integers(0, len(pool), k)]


def test_intern_matches_reference_and_host_path():
    rng = np.random.default_rng(11)
    n_docs = 64
    e, h = _engine(n_docs), _engine(n_docs)
    calls = []
    for _ in range(3):  # tables persist across calls: later ids continue, ranks re-sort
        m = 2000
        docs = rng.integers(0, n_docs, m).astype(np.uint32)
        calls.append((docs.tolist(), _random_names(rng, m)))
    want = reference(calls)
    for (docs, names), (wid, wrank) in zip(calls, want):
        gid, grank = e.agent_intern_dev(docs, names)
        assert np.array_equal(gid, wid)
        assert np.array_equal(grank, wrank)
        hid = h.agent_intern(docs, names)  # host path, same call
        assert np.array_equal(hid, gid)


def test_intern_arbitrary_bytes_and_one_document_many_names():
    e = _engine(4)
    names = [b"a\x00b", b"a\x00", b"a", b"\xff", b"", b"ROOT", b"a\x00b", b"\x00"]
    names += [b"n%04d" % i for i in range(900)] + [b"n0004", b"a"]
    docs = [2] * len(names)
    (wid, wrank), = reference([(docs, names)])
    gid, grank = e.agent_intern_dev(docs, names)
    assert np.array_equal(gid, wid) and np.array_equal(grank, wrank)


def test_intern_past_the_lds_table():
    # documents with more than the LDS table's 1,024 names intern with the table in HBM and ranks
    # from a sort (k_intern_big); ids and ranks as the reference's, in the same call as small
    # documents, and tables persist across calls
    rng = np.random.default_rng(5)
    e, h = _engine(3), _engine(3)
    calls = []
    for step in range(2):
        big = ["u%06d-%s" % (int(x), "x" * int(x % 7)) for x in rng.integers(0, 9000, 6000)]
        small = _random_names(rng, 300)
        docs = [1] * len(big) + [2] * len(small) + [0] * 50
        calls.append((docs, big + small + ["ROOT", "a"] * 25))
    for (docs, names), (wid, wrank) in zip(calls, reference(calls)):
        gid, grank = e.agent_intern_dev(docs, names)
        assert np.array_equal(gid, wid)
        assert np.array_equal(grank, wrank)
        assert np.array_equal(h.agent_intern(docs, names), gid)


def test_intern_rejects_more_than_u16_agents():
    # AgentId is u16 (doc.rs:66-80): 65,534 names fit (0xFFFF is ROOT, 0xFFFE unknown), more do not
    import crdt_amd
    e = _engine(2)
    names = ["x%06d" % i for i in range(65534)]
    gid, grank = e.agent_intern_dev([1] * len(names), names)
    assert np.array_equal(gid, np.arange(65534, dtype=np.uint16))
    assert np.array_equal(grank, np.arange(65534, dtype=np.uint32))  # (already in byte order)
    with pytest.raises(crdt_amd.CrdtError):
        e.agent_intern_dev([1], ["one more"])


def test_interned_agent_replays_like_the_host_interned_one():
    # ids from the device path drive a replay exactly as host-interned ids do
    from crdt_amd.traces import load_trace
    t = load_trace("sveltecomponent")
    k = 3000
    c = t.counts[:k]
    p = t.patches[: int(c.sum())]
    e, h = _engine(2), _engine(2)
    gid, _ = e.agent_intern_dev([0, 1], ["zed", "jeremy"])
    hid = h.agent_intern([0, 1], ["zed", "jeremy"])
    assert np.array_equal(gid, hid)
    assert (e.apply_trace([1], int(gid[1]), c, p) == 0).all()
    assert (h.apply_trace([1], int(hid[1]), c, p) == 0).all()
    assert int(e.digests()[1]) == int(h.digests()[1])


def test_replicated_staging_interns_on_the_device():
    # crdt_stage_remote_replicated with crdt_set_device_intern: every document's authors go
    # through k_intern in one call; ids, and so the replayed states, equal the host-interned path
    # (renamed agent = name index 3 of a 16-agent concurrent history, so the tie-break ranks move)
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from fuzz_gen import config5_wire
    w = config5_wire(3, base_len=2000, rounds=6, ops=4)
    n = 24
    names = ["c%02d-%s" % (d, "z" * (d % 5)) for d in range(n)]
    e, h = _engine(n), _engine(n)
    e.device_intern(True)
    e.stage_remote_replicated(w, 3, names)
    h.stage_remote_replicated(w, 3, names)
    assert (e.run() == 0).all() and (h.run() == 0).all()
    assert np.array_equal(e.digests(), h.digests())
