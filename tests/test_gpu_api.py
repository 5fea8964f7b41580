"""C-ABI behaviour on the GPU (include/crdt_gpu.h conventions): probe answers after a document's
stop point, shared device streams vs per-document copies, and documents named twice in one call.
Each compares the HIP engine (through the C ABI) with the oracle or with the engine's own
unshared run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire, load_trace  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402
from fuzz_gen import config1_probes  # noqa: E402
from test_gpu_parity import assert_same  # noqa: E402

UNKNOWN = np.array([0xFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 2], np.uint32)


def test_probes_after_a_stop_answer_unknown():
    # A probed call first leaves valid answers in every probe slot; the second call's document
    # stops at an out-of-bounds delete (root.rs:160) in its 4th txn: the probes of the txns it
    # never reached must answer "unknown", not the previous call's answers.
    t = load_trace("sveltecomponent")
    k = 400
    c = t.counts[:k]
    p = t.patches[: int(c.sum())]
    e = crdt_amd.Engine(1, 32)
    a = int(e.agent_intern([0], ["jeremy"])[0])
    q = config1_probes(c, p, a)
    tx = np.stack([np.full(k, a), c], 1).astype(np.uint32)
    st, ans = e.apply_local_probed([0], [0, k], tx, p, q)
    assert st[0] == 0 and not (ans == UNKNOWN).all(1).any()
    e.reset_async()
    bad = np.array([[0, 0, 5], [2, 1, 0], [1, 0, 2], [3, 50, 0], [0, 0, 1], [1, 1, 0]], np.uint32)
    cb = np.ones(len(bad), np.uint32)
    qb = np.array([[0, a, 0]] * len(bad), np.uint32)
    st, ans = e.apply_local_probed([0], [0, len(bad)], np.stack([np.full(len(bad), a), cb], 1), bad, qb)
    assert st[0] == -1
    o = OracleDoc()
    so, oans = o.probe_trace(o.agent("jeremy"), cb[:3], bad[:3], qb[:3])
    assert so == 0
    assert np.array_equal(ans[:3], oans)
    assert (ans[3:] == UNKNOWN).all(), ans[3:]


def test_share_streams_parity():
    # crdt_set_share_streams(1): documents staged from one host stream read one device copy of
    # it.  Digests, exports and statuses equal a run with one copy per document, for the local
    # shared form (config 3) and the replicated remote form (config 2).
    names = ["automerge-paper", "rustcode", "sveltecomponent"]
    traces = [load_trace(n) for n in names]
    n = 12
    which = [d % 3 for d in range(n)]
    res = []
    for share in (False, True):
        e = crdt_amd.Engine(n, 32)
        e.share_streams(share)
        ag = e.agent_intern(list(range(n)), ["jeremy"] * n)
        e.stage_local_shared(list(range(n)), which, int(ag[0]), traces)
        st = e.run()
        assert (st == 0).all(), st
        res.append((e.digests(), [e.export(d) for d in range(3)]))
    assert (res[0][0] == res[1][0]).all()
    for a, b in zip(res[0][1], res[1][1]):
        assert_same(a, b)
    w = load_remote_wire("sveltecomponent")
    dgs = []
    for share in (False, True):
        e = crdt_amd.Engine(8, 32)
        e.share_streams(share)
        e.stage_remote_replicated(w, 0, [f"client{d:02d}" for d in range(8)])
        st = e.run()
        assert (st == 0).all(), st
        dgs.append(e.digests())
    assert (dgs[0] == dgs[1]).all()
    # the digest does not cover agent names (bench.py checks renamed copies the same way)
    o = OracleDoc()
    assert o.apply_remote_wire(w) == 0
    assert (dgs[0] == np.uint64(o.digest())).all()


def test_document_named_twice_is_an_argument_error():
    e = crdt_amd.Engine(2, 32)
    a = int(e.agent_intern([0], ["x"])[0])
    with pytest.raises(crdt_amd.CrdtError) as ex:
        e.apply_local([(0, [(a, [(0, 0, 3)])]), (0, [(a, [(0, 0, 1)])])])
    assert "rc=-100" in str(ex.value)
    # nothing was applied: the document is still empty and accepts a valid call
    assert int(e.lens([0])[0]) == 0
    assert e.apply_local([(0, [(a, [(0, 0, 3)])])])[0] == 0
    assert int(e.lens([0])[0]) == 3
