"""GPU parity of text materialisation (ListCRDT::to_string with the rope on,
doc.rs:230-233, 430-432, 498-505) through the C ABI.

Pinned by the reference's own fixtures: the materialised text of each benchmark trace hashes to
the FNV-1a of the trace's endContent (benchmark_data/*.json.gz, via tests/golden/make_traces.py).
Concurrent histories (no reference fixture) are checked against the oracle's text_of.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import crdt_amd  # noqa: E402
from crdt_amd.traces import content_by_order, fnv1a64, load_remote_wire, load_trace, utf32_to_str  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402

NAMES = ["sveltecomponent", "rustcode", "automerge-paper"]


@pytest.mark.parametrize("leaf", [32, 4])
def test_trace_text_local(leaf):
    # the debug layout (leaf 4) holds AP in ~25,900 leaves (past round 1's 8,160-leaf directory)
    names = NAMES
    traces = [load_trace(n) for n in names]
    e = crdt_amd.Engine(len(names), leaf)
    ag = e.agent_intern(list(range(len(names))), ["jeremy"] * len(names))
    for d, t in enumerate(traces):
        assert e.apply_trace([d], int(ag[d]), t.counts, t.patches)[0] == 0
    e.set_content(list(range(len(names))), list(range(len(names))), [content_by_order(t) for t in traces])
    dg = e.text_digests()
    for d, t in enumerate(traces):
        txt = e.text(d)
        s = utf32_to_str(txt).encode()
        assert len(txt) == t.end_len and len(s) == t.end_bytes
        assert fnv1a64(s) == t.end_fnv, t.name          # the reference's endContent
        o = OracleDoc(leaf, 16 if leaf == 32 else 8)
        o.apply_trace(o.agent("jeremy"), t.counts, t.patches)
        ot, odg = o.text(content_by_order(t))
        assert np.array_equal(txt, ot)
        assert int(dg[d]) == odg


def test_trace_text_remote_shared_stream():
    # config 2 shape: many documents replay the AP remote form under different client ids and
    # share one content stream; every text digest must be the endContent's.
    t = load_trace("automerge-paper")
    w = load_remote_wire("automerge-paper")
    n = 8
    e = crdt_amd.Engine(n, 32)
    e.stage_remote_replicated(w, 0, [f"{0xC0FFEE ^ d:016x}" for d in range(n)])
    assert (e.run() == 0).all()
    c = content_by_order(t)
    e.set_content(list(range(n)), [0] * n, [c])
    e.materialize_async()
    e.sync()
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(w) == 0
    ot, odg = o.text(c)
    assert fnv1a64(utf32_to_str(ot).encode()) == t.end_fnv
    assert (e.text_digests() == np.uint64(odg)).all()
    assert np.array_equal(e.text(n - 1), ot)
    assert e.materialize_ms() > 0


def test_concurrent_text():
    from fuzz_gen import concurrent_wire, config5_wire
    wires = [concurrent_wire(s, n_agents=3, rounds=5)[0] for s in range(4)]
    wires += [config5_wire(200 + s, base_len=8192, rounds=6, ops=4) for s in range(4)]
    n = len(wires)
    e = crdt_amd.Engine(n, 32)
    st = e.apply_remote_wire(list(range(n)), wires)
    rng = np.random.default_rng(5)
    ok = [d for d in range(n) if st[d] == 0]
    assert len(ok) >= 4
    streams = []
    for d in ok:
        o = OracleDoc()
        o.apply_remote_wire(wires[d])
        streams.append(rng.integers(0x20, 0xD7FF, o.sizes()["next_order"], dtype=np.uint32))
    e.set_content(ok, list(range(len(ok))), streams)
    dg = e.text_digests()
    for i, d in enumerate(ok):
        o = OracleDoc()
        o.apply_remote_wire(wires[d])
        ot, odg = o.text(streams[i])
        assert np.array_equal(e.text(d), ot), d
        assert int(dg[d]) == odg


def test_text_errors():
    t = load_trace("sveltecomponent")
    e = crdt_amd.Engine(3, 32)
    ag = e.agent_intern([0, 1, 2], ["a"] * 3)
    e.apply_trace([0, 1, 2], int(ag[0]), t.counts, t.patches)
    c = content_by_order(t)
    # doc 0: full content, doc 1: one entry short, doc 2: none
    e.set_content([0, 1], [0, 1], [c, c[:-1]])
    dg = e.text_digests()
    assert dg[0] != 0 and dg[1] == 0 and dg[2] == 0
    assert len(e.text(0)) == t.end_len
    for d in (1, 2):
        with pytest.raises(crdt_amd.CrdtError):
            e.text(d)
    # empty documents have empty text
    e2 = crdt_amd.Engine(2, 32)
    e2.set_content([0, 1], [0, 0], [np.zeros(0, np.uint32)])
    assert len(e2.text(1)) == 0
    # a new replay invalidates the text; re-materialising follows the new state
    st = e2.apply_local([(0, [(int(e2.agent_intern([0], ["x"])[0]), [(0, 0, 3)])])])
    assert st[0] == 0
    e2.set_content([0], [0], [np.array([65, 66, 67], np.uint32)])
    assert utf32_to_str(e2.text(0)) == "ABC"


def test_json_file_to_text(tmp_path):
    # §8f row 4 end to end: a trace file in the reference's own format (gzip'd JSON, lib.rs:10-27)
    # -> native decoder (crdt_trace_load) -> GPU replay -> GPU materialisation == endContent.
    import gzip
    import json
    from crdt_amd.traces import ingest_json
    from test_trace_ingest import _replay_text, _to_json_obj
    t = load_trace("sveltecomponent")
    p = tmp_path / "sveltecomponent.json.gz"
    with gzip.open(p, "wt", encoding="utf-8") as f:
        json.dump(_to_json_obj(t, _replay_text(t)), f)
    g = ingest_json(str(p))
    n = 4
    e = crdt_amd.Engine(n, 32)
    ag = e.agent_intern(list(range(n)), ["jeremy"] * n)
    assert (e.apply_trace(list(range(n)), int(ag[0]), g.counts, g.patches) == 0).all()
    e.set_content(list(range(n)), [0] * n, [content_by_order(g)])
    for d in range(n):
        assert utf32_to_str(e.text(d)).encode() == g.end
    assert (e.lens() == g.end_len).all()
