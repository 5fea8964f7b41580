"""Native trace ingestion (include/crdt_trace.h) — host-only, runs on the CPU.

The decoder replaces crdt-testdata `load_testing_data` (src/testdata/src/lib.rs:29-48).  It is
pinned three ways:
  * the committed binary traces (data/traces/*.trc.gz, converted from the reference's
    benchmark_data by tests/golden/make_traces.py with Python's json module) are re-serialised as
    JSON — ASCII-escaped (\\uXXXX, surrogate pairs) and raw UTF-8 — and must decode to the same
    counts / patches / inserted text;
  * when /root/reference is present (the build container only), the reference's own
    benchmark_data/*.json.gz decode to exactly the committed traces, endContent FNV included;
  * Python's json module is the checker for randomised documents and for rejection of malformed
    input.
"""
import gzip
import json
import os
import random

import numpy as np
import pytest

import crdt_amd
from crdt_amd.traces import TRACE_NAMES, fnv1a64, ingest_json, load_trace

REF_DATA = "/root/reference/benchmark_data"


def _to_json_obj(t, end: str, start: str = ""):
    s = t.text.decode("utf-8")
    txns, k, off = [], 0, 0
    for i, c in enumerate(t.counts.tolist()):
        ps = []
        for _ in range(c):
            pos, dl, il = (int(x) for x in t.patches[k])
            ps.append([pos, dl, s[off: off + il]])
            off += il
            k += 1
        txns.append({"time": f"2021-01-{1 + i % 28:02d}T00:00:00.000Z", "patches": ps})
    return {"startContent": start, "endContent": end, "txns": txns}


def _replay_text(t) -> str:
    s = t.text.decode("utf-8")
    doc, off = [], 0
    for pos, dl, il in t.patches.tolist():
        del doc[pos: pos + dl]
        doc[pos:pos] = s[off: off + il]
        off += il
    return "".join(doc)


def _check_same(got, t):
    assert np.array_equal(got.counts, t.counts)
    assert np.array_equal(got.patches, t.patches)
    assert got.text == t.text


@pytest.fixture(scope="module", autouse=True)
def _built():
    crdt_amd.build()


@pytest.mark.parametrize("ascii_only", [True, False])
def test_sveltecomponent_json_roundtrip(tmp_path, ascii_only):
    t = load_trace("sveltecomponent")
    end = _replay_text(t)
    b = end.encode("utf-8")
    assert len(end) == t.end_len and len(b) == t.end_bytes and fnv1a64(b) == t.end_fnv
    p = tmp_path / "sv.json.gz"
    with gzip.open(p, "wt", encoding="utf-8") as f:
        json.dump(_to_json_obj(t, end), f, ensure_ascii=ascii_only)
    got = ingest_json(str(p))
    _check_same(got, t)
    assert got.end == b and got.end_len == t.end_len and got.end_fnv == t.end_fnv and got.start == b""


@pytest.mark.parametrize("name", ["automerge-paper", "rustcode"])
def test_large_traces_json_roundtrip(tmp_path, name):
    t = load_trace(name)
    p = tmp_path / (name + ".json.gz")
    with gzip.open(p, "wt", encoding="utf-8") as f:
        json.dump(_to_json_obj(t, "end \U0001F600 ok", start=""), f, ensure_ascii=(name == "rustcode"))
    got = ingest_json(str(p))
    _check_same(got, t)
    assert got.end_len == 8 and got.end == "end \U0001F600 ok".encode()


def test_plain_json_file(tmp_path):
    obj = {"endContent": "xy", "extra": {"a": [1, 2.5e3, None, True, False, {"b": "\\"}]},
           "txns": [{"patches": [[0, 0, "x"], [1, 0, "y"]], "time": 7}, {"patches": []}],
           "startContent": ""}
    p = tmp_path / "t.json"
    p.write_text(json.dumps(obj))
    got = ingest_json(str(p))
    assert got.counts.tolist() == [2, 0]
    assert got.patches.tolist() == [[0, 0, 1], [1, 0, 1]]
    assert got.text == b"xy" and got.end == b"xy"


def _parse(doc: bytes):
    import ctypes as C
    L = crdt_amd.lib()
    h = C.c_void_p()
    rc = L.crdt_trace_parse(doc, len(doc), C.byref(h))
    if rc != 0:
        return rc, None
    sz = np.zeros(7, np.uint64)
    assert L.crdt_trace_sizes(h, sz.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
    n_txns, n_patches, tb = int(sz[0]), int(sz[1]), int(sz[2])
    counts = np.zeros(n_txns, np.uint32)
    patches = np.zeros((n_patches, 3), np.uint32)
    text = C.create_string_buffer(max(tb, 1))
    assert L.crdt_trace_copy(h, counts.ctypes.data, patches.ctypes.data, text, None, None) == 0
    L.crdt_trace_free(h)
    return 0, (counts, patches, text.raw[:tb], int(sz[5]))


def test_random_documents_match_python_json():
    rng = random.Random(1234)
    alphabet = ["a", "\n", "\t", '"', "\\", "/", "é", "中", "\U0001F600", " ", "\x01", "퟿"]
    for it in range(200):
        txns = []
        for _ in range(rng.randrange(0, 6)):
            ps = [[rng.randrange(0, 1 << 32), rng.randrange(0, 1000),
                   "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 8)))]
                  for _ in range(rng.randrange(0, 5))]
            txns.append({"time": "t", "patches": ps})
        end = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 20)))
        obj = {"startContent": "", "endContent": end, "txns": txns}
        doc = json.dumps(obj, ensure_ascii=bool(it % 2), indent=(2 if it % 3 == 0 else None)).encode()
        rc, got = _parse(doc)
        assert rc == 0, (rc, crdt_amd.lib().crdt_last_error())
        counts, patches, text, end_len = got
        ref = json.loads(doc)
        assert counts.tolist() == [len(t["patches"]) for t in ref["txns"]]
        flat = [p for t in ref["txns"] for p in t["patches"]]
        assert patches.tolist() == [[p[0], p[1], len(p[2])] for p in flat]
        assert text == "".join(p[2] for p in flat).encode("utf-8")
        assert end_len == len(ref["endContent"])


@pytest.mark.parametrize("doc", [
    b"",
    b"{",
    b'{"startContent":"","endContent":"","txns":[]} x',
    b'{"startContent":"","endContent":""}',
    b'{"startContent":"","endContent":"","txns":[{"patches":[[-1,0,"a"]]}]}',
    b'{"startContent":"","endContent":"","txns":[{"patches":[[1.5,0,"a"]]}]}',
    b'{"startContent":"","endContent":"","txns":[{"patches":[[4294967296,0,"a"]]}]}',
    b'{"startContent":"","endContent":"","txns":[{"patches":[[0,0,1]]}]}',
    b'{"startContent":"","endContent":"","txns":[{"patches":[[0,0]]}]}',
    b'{"startContent":"","endContent":"","txns":[{"time":"x"}]}',
    b'{"startContent":"","endContent":"\\ud83d","txns":[]}',
    b'{"startContent":"","endContent":"\\ude00","txns":[]}',
    b'{"startContent":"","endContent":"\xff","txns":[]}',
    b'{"startContent":"","endContent":"\xed\xa0\x80","txns":[]}',
    b'{"startContent":"","endContent":"a\nb","txns":[]}',
    b'{"startContent":"","endContent":"\\x","txns":[]}',
])
def test_malformed_rejected(doc):
    assert not _valid_for_python(doc)            # Python's json agrees it is not a valid trace ...
    rc, _ = _parse(doc)                          # ... and the decoder rejects it
    assert rc == -104, rc


def _valid_for_python(doc: bytes) -> bool:
    try:
        o = json.loads(doc)
        o["startContent"].encode("utf-8"), o["endContent"].encode("utf-8")
        for t in o["txns"]:
            for p in t["patches"]:
                if not (len(p) == 3 and all(type(x) is int and 0 <= x < 2 ** 32 for x in p[:2])
                        and isinstance(p[2], str)):
                    return False
                p[2].encode("utf-8")
        return True
    except (ValueError, KeyError, TypeError, UnicodeError):
        return False


def test_io_errors(tmp_path):
    with pytest.raises(crdt_amd.CrdtError, match="rc=-105"):
        ingest_json(str(tmp_path / "missing.json.gz"))
    p = tmp_path / "trunc.json.gz"
    blob = gzip.compress(json.dumps({"startContent": "", "endContent": "", "txns": [
        {"patches": [[0, 0, "a" * 1000]]}] * 200}).encode())
    p.write_bytes(blob[: len(blob) // 2])
    with pytest.raises(crdt_amd.CrdtError):
        ingest_json(str(p))


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference benchmark_data only in the build container")
@pytest.mark.parametrize("name", TRACE_NAMES)
def test_reference_files_decode_to_committed_traces(name):
    got = ingest_json(os.path.join(REF_DATA, name + ".json.gz"))
    t = load_trace(name)
    _check_same(got, t)
    assert (got.end_len, got.end_bytes, got.end_fnv, got.start_len) == (t.end_len, t.end_bytes, t.end_fnv, t.start_len)
