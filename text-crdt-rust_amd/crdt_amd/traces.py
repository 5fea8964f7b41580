"""Trace ingestion: the repo's compact binary form of the reference's editing traces.

Mirrors crdt-testdata's `load_testing_data` (src/testdata/src/lib.rs:29-48): a trace is a list of
txns, each a list of patches (pos, del_len, ins_content); positions count Unicode scalar values.
The JSON->binary conversion is tests/golden/make_traces.py (run once in the build container);
`ingest_json` decodes a reference trace file (.json.gz) natively instead (include/crdt_trace.h).
Only lengths of inserted strings are used by the CRDT hot path (doc.rs:383: chars().count()).
"""
from __future__ import annotations

import gzip
import os
import struct
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
DATA_DIR = os.path.normpath(os.path.join(_HERE, "..", "..", "data", "traces"))
TRACE_NAMES = ("automerge-paper", "rustcode", "sveltecomponent")


@dataclass
class Trace:
    name: str
    counts: np.ndarray      # u32[n_txns]   patches per txn
    patches: np.ndarray     # u32[n_patches, 3]  (pos, del_len, ins_len)
    start_len: int
    end_len: int            # chars of endContent
    end_bytes: int
    end_fnv: int
    text: bytes             # all inserted strings, utf-8, concatenated

    @property
    def n_txns(self) -> int:
        return int(self.counts.shape[0])

    @property
    def n_patches(self) -> int:
        return int(self.patches.shape[0])

    @property
    def n_orders(self) -> int:
        return int(self.patches[:, 1].sum() + self.patches[:, 2].sum())


def load_trace(name: str, data_dir: str = DATA_DIR) -> Trace:
    path = os.path.join(data_dir, name + ".trc.gz")
    with gzip.open(path, "rb") as f:
        blob = f.read()
    if blob[:8] != b"CRDTTRC1":
        raise ValueError(f"{path}: bad magic")
    n_txns, n_patches, start_len, end_len, end_bytes, end_fnv = struct.unpack_from("<5IQ", blob, 8)
    off = 8 + 28
    counts = np.frombuffer(blob, dtype=np.uint32, count=n_txns, offset=off).copy()
    off += 4 * n_txns
    patches = np.frombuffer(blob, dtype=np.uint32, count=3 * n_patches, offset=off).reshape(n_patches, 3).copy()
    off += 12 * n_patches
    (tb,) = struct.unpack_from("<I", blob, off)
    text = blob[off + 4: off + 4 + tb]
    return Trace(name, counts, patches, start_len, end_len, end_bytes, end_fnv, text)


def load_remote_wire(name: str, data_dir: str = DATA_DIR) -> bytes:
    """Remote-form (RemoteTxn wire batch) of a trace, generated offline by
    tests/golden/make_remote.py (see include/crdt_gpu.h "Remote wire batch")."""
    with gzip.open(os.path.join(data_dir, name + ".rtx.gz"), "rb") as f:
        return f.read()


def content_by_order(t: Trace) -> np.ndarray:
    """Order-indexed UTF-32 content of a trace replayed as one agent's local txns (or their remote
    form): orders are assigned per LocalOp, deleted orders first, then the inserted chars
    (doc.rs:155-165, 376-469).  Entries at delete orders are 0 (never read)."""
    cps = np.frombuffer(t.text.decode("utf-8").encode("utf-32-le"), dtype="<u4").astype(np.uint32)
    dl = t.patches[:, 1].astype(np.int64)
    ins = t.patches[:, 2].astype(np.int64)
    start = np.concatenate([[0], np.cumsum(dl + ins)[:-1]]) + dl       # first inserted order per patch
    n_ins = int(ins.sum())
    if cps.shape[0] != n_ins:
        raise ValueError(f"{t.name}: {cps.shape[0]} inserted code points, patches say {n_ins}")
    ins_excl = np.concatenate([[0], np.cumsum(ins)[:-1]])
    orders = np.repeat(start, ins) + (np.arange(n_ins) - np.repeat(ins_excl, ins))
    out = np.zeros(t.n_orders, np.uint32)
    out[orders] = cps
    return out


def utf32_to_str(a: np.ndarray) -> str:
    return np.ascontiguousarray(a, dtype="<u4").tobytes().decode("utf-32-le")


def fnv1a64(b: bytes) -> int:
    """FNV-1a over bytes (the trace header's end_fnv of endContent, tests/golden/make_traces.py)."""
    h = 0xCBF29CE484222325
    a = np.frombuffer(b, dtype=np.uint8)
    for x in a.tolist():
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def ingest_json(path: str) -> Trace:
    """Decode a reference trace file (gzip'd or plain JSON, schema src/testdata/src/lib.rs:10-27) with
    the native streaming decoder of libcrdt_gpu.so (crdt_trace_load, include/crdt_trace.h), the
    replacement of crdt-testdata `load_testing_data` (lib.rs:29-48).  Host-only; no GPU needed."""
    import ctypes as C
    from . import _check, lib

    L = lib()
    h = C.c_void_p()
    _check(L.crdt_trace_load(os.fsencode(path), C.byref(h)), "crdt_trace_load")
    try:
        sz = np.zeros(7, np.uint64)
        _check(L.crdt_trace_sizes(h, sz.ctypes.data_as(C.POINTER(C.c_uint64))), "crdt_trace_sizes")
        n_txns, n_patches, text_b, start_len, start_b, end_len, end_b = (int(x) for x in sz)
        counts = np.zeros(n_txns, np.uint32)
        patches = np.zeros((n_patches, 3), np.uint32)
        text = C.create_string_buffer(max(text_b, 1))
        start = C.create_string_buffer(max(start_b, 1))
        end = C.create_string_buffer(max(end_b, 1))
        _check(L.crdt_trace_copy(h, counts.ctypes.data, patches.ctypes.data, text, start, end), "crdt_trace_copy")
    finally:
        L.crdt_trace_free(h)
    end_bytes = end.raw[:end_b]
    tr = Trace(os.path.basename(path).split(".")[0], counts, patches, start_len, end_len, end_b,
               fnv1a64(end_bytes), text.raw[:text_b])
    tr.start = start.raw[:start_b]
    tr.end = end_bytes
    return tr
