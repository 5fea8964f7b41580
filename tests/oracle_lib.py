"""ctypes wrapper over oracle/build/liboracle.so — TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

OK, ERR_POS_OOB, ERR_SEQ, ERR_UNKNOWN_AGENT, ERR_UNKNOWN_ID, ERR_NONTERMINATING = 0, -1, -2, -3, -4, -5
ERR_CAPACITY, ERR_EMPTY_TXN, ERR_FRONTIER, ERR_BAD_INPUT = -6, -7, -8, -9

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    vp, u32, u16, u64, i64 = C.c_void_p, C.c_uint32, C.c_uint16, C.c_uint64, C.c_int64
    P = C.POINTER
    L.orc_doc_new.restype = vp
    L.orc_doc_new.argtypes = [u32, u32, C.c_int]
    L.orc_doc_free.argtypes = [vp]
    L.orc_status.argtypes = [vp]
    L.orc_len.argtypes = [vp]
    L.orc_len.restype = u32
    L.orc_digest.argtypes = [vp]
    L.orc_digest.restype = u64
    L.orc_agent.argtypes = [vp, C.c_char_p]
    L.orc_apply_local.argtypes = [vp, u16, u32, P(u32)]
    L.orc_apply_local_trace.argtypes = [vp, u16, u32, P(u32), P(u32)]
    L.orc_apply_random.argtypes = [vp, u16, u32, u32]
    L.orc_apply_remote_wire.argtypes = [vp, C.c_char_p, C.c_size_t]
    L.orc_local_trace_to_wire.argtypes = [vp, u16, u32, P(u32), P(u32), C.c_void_p, i64]
    L.orc_local_trace_to_wire.restype = i64
    L.orc_sizes.argtypes = [vp, P(u64)]
    L.orc_export.argtypes = [vp] + [P(u32)] * 9
    L.orc_pos_to_loc.argtypes = [vp, u32, P(u32), P(u16), P(u32)]
    L.orc_loc_to_pos.argtypes = [vp, u32, P(u16), P(u32), P(u32), P(C.c_uint8)]
    L.orc_stats.argtypes = [vp, P(u64)]
    L.orc_text.argtypes = [vp, P(u32), u64, P(u32), u64, P(u64)]
    L.orc_text.restype = i64
    L.orc_cpu_baseline_random.argtypes = [u32, u32, u32, P(u32), P(u64), C.c_int]
    L.orc_cpu_baseline_random.restype = C.c_double
    L.orc_probe_trace.argtypes = [vp, u16, u32, P(u32), P(u32), P(u32), P(u32)]
    L.orc_dd_new.restype = vp
    L.orc_dd_free.argtypes = [vp]
    L.orc_dd_increment.argtypes = [vp, u32, u32]
    L.orc_dd_get.argtypes = [vp, P(u32), u32]
    L.orc_dd_get.restype = u32
    L.orc_cpu_baseline_local.argtypes = [u32, u32, u32, P(u32), P(u32), P(u64), C.c_int]
    L.orc_cpu_baseline_local.restype = C.c_double
    L.orc_cpu_baseline_remote.argtypes = [u32, u32, C.c_char_p, C.c_size_t, u32, P(C.c_char_p), P(u64), C.c_int]
    L.orc_cpu_baseline_remote.restype = C.c_double
    _lib = L
    return L


def _p(a, t=C.c_uint32):
    return a.ctypes.data_as(C.POINTER(t))


class OracleDoc:
    """One reference ListCRDT (restated).  leaf_cap/node_cap: 32/16 release, 4/8 debug."""

    def __init__(self, leaf_cap: int = 32, node_cap: int = 16, track_index: bool = True, split_index: bool = False):
        """split_index: the order index is the reference's SplitList (bucket 100) instead of a dense
        table (same answers; the CPU baseline uses it)."""
        self.L = lib()
        self.h = self.L.orc_doc_new(leaf_cap, node_cap, 2 if (track_index and split_index) else int(track_index))
        if not self.h:
            raise ValueError("bad caps")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_doc_free(self.h)
            self.h = None

    def agent(self, name: str) -> int:
        return self.L.orc_agent(self.h, name.encode())

    def apply_local(self, agent: int, ops) -> int:
        a = np.ascontiguousarray(np.asarray(ops, dtype=np.uint32).reshape(-1, 3))
        return self.L.orc_apply_local(self.h, agent, a.shape[0], _p(a))

    def local_insert(self, agent: int, pos: int, n: int) -> int:
        return self.apply_local(agent, [(pos, 0, n)])

    def local_delete(self, agent: int, pos: int, n: int) -> int:
        return self.apply_local(agent, [(pos, n, 0)])

    def apply_trace(self, agent: int, counts: np.ndarray, patches: np.ndarray) -> int:
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        p = np.ascontiguousarray(patches, dtype=np.uint32)
        return self.L.orc_apply_local_trace(self.h, agent, c.shape[0], _p(c), _p(p))

    def apply_remote_wire(self, wire: bytes) -> int:
        return self.L.orc_apply_remote_wire(self.h, wire, len(wire))

    def probe_trace(self, agent: int, counts, patches, probes):
        """apply the trace; after txn t answer pos_to_loc(probes[t,0]) and loc_to_pos(probes[t,1:3]);
        returns (status, answers [T, 4])"""
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        p = np.ascontiguousarray(patches, dtype=np.uint32)
        q = np.ascontiguousarray(probes, dtype=np.uint32).reshape(-1, 3)
        ans = np.zeros((c.shape[0], 4), np.uint32)
        st = self.L.orc_probe_trace(self.h, agent, c.shape[0], _p(c), _p(p), _p(q), _p(ans))
        return st, ans

    def apply_random(self, agent: int, n_ops: int, seed32: int) -> int:
        """config 4 generator (crdt_oracle.hpp random_change), n_ops local txns."""
        return self.L.orc_apply_random(self.h, agent, n_ops, seed32 & 0xFFFFFFFF)

    def trace_to_wire(self, agent: int, counts, patches) -> bytes:
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        p = np.ascontiguousarray(patches, dtype=np.uint32)
        n = self.L.orc_local_trace_to_wire(self.h, agent, c.shape[0], _p(c), _p(p), None, 0)
        if n < 0:
            raise RuntimeError(f"local->remote failed {n}")
        return n

    @property
    def status(self) -> int:
        return self.L.orc_status(self.h)

    def __len__(self) -> int:
        return int(self.L.orc_len(self.h))

    def digest(self) -> int:
        return int(self.L.orc_digest(self.h))

    def sizes(self) -> dict:
        s = np.zeros(12, dtype=np.uint64)
        self.L.orc_sizes(self.h, _p(s, C.c_uint64))
        keys = ["raw", "leaves", "canon", "cwo", "deletes", "dd", "txns", "parents", "frontier", "agents", "next_order", "len"]
        return {k: int(v) for k, v in zip(keys, s)}

    def export(self) -> dict:
        s = self.sizes()
        raw = np.zeros((s["raw"], 4), np.uint32)
        ls = np.zeros(s["leaves"], np.uint32)
        canon = np.zeros((s["canon"], 4), np.uint32)
        cwo = np.zeros((s["cwo"], 4), np.uint32)
        dels = np.zeros((s["deletes"], 3), np.uint32)
        dd = np.zeros((s["dd"], 3), np.uint32)
        txn = np.zeros((s["txns"], 5), np.uint32)
        par = np.zeros(s["parents"], np.uint32)
        fr = np.zeros(s["frontier"], np.uint32)
        self.L.orc_export(self.h, _p(raw), _p(ls), _p(canon), _p(cwo), _p(dels), _p(dd), _p(txn), _p(par), _p(fr))
        return dict(raw=raw, leaf_sizes=ls, canon=canon, cwo=cwo, deletes=dels, dd=dd, txns=txn,
                    parents=par, frontier=fr, len=s["len"], next_order=s["next_order"])

    def text(self, content):
        """(UTF-32 text, text digest) from an order-indexed content table (crdt_oracle.hpp text_of)."""
        c = np.ascontiguousarray(content, dtype=np.uint32)
        dg = np.zeros(1, np.uint64)
        n = self.L.orc_text(self.h, _p(c), c.shape[0], None, 0, _p(dg, C.c_uint64))
        if n < 0:
            raise ValueError("content table shorter than the document's orders")
        out = np.zeros(n, np.uint32)
        self.L.orc_text(self.h, _p(c), c.shape[0], _p(out), n, None)
        return out, int(dg[0])

    def pos_to_loc(self, pos):
        p = np.ascontiguousarray(pos, dtype=np.uint32)
        a = np.zeros(p.shape[0], np.uint16)
        q = np.zeros(p.shape[0], np.uint32)
        self.L.orc_pos_to_loc(self.h, p.shape[0], _p(p), _p(a, C.c_uint16), _p(q))
        return a, q

    def loc_to_pos(self, agent, seq):
        a = np.ascontiguousarray(agent, dtype=np.uint16)
        s = np.ascontiguousarray(seq, dtype=np.uint32)
        pos = np.zeros(a.shape[0], np.uint32)
        dl = np.zeros(a.shape[0], np.uint8)
        self.L.orc_loc_to_pos(self.h, a.shape[0], _p(a, C.c_uint16), _p(s), _p(pos), _p(dl, C.c_uint8))
        return pos, dl

    def stats(self) -> dict:
        s = np.zeros(3, np.uint64)
        self.L.orc_stats(self.h, _p(s, C.c_uint64))
        return dict(q2_triggers=int(s[0]), integrate_iters=int(s[1]), leaves_alloc=int(s[2]))


def trace_to_wire(counts, patches, agent_name: str = "jeremy", leaf_cap: int = 32) -> bytes:
    d = OracleDoc(leaf_cap, 16 if leaf_cap == 32 else 8)
    a = d.agent(agent_name)
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    p = np.ascontiguousarray(patches, dtype=np.uint32)
    n = d.L.orc_local_trace_to_wire(d.h, a, c.shape[0], _p(c), _p(p), None, 0)
    if n < 0:
        raise RuntimeError(f"local->remote failed {n}")
    d2 = OracleDoc(leaf_cap, 16 if leaf_cap == 32 else 8)
    a2 = d2.agent(agent_name)
    buf = C.create_string_buffer(int(n))
    m = d2.L.orc_local_trace_to_wire(d2.h, a2, c.shape[0], _p(c), _p(p), C.cast(buf, C.c_void_p), n)
    assert m == n
    return buf.raw


class DoubleDeletes:
    def __init__(self):
        self.L = lib()
        self.h = self.L.orc_dd_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_dd_free(self.h)

    def increment(self, base: int, n: int):
        self.L.orc_dd_increment(self.h, base, n)

    def get(self):
        out = np.zeros((256, 3), np.uint32)
        n = self.L.orc_dd_get(self.h, _p(out), 256)
        return [tuple(int(x) for x in r) for r in out[:n]]


# ---- layout sensitivity (the oracle at leaf 32 and leaf infinity, Q2 counted)
LEAF_UNBOUNDED = 0  # OracleDoc(LEAF_UNBOUNDED): one leaf that never splits (crdt_oracle.hpp L_UNBOUNDED)


def layout_items(ex: dict):
    """Item-level state of an exported document, in document order: (order, origin_left,
    origin_right, deleted) per item.  A run's first item carries the run's origin_left, the others
    their predecessor (span.rs:23-28 origin_left_at_offset)."""
    raw = ex["raw"].astype(np.int64)
    ln = np.abs(raw[:, 3].astype(np.int32)).astype(np.int64)
    ent = np.repeat(np.arange(raw.shape[0]), ln)
    off = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
    order = raw[ent, 0] + off
    ol = np.where(off == 0, raw[ent, 1], order - 1)
    return order, ol, raw[ent, 2], raw[ent, 3].astype(np.int32) < 0


def compare_layouts(a: dict, b: dict) -> dict:
    """Two exports of one history at different leaf layouts: same_order = the same items in the
    same document order with the same deleted flags; ol_diff / orr_diff = items whose stored
    origin differs (YjsSpan::prepend keeps the entry's origin_left, span.rs:61-64)."""
    oa, la, ra, da = layout_items(a)
    ob, lb, rb, db = layout_items(b)
    if oa.shape != ob.shape or not (np.array_equal(oa, ob) and np.array_equal(da, db)):
        return {"same_order": False}
    return {"same_order": True, "ol_diff": int((la != lb).sum()), "orr_diff": int((ra != rb).sum())}
