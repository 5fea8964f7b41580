"""crdt_amd — Python binding of the MI355X list-CRDT engine (include/crdt_gpu.h).

The product is the C ABI library text-crdt-rust_amd/build/libcrdt_gpu.so (HIP kernels for gfx950 +
C++ host).  This module is a thin ctypes layer used by tests and bench.py; it mirrors the
reference's `ListCRDT` surface (src/list/doc.rs) for one document (`ListCRDT`) and exposes the
batched many-document form (`Engine`).  There is no CPU fallback: without the built library or a
gfx950 device every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Iterable, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(PKG_DIR)
REPO = os.path.dirname(PKG_ROOT)
LIB_PATH = os.path.join(PKG_ROOT, "build", "libcrdt_gpu.so")
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")

OK = 0
STATUS_NAMES = {0: "OK", -1: "POS_OOB", -2: "SEQ", -3: "UNKNOWN_AGENT", -4: "UNKNOWN_ID", -5: "NONTERMINATING",
                -6: "CAPACITY", -7: "EMPTY_TXN", -8: "FRONTIER", -9: "BAD_INPUT", -10: "INTERNAL"}
ROOT_AGENT = 0xFFFF
ROOT_ORDER = 0xFFFFFFFF


class CrdtError(RuntimeError):
    pass


def _build_cmd(out: str, defines: Sequence[str]) -> list:
    # Codegen options for the replay's wave-uniform control flow (measured on k_replay, 8,192 AP
    # documents, scripts/gpu_ab.sh):
    #  -phi-elim-split-all-critical-edges: the fast paths have many early exits into one shared
    #   "not applicable" block; without edge splitting the register copies that block's phis need
    #   are placed before every conditional branch and run whether it is taken or not (118 -> 110 ms);
    #  -structurizecfg-skip-uniform-regions: uniform branches stay plain s_cbranch_scc jumps instead
    #   of being structurized into exec-mask flow blocks with 64-bit boolean phis (109 -> 99 ms).
    return ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-fno-strict-aliasing", "-mllvm", "-phi-elim-split-all-critical-edges=1",
            "-mllvm", "-structurizecfg-skip-uniform-regions=1", "-I" + INCLUDE, "-I" + CSRC, "-o", out + ".tmp"] + [
            "-D" + d for d in defines] + [os.path.join(CSRC, "engine.hip"), os.path.join(CSRC, "trace_ingest.cpp"), "-lz"]


def source_hash(defines: Sequence[str] = ()) -> str:
    """sha256 (16 hex digits) over every source the library is built from (csrc/*, the public
    headers) and the build line: what build() keys a rebuild on, embedded in the library
    (crdt_build_id) and printed by __graft_entry__.smoke()."""
    import hashlib
    h = hashlib.sha256()
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)) + [os.path.join(INCLUDE, x) for x in ("crdt_gpu.h", "crdt_trace.h")]
    for p in srcs:
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join(_build_cmd("OUT", defines)[1:]).replace(REPO, "").encode())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False, out: str = LIB_PATH, defines: Sequence[str] = ()) -> str:
    """Compile libcrdt_gpu.so for gfx950 with hipcc (in-tree).  The rebuild is keyed on
    source_hash() (sources + build line), stored beside the library (`out` + ".srchash") and
    embedded in it (crdt_build_id), not on file times.  `defines` only for diagnostic builds
    written to another `out` (e.g. CRDT_PROF)."""
    hsh = source_hash(defines)
    stamp = out + ".srchash"
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == hsh:
                return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = _build_cmd(out, list(defines) + [f'CRDT_SRC_HASH="{hsh}"'])
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise CrdtError("hipcc failed:\n" + (r.stderr or "")[-4000:])
    if not defines:  # (diagnostic builds, e.g. CRDT_PROF, may spill: they are never the product)
        check_codegen(out + ".tmp")
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(hsh + "\n")
    return out


def build_id(path: str = None) -> str:
    """crdt_build_id() of the library `path` (default: the one lib() loads)."""
    L = lib() if path is None else C.CDLL(path)
    L.crdt_build_id.restype = C.c_char_p
    return L.crdt_build_id().decode()


# The replay's speed rests on its register budget: 8 waves per SIMD need <= 64 VGPRs (the 512-
# VGPR file / 8), and a scratch spill of a value the replay loop updates would put memory round
# trips into every context access.  A toolchain change that breaks either would silently halve
# throughput (97 VGPRs = 4 waves/SIMD = 216 ms vs 185 ms), so build() refuses such
# a library.  k_replay may keep ONE 16-byte spill slot with at most 4 stores in the whole kernel:
# at 64 VGPRs the allocator spills a register quad holding the constant half {32, 0} of the
# double-delete block record that dd_insert's block split writes (stored at kernel entry and in
# the three inlined copies of that split, once per 32 double-delete entries; reloaded on the same
# rare paths).  Same-box A/B: no cost.  A spill of a value the replay loop updates
# would show up as more scratch stores.
SCRATCH_STORES_MAX = {"k_replay": 4}
CODEGEN_LIMITS = {
    "k_replay": {"vgpr_count": 64, "vgpr_spill_count": 16, "private_segment_fixed_size": 32},
    # the two-level-root instance (documents past the LDS root) runs at 4 waves per SIMD
    "k_replay_hr": {"vgpr_count": 128, "vgpr_spill_count": 0, "private_segment_fixed_size": 0},
    "k_publish": {"vgpr_count": 64, "vgpr_spill_count": 0, "private_segment_fixed_size": 0},
}
LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def kernel_resources(lib_path: str) -> dict:
    """Per-kernel resource metadata of the gfx950 code object inside `lib_path` (the AMDGPU
    metadata note: .vgpr_count, .sgpr_count, spills, .private_segment_fixed_size, LDS)."""
    import re
    import tempfile
    import shutil
    with tempfile.TemporaryDirectory() as td:
        # the HIP fat binary sits in the library's .hip_fatbin section; llvm-objdump --offloading
        # extracts its bundles next to the (copied) input
        cp = os.path.join(td, "lib.so")
        shutil.copyfile(lib_path, cp)
        r = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "--offloading", cp], capture_output=True, text=True)
        cos = [f for f in os.listdir(td) if "amdgcn-amd-amdhsa--gfx950" in f]
        if r.returncode != 0 or not cos:
            raise CrdtError("no gfx950 code object in " + lib_path + ": " + (r.stderr or "")[-500:])
        notes = subprocess.run([os.path.join(LLVM_BIN, "llvm-readelf"), "--notes", os.path.join(td, cos[0])],
                               capture_output=True, text=True, check=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)\s*$", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if line.lstrip().startswith("- "):
            cur = {}
        if k == "name":
            out[v] = cur
        elif re.fullmatch(r"-?\d+", v):
            cur[k] = int(v)
    return out


def scratch_stores(lib_path: str) -> dict:
    """Scratch store instructions per kernel of the gfx950 code object inside `lib_path`."""
    import re
    import tempfile
    import shutil
    with tempfile.TemporaryDirectory() as td:
        cp = os.path.join(td, "lib.so")
        shutil.copyfile(lib_path, cp)
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "--offloading", cp], capture_output=True, text=True)
        cos = [f for f in os.listdir(td) if "amdgcn-amd-amdhsa--gfx950" in f]
        if not cos:
            raise CrdtError("no gfx950 code object in " + lib_path)
        dis = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--no-show-raw-insn", os.path.join(td, cos[0])],
                             capture_output=True, text=True, check=True).stdout
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = 0
        elif cur and ("scratch_store" in line or "buffer_store" in line and "off, s[0:3]" in line):
            out[cur] += 1
    return out


def check_codegen(lib_path: str) -> dict:
    """Raise CrdtError if a guarded kernel exceeds CODEGEN_LIMITS (or SCRATCH_STORES_MAX); returns
    the guarded kernels' resources."""
    res = kernel_resources(lib_path)
    ss = scratch_stores(lib_path)
    for name, n in ss.items():
        for k, mx in SCRATCH_STORES_MAX.items():
            if f"{len(k)}{k}I" in name and n > mx:
                raise CrdtError(f"codegen guard: {name} has {n} scratch stores > {mx} (a spill inside the replay loop; "
                                f"see DESIGN.md §4)")
    seen = {}
    for name, r in res.items():
        for k, lim in CODEGEN_LIMITS.items():
            if f"{len(k)}{k}I" not in name:  # mangled template name, e.g. _ZN4crdt8k_replayILi32EE...
                continue
            seen[name] = r
            for field, mx in lim.items():
                if r.get(field, 0) > mx:
                    raise CrdtError(f"codegen guard: {name} {field} = {r.get(field)} > {mx} "
                                    f"(the replay's 8-waves/SIMD register budget; see DESIGN.md §4)")
    for k in CODEGEN_LIMITS:
        if not any(f"{len(k)}{k}I" in n for n in seen):
            raise CrdtError(f"codegen guard: kernel {k} not found in {lib_path}")
    return seen


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("CRDT_GPU_LIB", LIB_PATH)  # diagnostic builds only (e.g. -DCRDT_PROF)
    if not os.path.exists(path):
        raise CrdtError(f"{path} not built (run __graft_entry__.build())")
    L = C.CDLL(path)
    if path != LIB_PATH:  # a diagnostic library from an older tree may lack later entry points
        class _Missing:
            def __init__(self, name):
                self.name = name

            def __call__(self, *a):
                raise CrdtError(f"{self.name}: not in {path}")
        for name in EXPORTED_SYMBOLS:
            if not hasattr(L, name):
                setattr(L, name, _Missing(name))
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    P = C.POINTER

    class Cfg(C.Structure):
        _fields_ = [("leaf_cap", C.c_uint32), ("device", C.c_int32)]
    L.Cfg = Cfg
    L.crdt_engine_create.argtypes = [P(Cfg), P(vp)]
    L.crdt_engine_destroy.argtypes = [vp]
    L.crdt_docs_alloc.argtypes = [vp, u64]
    L.crdt_num_docs.argtypes = [vp]
    L.crdt_num_docs.restype = u64
    L.crdt_agent_intern.argtypes = [vp, u64, P(u32), P(C.c_char_p), P(C.c_uint16)]
    L.crdt_agent_intern_dev.argtypes = [vp, u64, P(u32), P(u64), C.c_char_p, P(C.c_uint16), P(u32)]
    L.crdt_apply_local.argtypes = [vp, u64, P(u32), P(u64), vp, vp, P(i32)]
    L.crdt_stage_local.argtypes = [vp, u64, P(u32), P(u64), vp, vp]
    L.crdt_apply_remote_wire.argtypes = [vp, u64, P(u32), P(C.c_char_p), P(u64), P(i32)]
    L.crdt_stage_remote_wire.argtypes = [vp, u64, P(u32), P(C.c_char_p), P(u64)]
    L.crdt_stage_remote_replicated.argtypes = [vp, C.c_char_p, u64, u32, P(C.c_char_p)]
    L.crdt_stage_random.argtypes = [vp, u64, P(u32), C.c_char_p, u32, u64]
    L.crdt_stage_local_shared.argtypes = [vp, u64, P(u32), P(u32), u32, P(u64), vp, vp]
    L.crdt_debug_state.argtypes = [vp, u32, P(u32)]
    L.crdt_fit.argtypes = [vp]
    # (round-5 entry points; a diagnostic library from before them (CRDT_GPU_LIB) loads without them)
    for f, at in (("crdt_fit_note", [vp, C.c_int]), ("crdt_test_fail_alloc_after", [C.c_longlong]),
                  ("crdt_reseed_random_async", [vp, u64, u64]), ("crdt_digest_dev_async", [vp, vp])):
        if hasattr(L, f):
            getattr(L, f).argtypes = at
    L.crdt_set_share_streams.argtypes = [vp, C.c_int]
    for f in ("crdt_set_device_intern", "crdt_set_query_kernel"):
        if hasattr(L, f):  # (older libraries, for A/B runs, lack them)
            getattr(L, f).argtypes = [vp, C.c_int]
    L.crdt_apply_local_probed.argtypes = [vp, u64, P(u32), P(u64), vp, vp, vp, vp, P(i32)]
    L.crdt_mem_bytes.argtypes = [vp]
    L.crdt_mem_bytes.restype = u64
    if hasattr(L, "crdt_device_bytes"):  # (older libraries, for A/B runs, lack it)
        L.crdt_device_bytes.argtypes = [P(u64), P(u64), C.c_int]
    L.crdt_reset_async.argtypes = [vp]
    L.crdt_run.argtypes = [vp, P(i32)]
    L.crdt_run_async.argtypes = [vp]
    L.crdt_publish_async.argtypes = [vp]
    L.crdt_sync.argtypes = [vp]
    L.crdt_pos_to_loc.argtypes = [vp, u64, P(u32), P(u32), P(C.c_uint16), P(u32)]
    L.crdt_loc_to_pos.argtypes = [vp, u64, P(u32), P(C.c_uint16), P(u32), P(u32), P(C.c_uint8)]
    L.crdt_pos_to_loc_dev_async.argtypes = [vp, u64, vp, vp, vp, vp]
    L.crdt_loc_to_pos_dev_async.argtypes = [vp, u64, vp, vp, vp, vp, vp]
    L.crdt_doc_len.argtypes = [vp, u64, P(u32), P(u32)]
    L.crdt_doc_status.argtypes = [vp, P(i32)]
    L.crdt_digest.argtypes = [vp, P(u64)]
    if hasattr(L, "crdt_canon_counts"):  # (older libraries, for A/B runs, lack it)
        L.crdt_canon_counts.argtypes = [vp, P(u32)]
    L.crdt_export_sizes.argtypes = [vp, u32, P(u64)]
    L.crdt_export.argtypes = [vp, u32] + [P(u32)] * 9
    L.crdt_last_timings.argtypes = [vp, P(C.c_double), P(C.c_double)]
    L.crdt_stream.argtypes = [vp]
    L.crdt_stream.restype = vp
    L.crdt_set_content.argtypes = [vp, u64, P(u32), P(u32), u32, P(u64), P(u32)]
    L.crdt_materialize_async.argtypes = [vp]
    L.crdt_set_content_copies.argtypes = [vp, u64, P(u32), P(u32), u64]
    L.crdt_text.argtypes = [vp, u32, P(u32), u64, P(u64)]
    L.crdt_text_digest.argtypes = [vp, P(u64)]
    L.crdt_last_materialize_ms.argtypes = [vp, P(C.c_double)]
    L.crdt_last_error.restype = C.c_char_p
    L.crdt_trace_load.argtypes = [C.c_char_p, P(vp)]
    L.crdt_trace_parse.argtypes = [C.c_char_p, u64, P(vp)]
    L.crdt_trace_sizes.argtypes = [vp, P(u64)]
    L.crdt_trace_copy.argtypes = [vp, vp, vp, C.c_char_p, C.c_char_p, C.c_char_p]
    L.crdt_trace_free.argtypes = [vp]
    L.crdt_trace_free.restype = None
    _lib = L
    return L


EXPORTED_SYMBOLS = [
    "crdt_engine_create", "crdt_engine_destroy", "crdt_docs_alloc", "crdt_num_docs", "crdt_agent_intern", "crdt_agent_intern_dev",
    "crdt_apply_local", "crdt_apply_remote_wire", "crdt_stage_local", "crdt_stage_remote_wire",
    "crdt_stage_remote_replicated", "crdt_reset_async", "crdt_run", "crdt_run_async", "crdt_publish_async",
    "crdt_sync", "crdt_pos_to_loc", "crdt_loc_to_pos", "crdt_pos_to_loc_dev_async", "crdt_loc_to_pos_dev_async",
    "crdt_doc_len", "crdt_doc_status", "crdt_digest", "crdt_export_sizes", "crdt_export", "crdt_last_timings",
    "crdt_stream", "crdt_last_error", "crdt_build_id", "crdt_stage_random", "crdt_debug_state",
    "crdt_stage_local_shared", "crdt_set_content", "crdt_materialize_async", "crdt_text", "crdt_text_digest",
    "crdt_last_materialize_ms", "crdt_set_content_copies", "crdt_canon_counts", "crdt_fit", "crdt_mem_bytes", "crdt_apply_local_probed", "crdt_set_share_streams", "crdt_set_device_intern", "crdt_set_query_kernel", "crdt_device_bytes",
    "crdt_fit_note", "crdt_reseed_random_async", "crdt_digest_dev_async", "crdt_test_fail_alloc_after",
    # include/crdt_trace.h (host-only trace ingestion)
    "crdt_trace_load", "crdt_trace_parse", "crdt_trace_sizes", "crdt_trace_copy", "crdt_trace_free",
]


def _p(a, t=C.c_uint32):
    return a.ctypes.data_as(C.POINTER(t))


def _check(rc: int, what: str):
    if rc != 0:
        err = lib().crdt_last_error()
        raise CrdtError(f"{what} failed rc={rc} {err.decode() if err else ''}")


class Engine:
    """Many documents on one MI355X.  Mirrors ListCRDT per document (index `doc`)."""

    def __init__(self, n_docs: int, leaf_cap: int = 32, device: int = 0):
        L = lib()
        self.L = L
        self.h = C.c_void_p()
        cfg = L.Cfg(leaf_cap, device)
        _check(L.crdt_engine_create(C.byref(cfg), C.byref(self.h)), "crdt_engine_create")
        _check(L.crdt_docs_alloc(self.h, n_docs), "crdt_docs_alloc")
        self.n_docs = n_docs
        self.leaf_cap = leaf_cap

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.L.crdt_engine_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- ListCRDT::get_or_create_agent_id (doc.rs:66-80)
    def agent_intern(self, docs: Sequence[int], names: Sequence[str]) -> np.ndarray:
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        out = np.zeros(len(names), np.uint16)
        _check(self.L.crdt_agent_intern(self.h, len(names), _p(d), arr, _p(out, C.c_uint16)), "agent_intern")
        return out

    def agent_intern_dev(self, docs: Sequence[int], names: Sequence) -> tuple:
        """get_or_create_agent_id on the device (k_intern): (ids u16, ranks u32) per name; names
        are str or bytes (any bytes).  Same ids as agent_intern on the same call."""
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        bs = [n.encode() if isinstance(n, str) else bytes(n) for n in names]
        off = np.zeros(len(bs) + 1, np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
        blob = b"".join(bs)
        out = np.zeros(len(bs), np.uint16)
        rank = np.zeros(len(bs), np.uint32)
        _check(self.L.crdt_agent_intern_dev(self.h, len(bs), _p(d), _p(off, C.c_uint64), blob, _p(out, C.c_uint16),
                                            _p(rank)), "agent_intern_dev")
        return out, rank

    @staticmethod
    def _local_arrays(per_doc):
        """per_doc: list of (doc, [(agent, ops[(pos,del,ins)...]), ...])."""
        docs, txn_off, txns, ops = [], [0], [], []
        for doc, tx in per_doc:
            docs.append(doc)
            for agent, o in tx:
                o = np.asarray(o, dtype=np.uint32).reshape(-1, 3)
                txns.append((agent, o.shape[0]))
                ops.append(o)
            txn_off.append(len(txns))
        return (np.array(docs, np.uint32), np.array(txn_off, np.uint64),
                np.array(txns, np.uint32).reshape(-1, 2),
                np.concatenate(ops).astype(np.uint32) if ops else np.zeros((0, 3), np.uint32))

    def apply_local(self, per_doc) -> np.ndarray:
        return self.apply_local_arrays(*self._local_arrays(per_doc))

    def apply_local_probed(self, d, off, tx, ops, probes):
        """apply_local_arrays with one probe (pos, agent, seq) after every txn; returns (status,
        answers [T, 4] = (agent, seq) of pos, (pos, deleted) of (agent, seq))"""
        d = np.ascontiguousarray(d, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        tx = np.ascontiguousarray(tx, dtype=np.uint32).reshape(-1, 2)
        ops = np.ascontiguousarray(ops, dtype=np.uint32).reshape(-1, 3)
        pr = np.ascontiguousarray(probes, dtype=np.uint32).reshape(-1, 3)
        ans = np.zeros((tx.shape[0], 4), np.uint32)
        st = np.zeros(d.shape[0], np.int32)
        _check(self.L.crdt_apply_local_probed(self.h, d.shape[0], _p(d), _p(off, C.c_uint64), tx.ctypes.data,
                                              ops.ctypes.data, pr.ctypes.data, ans.ctypes.data, _p(st, C.c_int32)),
               "apply_local_probed")
        return st, ans

    def apply_local_arrays(self, d, off, tx, ops) -> np.ndarray:
        """crdt_apply_local on CSR arrays: docs [n], txn_off [n+1] (u64), txns [T,2] (agent, n_ops),
        ops [sum n_ops, 3] (pos, del, ins)."""
        d = np.ascontiguousarray(d, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        tx = np.ascontiguousarray(tx, dtype=np.uint32).reshape(-1, 2)
        ops = np.ascontiguousarray(ops, dtype=np.uint32).reshape(-1, 3)
        st = np.zeros(d.shape[0], np.int32)
        _check(self.L.crdt_apply_local(self.h, d.shape[0], _p(d), _p(off, C.c_uint64), tx.ctypes.data,
                                       ops.ctypes.data, _p(st, C.c_int32)), "apply_local")
        return st

    def apply_trace(self, docs: Sequence[int], agent: int | Sequence[int], counts: np.ndarray, patches: np.ndarray,
                    stage_only: bool = False) -> np.ndarray:
        """Apply the same trace (txn patch counts + patches) to every doc in `docs`."""
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        n = d.shape[0]
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        agents = np.broadcast_to(np.asarray(agent, dtype=np.uint32), (n,))
        tx = np.zeros((n * counts.shape[0], 2), np.uint32)
        for i in range(n):
            tx[i * counts.shape[0]:(i + 1) * counts.shape[0], 0] = agents[i]
            tx[i * counts.shape[0]:(i + 1) * counts.shape[0], 1] = counts
        off = (np.arange(n + 1, dtype=np.uint64) * counts.shape[0]).astype(np.uint64)
        ops = np.ascontiguousarray(np.tile(np.asarray(patches, np.uint32).reshape(-1, 3), (n, 1)))
        if stage_only:
            _check(self.L.crdt_stage_local(self.h, n, _p(d), _p(off, C.c_uint64), tx.ctypes.data, ops.ctypes.data),
                   "stage_local")
            return np.zeros(n, np.int32)
        st = np.zeros(n, np.int32)
        _check(self.L.crdt_apply_local(self.h, n, _p(d), _p(off, C.c_uint64), tx.ctypes.data, ops.ctypes.data,
                                       _p(st, C.c_int32)), "apply_local")
        return st

    def apply_remote_wire(self, docs: Sequence[int], wires: Sequence[bytes], stage_only: bool = False) -> np.ndarray:
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        arr = (C.c_char_p * len(wires))(*wires)
        ln = np.array([len(w) for w in wires], np.uint64)
        if stage_only:
            _check(self.L.crdt_stage_remote_wire(self.h, d.shape[0], _p(d), arr, _p(ln, C.c_uint64)), "stage_remote")
            return np.zeros(d.shape[0], np.int32)
        st = np.zeros(d.shape[0], np.int32)
        _check(self.L.crdt_apply_remote_wire(self.h, d.shape[0], _p(d), arr, _p(ln, C.c_uint64), _p(st, C.c_int32)),
               "apply_remote_wire")
        return st

    def stage_remote_replicated(self, wire: bytes, rename_idx: int, names: Sequence[str]):
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        _check(self.L.crdt_stage_remote_replicated(self.h, wire, len(wire), rename_idx, arr), "stage_replicated")

    # --- shared local streams (config 3 corpora): doc i replays traces[stream_of_doc[i]] as `agent`
    def stage_local_shared(self, docs: Sequence[int], stream_of_doc: Sequence[int], agent: int, traces) -> None:
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        so = np.ascontiguousarray(stream_of_doc, dtype=np.uint32)
        txn_off = np.concatenate([[0], np.cumsum([t.counts.shape[0] for t in traces])]).astype(np.uint64)
        tx = np.zeros((int(txn_off[-1]), 2), np.uint32)
        tx[:, 0] = agent
        tx[:, 1] = np.concatenate([t.counts for t in traces])
        ops = np.ascontiguousarray(np.concatenate([np.asarray(t.patches, np.uint32).reshape(-1, 3) for t in traces]))
        _check(self.L.crdt_stage_local_shared(self.h, d.shape[0], _p(d), _p(so), len(traces), _p(txn_off, C.c_uint64),
                                              tx.ctypes.data, ops.ctypes.data), "stage_local_shared")

    # --- config 4: make_random_change (doc.rs:544-569) generated on the device
    def stage_random(self, docs: Sequence[int], agent: str, n_ops: int, seed: int):
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        _check(self.L.crdt_stage_random(self.h, d.shape[0], _p(d), agent.encode(), n_ops, seed), "stage_random")

    def apply_random(self, docs: Sequence[int], agent: str, n_ops: int, seed: int) -> np.ndarray:
        self.stage_random(docs, agent, n_ops, seed)
        st = self.run()
        return st[np.asarray(docs, dtype=np.int64)]

    def debug_state(self, doc: int) -> np.ndarray:
        out = np.zeros(23, np.uint32)
        _check(self.L.crdt_debug_state(self.h, doc, _p(out)), "debug_state")
        return out

    def fit(self):
        """shrink capacities to the staged streams' use (after run + publish)"""
        _check(self.L.crdt_fit(self.h), "fit")

    def fit_note(self, apply: bool = False):
        """apply=False: note the capacities fit() would set into each document's running maximum;
        apply=True: capacities = the noted maxima (config 4 corpus batches on one engine)"""
        _check(self.L.crdt_fit_note(self.h, int(apply)), "fit_note")

    def reseed_random_async(self, seed: int, id_base: int):
        """generated-edit documents (stage_random) become documents id_base + d of the corpus"""
        _check(self.L.crdt_reseed_random_async(self.h, C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), C.c_uint64(id_base)),
               "reseed_random_async")

    def digests_dev_async(self, dev_ptr: int):
        """copy the per-document digests to a device buffer (n_docs u64) on the engine stream"""
        _check(self.L.crdt_digest_dev_async(self.h, C.c_void_p(dev_ptr)), "digest_dev_async")

    def share_streams(self, on: bool = True):
        """documents staged from the same host stream read one device copy"""
        _check(self.L.crdt_set_share_streams(self.h, int(on)), "share_streams")

    QUERY_KERNELS = {"lds": 0, "per_thread": 1, "merge": 2}

    def query_kernel(self, mode: str):
        """kernels behind the device query entry points: "lds" (default), "per_thread", "merge"
        (sorted batches; same answers for any batch)"""
        _check(self.L.crdt_set_query_kernel(self.h, self.QUERY_KERNELS[mode]), "query_kernel")

    def device_intern(self, on: bool = True):
        """stage_remote_replicated interns every document's authors with k_intern (same ids)"""
        _check(self.L.crdt_set_device_intern(self.h, int(on)), "device_intern")

    def mem_bytes(self) -> int:
        """device bytes held by the per-document pools + staged records"""
        return int(self.L.crdt_mem_bytes(self.h))

    @staticmethod
    def device_bytes(reset_peak: bool = False):
        """(current, peak) device bytes held by this process's engines (crdt_device_bytes)"""
        cur, peak = C.c_uint64(), C.c_uint64()
        lib().crdt_device_bytes(C.byref(cur), C.byref(peak), int(reset_peak))
        return cur.value, peak.value

    def reset_async(self):
        _check(self.L.crdt_reset_async(self.h), "reset")

    def run(self) -> np.ndarray:
        st = np.zeros(self.n_docs, np.int32)
        _check(self.L.crdt_run(self.h, _p(st, C.c_int32)), "run")
        return st

    def run_async(self):
        _check(self.L.crdt_run_async(self.h), "run_async")

    def publish_async(self):
        _check(self.L.crdt_publish_async(self.h), "publish")

    def sync(self):
        _check(self.L.crdt_sync(self.h), "sync")

    def status(self) -> np.ndarray:
        st = np.zeros(self.n_docs, np.int32)
        _check(self.L.crdt_doc_status(self.h, _p(st, C.c_int32)), "status")
        return st

    def lens(self, docs=None) -> np.ndarray:
        d = np.arange(self.n_docs, dtype=np.uint32) if docs is None else np.ascontiguousarray(docs, dtype=np.uint32)
        out = np.zeros(d.shape[0], np.uint32)
        _check(self.L.crdt_doc_len(self.h, d.shape[0], _p(d), _p(out)), "doc_len")
        return out

    def digests(self) -> np.ndarray:
        out = np.zeros(self.n_docs, np.uint64)
        _check(self.L.crdt_digest(self.h, _p(out, C.c_uint64)), "digest")
        return out

    def canon_counts(self) -> np.ndarray:
        """canonical spans of every document's published index"""
        out = np.zeros(self.n_docs, np.uint32)
        _check(self.L.crdt_canon_counts(self.h, _p(out)), "canon_counts")
        return out

    def pos_to_loc(self, docs, pos):
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        p = np.ascontiguousarray(pos, dtype=np.uint32)
        a = np.zeros(p.shape[0], np.uint16)
        s = np.zeros(p.shape[0], np.uint32)
        _check(self.L.crdt_pos_to_loc(self.h, p.shape[0], _p(d), _p(p), _p(a, C.c_uint16), _p(s)), "pos_to_loc")
        return a, s

    def loc_to_pos(self, docs, agent, seq):
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        a = np.ascontiguousarray(agent, dtype=np.uint16)
        s = np.ascontiguousarray(seq, dtype=np.uint32)
        p = np.zeros(s.shape[0], np.uint32)
        dl = np.zeros(s.shape[0], np.uint8)
        _check(self.L.crdt_loc_to_pos(self.h, s.shape[0], _p(d), _p(a, C.c_uint16), _p(s), _p(p), _p(dl, C.c_uint8)),
               "loc_to_pos")
        return p, dl

    def export_sizes(self, doc: int) -> dict:
        s = np.zeros(12, np.uint64)
        _check(self.L.crdt_export_sizes(self.h, doc, _p(s, C.c_uint64)), "export_sizes")
        keys = ["raw", "leaves", "canon", "cwo", "deletes", "dd", "txns", "parents", "frontier", "agents",
                "next_order", "len"]
        return {k: int(v) for k, v in zip(keys, s)}

    def export(self, doc: int) -> dict:
        s = np.zeros(12, np.uint64)
        _check(self.L.crdt_export_sizes(self.h, doc, _p(s, C.c_uint64)), "export_sizes")
        n = [int(x) for x in s]
        raw = np.zeros((n[0], 4), np.uint32)
        ls = np.zeros(n[1], np.uint32)
        canon = np.zeros((n[2], 4), np.uint32)
        cwo = np.zeros((n[3], 4), np.uint32)
        dl = np.zeros((n[4], 3), np.uint32)
        dd = np.zeros((n[5], 3), np.uint32)
        tx = np.zeros((n[6], 5), np.uint32)
        pa = np.zeros(n[7], np.uint32)
        fr = np.zeros(n[8], np.uint32)
        _check(self.L.crdt_export(self.h, doc, _p(raw), _p(ls), _p(canon), _p(cwo), _p(dl), _p(dd), _p(tx), _p(pa),
                                  _p(fr)), "export")
        return dict(raw=raw, leaf_sizes=ls, canon=canon, cwo=cwo, deletes=dl, dd=dd, txns=tx, parents=pa,
                    frontier=fr, len=n[11], next_order=n[10])

    # --- text materialisation (ListCRDT::to_string with the rope on, doc.rs:498-505)
    def set_content(self, docs: Sequence[int], stream_of_doc: Sequence[int], streams: Sequence[np.ndarray]):
        """docs[i] reads the order-indexed UTF-32 table streams[stream_of_doc[i]]."""
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        so = np.ascontiguousarray(stream_of_doc, dtype=np.uint32)
        off = np.concatenate([[0], np.cumsum([len(x) for x in streams])]).astype(np.uint64)
        data = np.ascontiguousarray(np.concatenate([np.asarray(x, np.uint32) for x in streams])
                                    if streams else np.zeros(0, np.uint32))
        _check(self.L.crdt_set_content(self.h, d.shape[0], _p(d), _p(so), len(streams), _p(off, C.c_uint64),
                                       _p(data)), "set_content")

    def set_content_copies(self, docs: Sequence[int], content: np.ndarray):
        """every docs[i] gets its own device copy of one order-indexed UTF-32 table"""
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        c = np.ascontiguousarray(content, dtype=np.uint32)
        _check(self.L.crdt_set_content_copies(self.h, d.shape[0], _p(d), _p(c), c.shape[0]), "set_content_copies")

    def materialize_async(self):
        _check(self.L.crdt_materialize_async(self.h), "materialize")

    def text(self, doc: int) -> np.ndarray:
        n = C.c_uint64()
        _check(self.L.crdt_text(self.h, doc, None, 0, C.byref(n)), "text")
        out = np.zeros(n.value, np.uint32)
        _check(self.L.crdt_text(self.h, doc, _p(out), n.value, C.byref(n)), "text")
        return out

    def text_digests(self) -> np.ndarray:
        out = np.zeros(self.n_docs, np.uint64)
        _check(self.L.crdt_text_digest(self.h, _p(out, C.c_uint64)), "text_digest")
        return out

    def materialize_ms(self) -> float:
        x = C.c_double()
        self.L.crdt_last_materialize_ms(self.h, C.byref(x))
        return x.value

    def timings(self):
        a, b = C.c_double(), C.c_double()
        self.L.crdt_last_timings(self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def stream(self) -> int:
        return self.L.crdt_stream(self.h) or 0


class ListCRDT:
    """One document with the reference's method names (src/list/doc.rs), on its own engine."""

    def __init__(self, leaf_cap: int = 32, device: int = 0):
        self.e = Engine(1, leaf_cap, device)

    def get_or_create_agent_id(self, name: str) -> int:         # doc.rs:66
        return int(self.e.agent_intern([0], [name])[0])

    def apply_local_txn(self, agent: int, ops) -> int:          # doc.rs:376
        return int(self.e.apply_local([(0, [(agent, ops)])])[0])

    def local_insert(self, agent: int, pos: int, ins_len: int) -> int:   # doc.rs:472
        return self.apply_local_txn(agent, [(pos, 0, ins_len)])

    def local_delete(self, agent: int, pos: int, del_span: int) -> int:  # doc.rs:478
        return self.apply_local_txn(agent, [(pos, del_span, 0)])

    def apply_remote_wire(self, wire: bytes) -> int:            # doc.rs:242 (batch of RemoteTxn)
        return int(self.e.apply_remote_wire([0], [wire])[0])

    def set_content(self, content: np.ndarray):
        self.e.set_content([0], [0], [content])

    def to_string(self) -> str:                                 # doc.rs:498-505 (rope on)
        from .traces import utf32_to_str
        return utf32_to_str(self.e.text(0))

    def __len__(self) -> int:                                   # doc.rs:484
        return int(self.e.lens([0])[0])

    def status(self) -> int:
        return int(self.e.status()[0])
