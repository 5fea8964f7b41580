"""ctypes wrapper over tests/emu/build/libemu.so — TEST INFRASTRUCTURE.

The emulator runs the product's replay_core.h control logic on the CPU (WaveCPU backend) so the
GPU algorithm can be diffed against the oracle in the CPU-only test suite.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
EMU_DIR = os.path.join(ROOT, "tests", "emu")
LIB_PATH = os.environ.get("CRDT_EMU_LIB") or os.path.join(EMU_DIR, "build", "libemu.so")  # (env: a coverage build)
_lib = None


def build() -> None:
    # (one make at a time: parallel test workers must not load a library another one is writing)
    import fcntl
    os.makedirs(os.path.join(EMU_DIR, "build"), exist_ok=True)
    with open(os.path.join(EMU_DIR, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", EMU_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        u32, u16, vp, P = C.c_uint32, C.c_uint16, C.c_void_p, C.POINTER
        L.emu_new.restype = vp
        L.emu_new.argtypes = [u32]
        L.emu_free.argtypes = [vp]
        L.emu_agent.argtypes = [vp, C.c_char_p]
        L.emu_run_local.argtypes = [vp, u16, u32, P(u32), P(u32), u32]
        L.emu_run_wire.argtypes = [vp, C.c_char_p, C.c_size_t, u32]
        L.emu_run_wire_local.argtypes = [vp, C.c_char_p, C.c_size_t, C.c_char_p, u32, P(u32), P(u32), u32]
        L.emu_run_random.argtypes = [vp, u16, u32, u32, u32]
        L.emu_run_local_probed.argtypes = [vp, u16, u32, P(u32), P(u32), P(u32), P(u32), u32]
        L.emu_sizes.argtypes = [vp, P(C.c_uint64)]
        L.emu_export.argtypes = [vp] + [P(u32)] * 8
        L.emu_check.argtypes = [vp, C.c_char_p, C.c_int]
        _lib = L
    return _lib


def _p(a, t=C.c_uint32):
    return a.ctypes.data_as(C.POINTER(t))


class EmuDoc:
    def __init__(self, leaf_cap: int = 32):
        self.L = lib()
        self.h = self.L.emu_new(leaf_cap)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.emu_free(self.h)

    def agent(self, name: str) -> int:
        return self.L.emu_agent(self.h, name.encode())

    def run_local(self, agent, counts, patches, leaf_div: int = 48) -> int:
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        p = np.ascontiguousarray(patches, dtype=np.uint32)
        return self.L.emu_run_local(self.h, agent, c.shape[0], _p(c), _p(p), leaf_div)

    def run_local_probed(self, agent, counts, patches, probes, leaf_div: int = 48):
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        p = np.ascontiguousarray(patches, dtype=np.uint32)
        q = np.ascontiguousarray(probes, dtype=np.uint32).reshape(-1, 3)
        ans = np.zeros((c.shape[0], 4), np.uint32)
        st = self.L.emu_run_local_probed(self.h, agent, c.shape[0], _p(c), _p(p), _p(q), _p(ans), leaf_div)
        return st, ans

    def run_wire_local(self, wire: bytes, name: str, counts, patches, leaf_div: int = 48) -> int:
        c = np.ascontiguousarray(counts, np.uint32)
        p = np.ascontiguousarray(patches, np.uint32)
        return self.L.emu_run_wire_local(self.h, wire, len(wire), name.encode(), c.shape[0], _p(c), _p(p), leaf_div)

    def run_wire(self, wire: bytes, leaf_div: int = 48) -> int:
        return self.L.emu_run_wire(self.h, wire, len(wire), leaf_div)

    def run_random(self, agent: int, n_ops: int, seed32: int, leaf_div: int = 48) -> int:
        return self.L.emu_run_random(self.h, agent, n_ops, seed32 & 0xFFFFFFFF, leaf_div)

    def check(self) -> str:
        buf = C.create_string_buffer(512)
        r = self.L.emu_check(self.h, buf, 512)
        return "" if r == 0 else buf.value.decode()

    def sizes(self) -> dict:
        s = np.zeros(14, np.uint64)
        self.L.emu_sizes(self.h, _p(s, C.c_uint64))
        k = ["raw", "leaves", "cwo", "deletes", "dd", "txns", "parents", "frontier", "agents", "next_order", "len", "rec_pos",
             "grow_events", "grow_mask"]
        return {a: int(b) for a, b in zip(k, s)}

    def export(self) -> dict:
        s = self.sizes()
        raw = np.zeros((s["raw"], 4), np.uint32)
        ls = np.zeros(s["leaves"], np.uint32)
        cwo = np.zeros((s["cwo"], 4), np.uint32)
        dl = np.zeros((s["deletes"], 3), np.uint32)
        dd = np.zeros((s["dd"], 3), np.uint32)
        tx = np.zeros((s["txns"], 5), np.uint32)
        pa = np.zeros(s["parents"], np.uint32)
        fr = np.zeros(s["frontier"], np.uint32)
        self.L.emu_export(self.h, _p(raw), _p(ls), _p(cwo), _p(dl), _p(dd), _p(tx), _p(pa), _p(fr))
        return dict(raw=raw, leaf_sizes=ls, cwo=cwo, deletes=dl, dd=dd, txns=tx, parents=pa, frontier=fr,
                    len=s["len"], next_order=s["next_order"])


def diff_states(a: dict, b: dict, keys=("raw", "leaf_sizes", "cwo", "deletes", "dd", "txns", "parents", "frontier", "len", "next_order")):
    """Return list of mismatching keys (with first differing index for arrays)."""
    bad = []
    for k in keys:
        x, y = a[k], b[k]
        if isinstance(x, np.ndarray):
            if x.shape != y.shape:
                bad.append(f"{k}: shape {x.shape} vs {y.shape}")
            elif not np.array_equal(x, y):
                i = int(np.argwhere(x != y)[0][0])
                bad.append(f"{k}: first diff at {i}: {x[i]} vs {y[i]}")
        elif x != y:
            bad.append(f"{k}: {x} vs {y}")
    return bad
