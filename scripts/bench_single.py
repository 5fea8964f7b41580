"""Single-document latency: one document replayed by one wave (the reference's own single-document
benches), next to one host thread on the oracle.

Workloads: `ap` = config 1, automerge-paper as local txns (benches/yjs.rs:41-48); `ap_remote` =
the same trace as one remote wire (config 2's per-document work, one document); `kevin` = 5 M
single-char front inserts (benches/yjs.rs:51-62).  GPU: the k_replay HIP-event time of one clean
launch (reset + replay, best of --reps), inputs resident.  CPU: the oracle (C++ restatement of the
reference's B-tree path, leaf 32 / node 16, SplitList index) on one host thread, best of --reps.
Parity: the GPU document's digest equals the oracle's.  Prints one JSON line per workload in the
bench schema (value = GPU ms, lower is better; bench.py stays the driver's bench)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

ap = argparse.ArgumentParser()
ap.add_argument("--workloads", default="ap,ap_remote,kevin")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire, load_trace  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def gpu_ms(e, reps):
    ev = [C.c_void_p() for _ in range(2)]
    for x in ev:
        hip.hipEventCreate(C.byref(x))
    s_ = C.c_void_p(e.stream())
    ms = []
    for _ in range(reps):
        e.reset_async()
        hip.hipEventRecord(ev[0], s_)
        e.run_async()
        hip.hipEventRecord(ev[1], s_)
        e.sync()
        x = C.c_float()
        hip.hipEventElapsedTime(C.byref(x), ev[0], ev[1])
        ms.append(x.value)
    assert (e.status() == 0).all()
    return min(ms)


def cpu_ms(fn, reps):
    best, dg = None, None
    for _ in range(reps):
        o = OracleDoc(32, 16, split_index=True)
        t0 = time.perf_counter()
        fn(o)
        dt = (time.perf_counter() - t0) * 1e3
        best = dt if best is None else min(best, dt)
        dg = o.digest()
    return best, dg


for wl in a.workloads.split(","):
    e = crdt_amd.Engine(1, 32)
    if wl == "ap":
        t = load_trace("automerge-paper")
        ag = e.agent_intern([0], ["jeremy"])
        e.apply_trace([0], int(ag[0]), t.counts, t.patches, stage_only=True)
        ops = int(np.asarray(t.counts).sum())
        cms, odg = cpu_ms(lambda o: o.apply_trace(o.agent("jeremy"), t.counts, t.patches), a.reps)
        desc = "config1: automerge-paper as local txns (benches/yjs.rs:41-48), one document"
    elif wl == "ap_remote":
        w = load_remote_wire("automerge-paper")
        e.stage_remote_replicated(w, 0, ["u00000"])
        t = load_trace("automerge-paper")
        ops = int(np.asarray(t.counts).sum())
        cms, odg = cpu_ms(lambda o: o.apply_remote_wire(w), a.reps)
        desc = "automerge-paper as one remote wire (config 2's per-document work), one document"
    elif wl == "kevin":
        ops = 5_000_000
        cnt = np.ones(ops, np.uint32)
        pt = np.zeros((ops, 3), np.uint32)
        pt[:, 2] = 1
        ag = e.agent_intern([0], ["seph"])

        class T:
            counts = cnt
            patches = pt
        e.stage_local_shared([0], [0], int(ag[0]), [T])
        cms, odg = cpu_ms(lambda o: o.apply_trace(o.agent("seph"), cnt, pt), a.reps)
        desc = "kevin: 5M single-char front inserts (benches/yjs.rs:51-62), one document"
    else:
        raise SystemExit(f"unknown workload {wl}")
    st = e.run()
    assert (st == 0).all(), np.unique(st)
    e.fit()
    ms = gpu_ms(e, a.reps)
    ok = bool(int(e.digests()[0]) == int(odg))
    e.close()
    print(json.dumps({
        "build_id": crdt_amd.build_id(),
        "metric": f"single-document replay time ({wl})", "value": ms, "unit": "ms", "n_gpus": 1, "steps": a.reps,
        "higher_is_better": False, "dtype": "u32", "data": "reference trace" if wl != "kevin" else "synthetic (the bench's shape)",
        "config": {"workload": desc, "docs": 1, "ops": ops, "leaf_cap": 32},
        "ops_per_s": ops / (ms * 1e-3), "parity_ok": ok,
        "cpu_baseline": {"value": cms, "unit": "ms", "cores": 1, "kind": "port",
                         "sample": "the whole document on the oracle (reference B-tree restatement, leaf 32 / node 16, "
                                   "SplitList index), one host thread, best of %d" % a.reps},
        "gpu_over_cpu_time": ms / cms,
    }), flush=True)
