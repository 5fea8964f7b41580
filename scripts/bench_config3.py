"""Secondary measurement: BASELINE config 3 shape (mixed corpus, local txns).

Document d replays trace [automerge-paper, rustcode, sveltecomponent][splitmix64(d) % 3] as local
txns (apply_local_txn path).  The three traces are encoded and uploaded once and copied per
document on the device (crdt_stage_local_shared).  One step = reset + replay + publish.  Parity:
every document's digest equals the committed oracle golden digest of its trace.  The CPU leg
times the oracle on a bounded sample.  Prints one JSON line (bench.py stays the driver's bench)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=8192)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--cpu-docs", type=int, default=768)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from crdt_amd.traces import load_trace  # noqa: E402
from bench import splitmix64  # noqa: E402

names = ["automerge-paper", "rustcode", "sveltecomponent"]
traces = [load_trace(n) for n in names]
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_golden.json")))
which = np.array([splitmix64(d) % 3 for d in range(a.docs)], np.uint32)
e = crdt_amd.Engine(a.docs, 32)
ag = e.agent_intern(list(range(a.docs)), ["jeremy"] * a.docs)
assert (ag == ag[0]).all()
t0 = time.time()
e.stage_local_shared(list(range(a.docs)), which, int(ag[0]), traces)
st = e.run()
assert (st == 0).all(), np.unique(st)
stage_s = time.time() - t0
ts, rms = [], []
for _ in range(a.steps):
    e.sync()
    t1 = time.perf_counter()
    e.reset_async()
    e.run_async()
    e.publish_async()
    e.sync()
    ts.append(time.perf_counter() - t1)
    rms.append(e.timings()[0])
dg = e.digests()
want = np.array([int(gold[f"{names[k]}/L32"]["digest"], 16) for k in which], np.uint64)
ok = bool((e.status() == 0).all()) and bool((dg == want).all())
ops = int(sum(traces[k].n_patches for k in which))
# CPU leg: the oracle replaying the same traces (16 threads), a bounded sample per trace
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes as C  # noqa: E402
from oracle_lib import lib as olib  # noqa: E402
L = olib()
cpu_ops, cpu_s = 0, 0.0
for k, t in enumerate(traces):
    n = max(1, int(round(a.cpu_docs * (which == k).mean())))
    c = np.ascontiguousarray(t.counts, np.uint32)
    p = np.ascontiguousarray(t.patches, np.uint32)
    ck = C.c_uint64()
    L.orc_cpu_baseline_local.restype = C.c_double
    s = L.orc_cpu_baseline_local(n, 16, c.shape[0], c.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 p.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(ck))
    cpu_ops += n * t.n_patches
    cpu_s += s
t = min(ts)
print(json.dumps({
    "metric": "CRDT ops remapped+merged/sec (config 3: mixed local corpus)", "value": ops / t, "unit": "ops/s",
    "docs": a.docs, "ops": ops, "ms_per_step": t * 1e3,
    "mix": {n: int((which == k).sum()) for k, n in enumerate(names)},
    "cpu_sample": {"ops_per_s": cpu_ops / cpu_s, "threads": 16, "seconds": cpu_s},
    "parity_ok": ok, "stage_s": stage_s,
}))
