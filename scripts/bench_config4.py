"""Secondary measurement: BASELINE config 4 shape (random-edit documents generated on the device).

Each document replays `--ops` local txns drawn inside the replay wave from one GEN record
(make_random_change semantics, doc.rs:544-569).  One step = reset + replay + publish.  Prints one
JSON line.  Not the driver's bench (bench.py is); the CPU leg replays a bounded sample of the same
documents with the oracle (test infrastructure, used only as the baseline)."""
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
ap.add_argument("--docs", type=int, default=32768)
ap.add_argument("--ops", type=int, default=20000)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--seed", type=int, default=0xC0FFEE)
ap.add_argument("--cpu-docs", type=int, default=64)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from bench import splitmix64  # noqa: E402

e = crdt_amd.Engine(a.docs, 32)
t0 = time.time()
e.stage_random(list(range(a.docs)), "gen", a.ops, a.seed)
st = e.run()  # untimed: capacity growth
assert (st == 0).all(), np.unique(st)
e.publish_async()
e.sync()
dg0 = e.digests().copy()
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
ok = bool((e.status() == 0).all()) and bool((e.digests() == dg0).all())
# CPU leg: the oracle on a sample of the same documents (one thread per doc via a pool of 16)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from concurrent.futures import ThreadPoolExecutor  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402


def one(d):
    o = OracleDoc()
    assert o.apply_random(o.agent("gen"), a.ops, splitmix64(a.seed ^ d) & 0xFFFFFFFF) == 0
    return o.digest()


c0 = time.perf_counter()
with ThreadPoolExecutor(16) as ex:
    cdg = list(ex.map(one, range(a.cpu_docs)))
csec = time.perf_counter() - c0
ok = ok and all(int(dg0[d]) == cdg[d] for d in range(a.cpu_docs))
t = min(ts)
print(json.dumps({
    "metric": "CRDT ops remapped+merged/sec (config 4: on-device random edits)", "value": a.docs * a.ops / t,
    "unit": "ops/s", "docs": a.docs, "ops_per_doc": a.ops, "ms_per_step": t * 1e3,
    "cpu_sample": {"docs": a.cpu_docs, "threads": 16, "ops_per_s": a.cpu_docs * a.ops / csec,
                   "note": "oracle C++ restatement via ctypes threads (GIL released in C)"},
    "parity_ok": ok, "stage_s": time.time() - t0 - sum(ts) - csec,
}))
