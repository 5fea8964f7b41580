"""The reference's "kevin" benchmark (benches/yjs.rs:51-62): ListCRDT::new(), then 5,000,000
local_insert(agent, 0, " ") -- every insert at the front of the document.

Timed lines (one MI355X), each replay = reset + one k_replay launch of the staged LC records:
  * single document: the reference's benchmark as written (one sequential chain, one wave);
  * `--docs` documents at once (each its own kevin history; the records are one shared device
    copy): the batch form the engine is built for.
Beside them the oracle (C++ restatement of the reference B-tree path, leaf 32 / node 16) replays
the same single document on one host thread, as criterion would time the Rust crate.  Parity: the
GPU digest equals the oracle's.  Prints one JSON line."""
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
ap.add_argument("--n", type=int, default=5_000_000)
ap.add_argument("--docs", type=int, default=512)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402

n = a.n
c = np.ones(n, np.uint32)
p = np.zeros((n, 3), np.uint32)
p[:, 2] = 1
hip = C.CDLL("libamdhip64.so")


def timed(e, reps):
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


o = OracleDoc(32, 16, split_index=True)
t0 = time.perf_counter()
assert o.apply_trace(o.agent("seph"), c, p) == 0
cpu_s = time.perf_counter() - t0
res = {}
for docs in (1, a.docs):
    e = crdt_amd.Engine(docs, 32)
    e.share_streams(True)
    ag = e.agent_intern(list(range(docs)), ["seph"] * docs)
    class T:  # one shared stream: the kevin trace
        counts = c
        patches = p
    e.stage_local_shared(list(range(docs)), [0] * docs, int(ag[0]), [T])
    st = e.run()
    assert (st == 0).all(), np.unique(st)
    e.fit()
    ms = timed(e, a.reps)
    dg = e.digests()
    res[docs] = {"docs": docs, "k_replay_ms": ms, "ops_per_s": docs * n / (ms * 1e-3),
                 "parity_ok": bool((dg == np.uint64(o.digest())).all()), "hbm_bytes": e.mem_bytes()}
    e.close()
print(json.dumps({
    "build_id": crdt_amd.build_id(),
    "metric": "kevin: 5M front inserts (benches/yjs.rs:51-62)", "unit": "ops/s", "ops_per_doc": n,
    "single_doc": res[1], "batch": res[a.docs],
    "cpu_single_thread": {"seconds": cpu_s, "ops_per_s": n / cpu_s, "kind": "port",
                          "sample": "one kevin document on the oracle (reference B-tree restatement, leaf 32 / node 16, "
                                    "SplitList index), one host thread"},
    "parity_ok": res[1]["parity_ok"] and res[a.docs]["parity_ok"],
}))
