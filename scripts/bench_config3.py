"""Secondary measurement: BASELINE config 3 (mixed corpus of 65,536 documents, local txns, 1 GPU).

Document d replays trace [automerge-paper, rustcode, sveltecomponent][splitmix64(d) % 3] as local
txns (apply_local_txn path; variable lengths -> ragged work per wave).  The three traces are
encoded once; with --share (default) the documents of one trace read one device copy of its
record stream (read-only input), which is what lets 65,536 documents' state fit one MI355X;
--no-share gives every document its own copy.  Every document keeps its own state.  One step =
reset + replay + publish (every document's flat position index).  Parity: every document's
digest equals the committed oracle golden digest of its trace.  The CPU leg times the oracle
(restatement of the reference B-tree path, SplitList order index) on a bounded sample with every
host core this process may use.  Prints one JSON line (bench.py stays the driver's bench)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=65536)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--share", dest="share", action="store_true", default=True)
ap.add_argument("--no-share", dest="share", action="store_false")
ap.add_argument("--cpu-seconds", type=float, default=15.0)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from crdt_amd.traces import load_trace  # noqa: E402
from bench import splitmix64, cpu_share, cpu_baseline_local, sampled, measured_traffic, SIMDS, HBM_PEAK_GBS  # noqa: E402

names = ["automerge-paper", "rustcode", "sveltecomponent"]
traces = [load_trace(n) for n in names]
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_golden.json")))
which = np.array([splitmix64(d) % 3 for d in range(a.docs)], np.uint32)
e = crdt_amd.Engine(a.docs, 32)
if a.share:
    e.share_streams(True)
ag = e.agent_intern(list(range(a.docs)), ["jeremy"] * a.docs)
assert (ag == ag[0]).all()
t0 = time.time()
e.stage_local_shared(list(range(a.docs)), which, int(ag[0]), traces)
st = e.run()  # untimed: capacity growth, index sizing
assert (st == 0).all(), np.unique(st)
e.publish_async()
e.sync()
stage_s = time.time() - t0
mem = e.mem_bytes()
hip = C.CDLL("libamdhip64.so")
ev = [C.c_void_p() for _ in range(4)]
for x in ev:
    hip.hipEventCreate(C.byref(x))
s_ = C.c_void_p(e.stream())
ts, rms, pms = [], [], []
for _ in range(a.steps):
    e.sync()
    t1 = time.perf_counter()
    e.reset_async()
    hip.hipEventRecord(ev[0], s_)
    e.run_async()
    hip.hipEventRecord(ev[1], s_)
    e.publish_async()
    hip.hipEventRecord(ev[2], s_)
    e.sync()
    ts.append(time.perf_counter() - t1)
    x, y = C.c_float(), C.c_float()
    hip.hipEventElapsedTime(C.byref(x), ev[0], ev[1])
    hip.hipEventElapsedTime(C.byref(y), ev[1], ev[2])
    rms.append(x.value)
    pms.append(y.value)
dg = e.digests()
want = np.array([int(gold[f"{names[k]}/L32"]["digest"], 16) for k in which], np.uint64)
ok = bool((e.status() == 0).all()) and bool((dg == want).all())
ops = int(sum(traces[k].n_patches for k in which))
canon_total = int(e.canon_counts().astype(np.int64).sum())
rk = float(np.mean(rms))
alg = 32 * canon_total + 24 * ops  # docs x (32 B x canonical spans + 24 B x ops)
wl = "config3" if a.share else "config3_noshare"
# CPU leg: the oracle replaying the same mix on every core this process may use
threads, affinity, quota = cpu_share()
mix = np.bincount(which, minlength=3) / a.docs
cpu_ops, cpu_s = 0, 0.0
for k, t in enumerate(traces):
    n, s = sampled(lambda m: cpu_baseline_local(t, m, threads), threads, a.cpu_seconds * mix[k], 4096)
    cpu_ops += n * t.n_patches
    cpu_s += s
t = min(ts)
print(json.dumps({
    "build_id": crdt_amd.build_id(),
    "metric": "CRDT ops remapped+merged/sec (config 3: mixed local corpus)", "value": ops / t, "unit": "ops/s",
    "n_gpus": 1, "steps": a.steps, "ms_per_step": t * 1e3, "higher_is_better": True, "dtype": "u32",
    "data": "synthetic-from-trace: benchmark_data traces, doc d replays trace splitmix64(d) % 3",
    "config": {"workload": f"config3: {a.docs} docs x [AP, RC, SV] local txns, replay+publish", "docs": a.docs,
               "ops": ops, "mix": {n: int((which == k).sum()) for k, n in enumerate(names)},
               "record_streams": "one device copy per trace (read-only input)" if a.share else "one copy per document",
               "waves_per_simd": a.docs / SIMDS, "hbm_bytes_per_doc": mem / a.docs, "hbm_bytes": mem},
    "roofline": {"bound": "hbm", "achieved": alg / (rk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": alg / (rk * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": measured_traffic(a.docs, "k_replay", wl),
                 "traffic_file": f"profiles/traffic_k_replay_{wl}.json", "kernel": "k_replay<32>", "kernel_ms": rk,
                 "alg_bytes_per_launch": alg, "canonical_spans": canon_total,
                 "alg_bytes_formula": "SURVEY 8(d): docs x (32 B x canonical spans + 24 B x ops)"},
    "kernels_ms": {"k_replay": rk, "k_publish": float(np.mean(pms))},
    "cpu_baseline": {"value": cpu_ops / cpu_s, "unit": "ops/s", "threads_used": threads, "host_cores": os.cpu_count(),
                     "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "kind": "port",
                     "sample": f"oracle (reference B-tree restatement, SplitList index) on the same mix, {cpu_s:.1f} s"},
    "parity_ok": ok, "parity": "every document's digest == committed golden digest of its trace", "stage_s": stage_s,
}))
