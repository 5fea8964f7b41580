"""Secondary measurement: BASELINE config 4 (random-edit documents; the per-GPU share of a
1M-document corpus: 125,000 documents per MI355X).

Each document replays `--ops` local txns drawn inside the replay wave from one GEN record
(make_random_change semantics, doc.rs:544-569; no input records per op).  One step = reset +
replay + publish.  Parity: the digests of a sampled subset of documents equal the oracle's
replay of the same generated ops (the oracle is the checker here, and the CPU baseline).  Prints
one JSON line (bench.py stays the driver's bench)."""
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
ap.add_argument("--docs", type=int, default=125000)
ap.add_argument("--ops", type=int, default=20000)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--seed", type=int, default=0xC0FFEE)
ap.add_argument("--check-docs", type=int, default=64, help="documents checked against the oracle")
ap.add_argument("--cpu-seconds", type=float, default=15.0)
a = ap.parse_args()

import crdt_amd  # noqa: E402
from bench import splitmix64, cpu_share, measured_traffic, SIMDS, HBM_PEAK_GBS  # noqa: E402

e = crdt_amd.Engine(a.docs, 32)
t0 = time.time()
e.stage_random(list(range(a.docs)), "gen", a.ops, a.seed)
st = e.run()  # untimed: capacity growth, index sizing
assert (st == 0).all(), np.unique(st)
e.publish_async()
e.sync()
dg0 = e.digests().copy()
stage_s = time.time() - t0
mem = e.mem_bytes()
hip = C.CDLL("libamdhip64.so")
ev = [C.c_void_p() for _ in range(3)]
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
ok = bool((e.status() == 0).all()) and bool((e.digests() == dg0).all())
canon_total = int(e.canon_counts().astype(np.int64).sum())
# parity on a sample + the CPU baseline: the oracle on sampled documents, every host core
sys.path.insert(0, os.path.join(ROOT, "tests"))
from concurrent.futures import ThreadPoolExecutor  # noqa: E402
from oracle_lib import OracleDoc  # noqa: E402

rng = np.random.default_rng(7)
check = sorted(set(rng.integers(0, a.docs, a.check_docs).tolist()) | {0, a.docs - 1})


def one(d):
    o = OracleDoc(32, 16, split_index=True)
    assert o.apply_random(o.agent("gen"), a.ops, splitmix64(a.seed ^ d) & 0xFFFFFFFF) == 0
    return o.digest()


threads, affinity, quota = cpu_share()
with ThreadPoolExecutor(threads) as ex:
    cdg = list(ex.map(one, check))
ok = ok and all(int(dg0[d]) == g for d, g in zip(check, cdg))
from bench import sampled  # noqa: E402
from oracle_lib import lib as olib  # noqa: E402


def cpu(n):
    seeds = np.array([splitmix64(a.seed ^ d) & 0xFFFFFFFF for d in range(n)], np.uint32)
    ck = C.c_uint64()
    return olib().orc_cpu_baseline_random(n, threads, a.ops, seeds.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(ck), 1)


cdocs, csec = sampled(cpu, threads, a.cpu_seconds, 1 << 20)
t = min(ts)
rk = float(np.mean(rms))
alg = 32 * canon_total + 24 * a.docs * a.ops  # docs x (32 B x canonical spans + 24 B x ops)
print(json.dumps({
    "metric": "CRDT ops remapped+merged/sec (config 4: on-device random edits)", "value": a.docs * a.ops / t,
    "unit": "ops/s", "n_gpus": 1, "steps": a.steps, "ms_per_step": t * 1e3, "higher_is_better": True,
    "dtype": "u32", "data": "synthetic: make_random_change semantics generated in the replay wave",
    "config": {"workload": f"config4: {a.docs} docs/GPU (1M docs / 8 GPUs) x {a.ops} random ops, replay+publish",
               "docs_per_gpu": a.docs, "ops_per_doc": a.ops, "waves_per_simd": a.docs / SIMDS,
               "hbm_bytes_per_doc": mem / a.docs, "hbm_bytes": mem},
    "roofline": {"bound": "hbm", "achieved": alg / (rk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": alg / (rk * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": measured_traffic(a.docs, "k_replay", "config4"),
                 "kernel": "k_replay<32>",
                 "kernel_ms": rk, "alg_bytes_per_launch": alg, "canonical_spans": canon_total,
                 "alg_bytes_formula": "SURVEY 8(d): docs x (32 B x canonical spans + 24 B x ops)"},
    "kernels_ms": {"k_replay": rk, "k_publish": float(np.mean(pms))},
    "cpu_baseline": {"value": cdocs * a.ops / csec, "unit": "ops/s", "threads_used": threads,
                     "host_cores": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
                     "kind": "port", "sample": f"{cdocs} docs x {a.ops} generated ops on the oracle (reference B-tree "
                                               f"restatement, SplitList index), {threads} threads, {csec:.1f} s"},
    "parity_ok": ok, "parity": f"{len(check)} sampled documents' digests == oracle; every step's digests equal",
    "stage_s": stage_s,
}))
