"""Secondary measurement: BASELINE config 5 (concurrent, deletion-heavy remote merges).

Per document: agent "base" inserts a 1M-char run (one txn), then 16 agents x 64 rounds x 64
single-op txns against the round-start snapshot (60 % deletes of 1..64 base items -> double
deletes, 40 % 1..8-char inserts at 32 shared hotspots -> integrate's Equal-branch ties), delivered
in a seeded interleaving.  `--distinct` seeded histories are generated on the host and document d
replays history d % distinct.  Default (SURVEY §8(d)'s shape): every document its own history --
its own ops and its own delivery order -- from the C++ generator (tests/gen/config5_gen.cpp,
`--gen c`), each document reading its own device copy of its records (no shared streams, so no
grouping of documents by history in the launch order).  `--gen py --distinct 8 --share` is round
5's line: 8 histories of tests/fuzz_gen.py config5_wire shared by all documents, one device copy
per history.  One step = reset + replay (k_replay) + publish.

Parity: every step's digests equal, and the digest of every document of a sample (all of them
with few histories; `--check-docs` documents, first and last included, with per-document
histories) equals the oracle's replay of its history (the oracle is the checker and the CPU
baseline).  Roofline: SURVEY §8(d) algorithmic bytes = docs x (32 B x
canonical spans + 24 B x ops) over the k_replay HIP-event time.  Prints one JSON line in the bench
schema (bench.py stays the driver's bench)."""
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
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=1024)
ap.add_argument("--distinct", type=int, default=0, help="distinct seeded histories (doc d replays d %% distinct; 0: one per document)")
ap.add_argument("--gen", choices=["c", "py"], default="c", help="history generator: c (tests/gen, default) or py (fuzz_gen.config5_wire)")
ap.add_argument("--share", action="store_true", help="documents of one history read one device copy of its records")
ap.add_argument("--check-docs", type=int, default=64, help="documents checked against the oracle (per-document histories)")
ap.add_argument("--base", type=int, default=1 << 20)
ap.add_argument("--agents", type=int, default=16)
ap.add_argument("--rounds", type=int, default=64)
ap.add_argument("--ops", type=int, default=64, help="txns per agent per round")
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--leaf", type=int, default=32)
ap.add_argument("--cpu-seconds", type=float, default=15.0)
ap.add_argument("--no-cpu", action="store_true")
a = ap.parse_args()

import crdt_amd  # noqa: E402
from bench import cpu_share, sampled, wire_ops, measured_traffic, SIMDS, HBM_PEAK_GBS  # noqa: E402
from fuzz_gen import config5_wire, config5_wires  # noqa: E402
from oracle_lib import OracleDoc, lib as olib  # noqa: E402

a.distinct = a.distinct or a.docs
threads, affinity, quota = cpu_share()
t0 = time.time()
if a.gen == "py":
    wires = [config5_wire(900 + s, base_len=a.base, n_agents=a.agents, rounds=a.rounds, ops=a.ops) for s in range(a.distinct)]
else:
    wires = config5_wires([0xC5000000 + s for s in range(a.distinct)], base_len=a.base, n_agents=a.agents, rounds=a.rounds,
                          ops=a.ops, threads=threads)
gen_s = time.time() - t0
print(f"generated {a.distinct} histories in {gen_s:.1f} s", file=sys.stderr, flush=True)
ops_of = [wire_ops(w)[0] for w in wires]
doc_w = [d % a.distinct for d in range(a.docs)]
total_ops = sum(ops_of[k] for k in doc_w)

e = crdt_amd.Engine(a.docs, a.leaf)
# --share: documents of one history read one device copy of its records (read-only during the replay)
e.share_streams(a.share)
t0 = time.time()
e.apply_remote_wire(list(range(a.docs)), [wires[k] for k in doc_w], stage_only=True)
stage_s = time.time() - t0
print(f"staged {a.docs} documents in {stage_s:.1f} s", file=sys.stderr, flush=True)
st = e.run()  # untimed: capacity growth, index sizing
assert (st == 0).all(), np.unique(st)
e.publish_async()
e.sync()
e.fit()
dg0 = e.digests().copy()
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
canon = e.canon_counts().astype(np.int64)
sizes0 = e.export_sizes(0)

# parity: the oracle's digest of every checked history; every checked document equals its history's
from concurrent.futures import ThreadPoolExecutor  # noqa: E402


def one(k):
    o = OracleDoc(a.leaf, 16 if a.leaf == 32 else 8, split_index=True)
    assert o.apply_remote_wire(wires[k]) == 0
    return o.digest()


if a.distinct <= 64:
    check = list(range(a.docs))
else:
    rng = np.random.default_rng(55)
    check = sorted(set(rng.integers(0, a.docs, a.check_docs).tolist()) | {0, a.docs - 1})
hist = sorted(set(doc_w[d] for d in check))
with ThreadPoolExecutor(max(1, min(threads, len(hist)))) as ex:
    odg = dict(zip(hist, ex.map(one, hist)))
ok = ok and all(int(dg0[d]) == odg[doc_w[d]] for d in check)

cpu = None
if not a.no_cpu:
    def cpu_run(n):  # n documents, history d % distinct, one document per task on `threads` threads
        if a.distinct >= n:  # (one history per document: `threads` workers, one document each at a time)
            def one_doc(d):
                ck = C.c_uint64()
                olib().orc_cpu_baseline_remote(1, 1, wires[d], len(wires[d]), 0xFFFFFFFF, None, C.byref(ck), 1)
            t1 = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(one_doc, range(n)))
            return time.perf_counter() - t1
        per = [n // a.distinct + (1 if k < n % a.distinct else 0) for k in range(a.distinct)]
        tot = 0.0
        ck = C.c_uint64()
        for k, m in enumerate(per):
            if m:
                tot += olib().orc_cpu_baseline_remote(m, threads, wires[k], len(wires[k]), 0xFFFFFFFF, None, C.byref(ck), 1)
        return tot
    cdocs, csec = sampled(cpu_run, threads, a.cpu_seconds, 4096)
    cops = sum(ops_of[d % a.distinct] for d in range(cdocs))
    cpu = {"value": cops / csec, "unit": "ops/s", "cores": threads, "threads_used": threads, "host_cores": os.cpu_count(),
           "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "kind": "port",
           "sample": f"{cdocs} config-5 documents (histories d % {a.distinct}) on the oracle (reference B-tree "
                     f"restatement, leaf {a.leaf}, SplitList index), {threads} threads, one document per task, {csec:.1f} s"}

t = min(ts)
rk = float(np.mean(rms))
# the PMC pass this line's traffic comes from: per-document histories (scripts/gpu_pmc.sh c5d) or
# the shared-history shape (c5)
tw = "config5d" if (a.gen == "c" and a.distinct == a.docs and not a.share) else "config5"
alg = int(32 * int(canon.sum()) + 24 * total_ops)
print(json.dumps({
    "build_id": crdt_amd.build_id(),
    "metric": "CRDT ops remapped+merged/sec (config 5: concurrent deletion-heavy remote merges)",
    "value": total_ops / t, "unit": "ops/s", "n_gpus": 1, "steps": a.steps, "ms_per_step": t * 1e3,
    "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
    "data": ("synthetic: tests/gen/config5_gen.cpp (seeded, one history per seed: 16 agents, hotspot ties, overlapping "
             "deletes, per-history delivery interleaving)" if a.gen == "c" else
             "synthetic: tests/fuzz_gen.py config5_wire (seeded; 16 agents, hotspot ties, overlapping deletes)"),
    "config": {"workload": f"config5: {a.docs} docs/GPU x ({a.base}-char base + {a.agents} agents x {a.rounds} rounds x "
                           f"{a.ops} txns), replay+publish", "docs_per_gpu": a.docs, "distinct_histories": a.distinct,
               "generator": a.gen, "shared_streams": a.share,
               "ops_per_doc": ops_of[0], "leaf_cap": a.leaf, "waves_per_simd": a.docs / SIMDS,
               "hbm_bytes_per_doc": mem / a.docs, "hbm_bytes": mem, "device_peak_bytes": crdt_amd.Engine.device_bytes()[1],
               "doc0": {"raw_entries": sizes0["raw"], "leaves": sizes0["leaves"], "double_deletes": sizes0["dd"],
                        "canonical_spans": sizes0["canon"], "len": sizes0["len"]}},
    "roofline": {"bound": "hbm", "achieved": alg / (rk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": alg / (rk * 1e-3) / 1e9 / HBM_PEAK_GBS,
                 "traffic": measured_traffic(a.docs, "k_replay", tw) if a.leaf == 32 else None,
                 "traffic_file": f"profiles/traffic_k_replay_{tw}.json", "kernel": f"k_replay<{a.leaf}>",
                 "kernel_ms": rk, "alg_bytes_per_launch": alg,
                 "alg_bytes_formula": "SURVEY 8(d): docs x (32 B x canonical spans + 24 B x ops)"},
    "kernels_ms": {"k_replay": rk, "k_publish": float(np.mean(pms))},
    "cpu_baseline": cpu,
    "parity_ok": ok, "parity": f"{len(check)} documents' digests == the oracle's replay of their histories ({len(hist)} "
                               f"histories checked of {a.distinct}); every step's digests equal",
    "gen_s": gen_s, "stage_s": stage_s,
}))
