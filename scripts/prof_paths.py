"""Diagnostic: per-path attribution of k_replay (build with -DCRDT_PROF into
build/libcrdt_gpu_prof.so, run with CRDT_GPU_LIB pointing at it).  Documents d % 4 == 0 record
s_memtime cycles per path, d % 4 == 1 calls per path, d % 4 == 2 txns per path (config 2: every
document replays the same trace, so the three views combine)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import numpy as np  # noqa: E402
import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire, load_trace  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
mode = sys.argv[2] if len(sys.argv) > 2 else "remote"
local = mode == "local"
e = crdt_amd.Engine(n, 32)
if mode == "random":  # config 4: 20,000 generated ops per document (bench_config4.py's shape)
    e.stage_random(list(range(n)), "gen", 20000, 0xC0FFEE)
elif mode == "kevin":  # benches/yjs.rs:51-62 shape: single-char prepends (200,000 per document)
    k = int(os.environ.get("KEVIN_OPS", "200000"))  # (compact local txns: "generic" = the inserts that split the leaf)
    class T:
        counts = np.ones(k, np.uint32)
        patches = np.zeros((k, 3), np.uint32)
    T.patches[:, 2] = 1
    e.share_streams(True)
    ag = e.agent_intern(list(range(n)), ["seph"] * n)
    e.stage_local_shared(list(range(n)), [0] * n, int(ag[0]), [T])
elif mode == "config5":  # one seeded concurrent history (SURVEY 8(d) shape) on every document
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fuzz_gen import config5_wire
    e.stage_remote_replicated(config5_wire(7, base_len=1 << 20, n_agents=16, rounds=64, ops=64), 0xFFFFFFFF, [""] * n)
elif mode.startswith("wire:"):  # a remote wire file (e.g. data/micro/fd200.rtx.gz) on every document
    import gzip
    e.stage_remote_replicated(gzip.open(os.path.join(ROOT, mode[5:]), "rb").read(), 0, ["u%05d" % i for i in range(n)])
elif local:
    t = load_trace("automerge-paper")
    ag = e.agent_intern(list(range(n)), ["jeremy"] * n)
    e.apply_trace(list(range(n)), int(ag[0]), t.counts, t.patches, stage_only=True)
else:
    e.stage_remote_replicated(load_remote_wire("automerge-paper"), 0, ["u%05d" % i for i in range(n)])
e.run()
e.fit()  # (as bench.py / prof_replay.py: capacities = the stream's use, then one clean launch)
e.reset_async()
e.run_async()
e.sync()
ms = e.timings()[0]
P0 = 19  # DocState.prof0
names = ["typing", "generic", "delete", "insert"]
view = {}
for m, lab in enumerate(["cycles", "calls", "txns"]):
    s = np.array([e.debug_state(d) for d in range(m, n, 4 * max(1, n // 256))]).astype(np.float64)
    view[lab] = s[:, P0:P0 + 4].mean(axis=0)
tot = view["cycles"].sum()
print(f"docs {n} {mode} replay_ms {e.timings()[0]:.1f}")
for i, k in enumerate(names):
    c, calls, tx = view["cycles"][i], view["calls"][i], view["txns"][i]
    print(f"  {k:8s} cycles {c:.4g} ({c / tot:.1%})  calls {calls:.0f}  txns {tx:.0f}  cycles/call {c / max(calls, 1):.0f}  cycles/txn {c / max(tx, 1):.0f}")
s = np.array([e.debug_state(d) for d in range(3, n, 4 * max(1, n // 256))]).astype(np.float64)[:, P0:P0 + 4].mean(axis=0)
if mode == "kevin":
    print(f"  compact local loop cycles by part: split_at {s[0]:.4g}, rest of the splitting inserts {s[1]:.4g}, other fast txns {s[2]:.4g}, "
          f"next record {s[3]:.4g}")
elif mode == "random":
    print(f"  generated-op cycles by part: draw + op {s[0]:.4g}, fast path without cursor {s[1]:.4g}, cursor in leaf {s[2]:.4g}, leaf switch (commit + descent + load) {s[3]:.4g}")
elif os.environ.get("PROF_TXN2"):  # a -DCRDT_PROF_TXN2 build: apply_txn's bookkeeping by part
    print(f"  apply_txn cycles by part: prologue (author switch, fits, assign_order_to_client) {s[0]:.4g}, ops {s[1]:.4g}, "
          f"parents {s[2]:.4g}, insert_txn (frontier, shadow, txns) {s[3]:.4g}")
elif os.environ.get("PROF_TXN"):  # a -DCRDT_PROF_TXN build: apply_txn's cycles by part
    print(f"  apply_txn cycles by part: txn bookkeeping (fits, orders, parents, insert_txn) {s[0]:.4g}, integrate scan {s[1]:.4g}, "
          f"deletes (incl. double deletes) {s[2]:.4g}, op fetch + origins + insert_internal {s[3]:.4g}")
elif os.environ.get("PROF_LOOP"):  # a -DCRDT_PROF_LOOP build: detail of the leaf-split loop
    print(f"  leaf-split loop cycles by part: delete_general without split_at {s[0]:.4g}, split_at {s[1]:.4g}, "
          f"find_order + checks {s[2]:.4g}, delete_segment {s[3]:.4g}")
else:
    print(f"  delete-call cycles by part: run detection {s[0]:.4g}, first segment {s[1]:.4g}, leaf-split loop {s[2]:.4g}, tail {s[3]:.4g}")
