"""Diagnostic: per-path cycle attribution of k_replay (build with -DCRDT_PROF into
build/libcrdt_gpu_prof.so, run with CRDT_GPU_LIB pointing at it).  Prints, per document averaged,
the s_memtime cycles spent in fast paths vs the general interpreter."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import numpy as np  # noqa: E402
import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
e = crdt_amd.Engine(n, 32)
e.stage_remote_replicated(load_remote_wire("automerge-paper"), 0, ["u%05d" % i for i in range(n)])
e.run()
e.reset_async()
e.run_async()
e.sync()
ms = e.timings()[0]
s = np.array([e.debug_state(d) for d in range(0, n, max(1, n // 64))]).astype(np.float64)
c = {"typing": s[:, 18].mean(), "generic": s[:, 19].mean(), "delete": s[:, 20].mean(), "insert": s[:, 21].mean()}
tot = sum(c.values())
print(f"docs {n} replay_ms {ms:.1f}  per-doc clock ticks: " + "  ".join(f"{k} {v:.4g} ({v / tot:.1%})" for k, v in c.items()))
