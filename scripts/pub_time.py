"""Diagnostic: k_publish time for config 2 (docs x automerge-paper remote) with the library named by
CRDT_GPU_LIB; also checks the query round trip on a sample."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import numpy as np
import crdt_amd
from crdt_amd.traces import load_remote_wire
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
e = crdt_amd.Engine(n, 32)
e.stage_remote_replicated(load_remote_wire("automerge-paper"), 0, ["u%05d" % i for i in range(n)])
assert (e.run() == 0).all()
e.publish_async(); e.sync(); e.fit()
ms = []
for _ in range(5):
    e.publish_async(); e.sync()
    e.L.crdt_sync(e.h)
    t0 = time.perf_counter(); e.publish_async(); e.sync(); ms.append((time.perf_counter() - t0) * 1e3)
lens = e.lens()
pos = np.arange(0, int(lens[7]), 7, dtype=np.uint32)
a, s = e.pos_to_loc(np.full(pos.shape, 7, np.uint32), pos)
p, d = e.loc_to_pos(np.full(pos.shape, 7, np.uint32), a, s)
print(os.environ.get("CRDT_GPU_LIB", "default"), "publish ms (wall, sync)", ["%.2f" % x for x in ms], "roundtrip_ok", bool((p == pos).all() and (d == 0).all()))
