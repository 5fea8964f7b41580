"""Profiling driver for k_materialize: stage `docs` copies of the AP remote form, replay, publish,
give every document its own copy of the trace's content stream (bench.py's leg), then materialise twice; the last k_materialize dispatch of the
process is the measured one (same launch as bench.py's materialize leg)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import crdt_amd  # noqa: E402
from crdt_amd.traces import content_by_order, load_remote_wire, load_trace  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=8192)
ap.add_argument("--shared", action="store_true", help="one shared content stream (default: a copy per document, as bench.py)")
ap.add_argument("--trace", default="automerge-paper")
a = ap.parse_args()
e = crdt_amd.Engine(a.docs, 32)
e.stage_remote_replicated(load_remote_wire(a.trace), 0, ["u%05d" % i for i in range(a.docs)])
st = e.run()
e.publish_async()
e.sync()
c = content_by_order(load_trace(a.trace))
if a.shared:
    e.set_content(list(range(a.docs)), [0] * a.docs, [c])
else:  # bench.py's materialize leg: every document reads its own HBM copy of the content
    e.set_content_copies(list(range(a.docs)), c)
for _ in range(2):
    e.materialize_async()
    e.sync()
print("status ok:", bool((st == 0).all()), "materialize_ms", e.materialize_ms())
