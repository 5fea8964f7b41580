"""Profiling driver: stage `docs` copies of a trace's remote form, replay (with capacity growth),
then with --clean reset and replay once more as ONE k_replay launch (what bench.py times), and
publish.  The last k_replay dispatch of the process is the clean one."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire, load_trace  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=64)
ap.add_argument("--trace", default="automerge-paper")
ap.add_argument("--local", action="store_true")
ap.add_argument("--wire", default=None, help="a .rtx.gz remote wire file instead of a trace")
ap.add_argument("--clean", action="store_true", help="reset and replay once more (single launch)")
ap.add_argument("--no-fit", action="store_true", help="keep the growth capacities (as bench_config3.py; an older "
                "library's fit may not fit memory)")
ap.add_argument("--random", type=int, default=0, help="config 4: this many generated ops per document")
ap.add_argument("--config3", action="store_true",
                help="config 3: mixed local corpus, document d replays trace splitmix64(d) %% 3 (shared record streams)")
ap.add_argument("--no-share", action="store_true", help="config 3: one record stream copy per document")
ap.add_argument("--config5", action="store_true",
                help="config 5: bench_config5.py's 8 seeded concurrent histories (1 M-char base, 16 agents x 64 rounds x 64 txns)")
a = ap.parse_args()
e = crdt_amd.Engine(a.docs, 32)
if a.config3:
    import numpy as np
    sys.path.insert(0, ROOT)
    from bench import splitmix64
    names = ["automerge-paper", "rustcode", "sveltecomponent"]
    traces = [load_trace(x) for x in names]
    which = np.array([splitmix64(d) % 3 for d in range(a.docs)], np.uint32)
    if not a.no_share:
        e.share_streams(True)
    ag = e.agent_intern(list(range(a.docs)), ["jeremy"] * a.docs)
    e.stage_local_shared(list(range(a.docs)), which, int(ag[0]), traces)
elif a.config5:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fuzz_gen import config5_wire
    # scripts/bench_config5.py's workload: 8 seeded histories, document d replays history d % 8,
    # the documents of one history reading one device copy of its records
    wires = [config5_wire(900 + s, base_len=1 << 20, n_agents=16, rounds=64, ops=64) for s in range(8)]
    e.share_streams(True)
    e.apply_remote_wire(list(range(a.docs)), [wires[d % 8] for d in range(a.docs)], stage_only=True)
elif a.random:
    e.stage_random(list(range(a.docs)), "gen", a.random, 0xC0FFEE)
elif a.local:
    t = load_trace(a.trace)
    ag = e.agent_intern(list(range(a.docs)), ["jeremy"] * a.docs)
    e.apply_trace(list(range(a.docs)), int(ag[0]), t.counts, t.patches, stage_only=True)
else:
    if a.wire:
        import gzip
        w = gzip.open(a.wire, "rb").read()
    else:
        w = load_remote_wire(a.trace)
    e.stage_remote_replicated(w, 0, ["u%05d" % i for i in range(a.docs)])
t0 = time.time()
st = e.run()
e.publish_async()
e.sync()
if not a.no_fit:
    e.fit()  # as bench.py: capacities = the stream's use
replay_ms = e.timings()[0]  # (the growth loop's last launch: without --clean not a full replay)
if a.clean:
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    ev = [C.c_void_p() for _ in range(2)]
    for x in ev:
        hip.hipEventCreate(C.byref(x))
    s_ = C.c_void_p(e.stream())
    e.reset_async()
    hip.hipEventRecord(ev[0], s_)
    e.run_async()
    hip.hipEventRecord(ev[1], s_)
    e.sync()
    ms = C.c_float()
    hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1])
    replay_ms = ms.value  # the clean launch, HIP events on the engine stream (as bench.py)
    st = e.status()
pub_ms = None
if a.clean:
    hip.hipEventRecord(ev[0], s_)
    e.publish_async()
    hip.hipEventRecord(ev[1], s_)
    e.sync()
    hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1])
    pub_ms = ms.value  # publish (k_publish + k_pub_index) of the clean replay, HIP events
else:
    e.publish_async()
    e.sync()
import hashlib  # noqa: E402
dg = e.digests()
print("status ok:", bool((st == 0).all()), "replay_ms", replay_ms, "pub_ms", pub_ms, "wall", time.time() - t0,
      "digests", hashlib.sha256(dg.tobytes()).hexdigest()[:12])
