"""Secondary measurement: agent-name interning for a large corpus: every
document interns `--names` distinct client names (as config 5's 16 agents, for a 1M-document
corpus sharded 8 ways), each named `--reps` times in a batch.  Device path (crdt_agent_intern_dev,
k_intern) vs the host path (crdt_agent_intern) on identical calls; ids must agree."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import crdt_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=125000)
ap.add_argument("--names", type=int, default=16)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--replicated", action="store_true",
                help="time crdt_stage_remote_replicated (bench.py's staging: AP remote, one client name per "
                     "document) with device vs host interning; replay both and compare digests")
a = ap.parse_args()
if a.replicated:
    from crdt_amd.traces import load_remote_wire
    wire = load_remote_wire("automerge-paper")
    names = ["%08x-client" % ((d * 2654435761) % (1 << 32)) for d in range(a.docs)]
    out = {"metric": "crdt_stage_remote_replicated seconds (AP remote, renamed author per document)", "docs": a.docs}
    dg = {}
    for mode in ("device", "host"):
        e = crdt_amd.Engine(a.docs, 32)
        e.device_intern(mode == "device")
        t0 = time.perf_counter()
        e.stage_remote_replicated(wire, 0, names)
        out[mode + "_stage_s"] = time.perf_counter() - t0
        st = e.run()
        assert (st == 0).all()
        dg[mode] = e.digests()
        del e
    out["parity_ok"] = bool(np.array_equal(dg["device"], dg["host"]))
    print(json.dumps(out))
    sys.exit(0)
rng = np.random.default_rng(5)
docs = np.repeat(np.arange(a.docs, dtype=np.uint32), a.names * a.reps)
k = rng.integers(0, a.names, docs.shape[0])
names = ["client-%08x-%02d" % (int(d) * 2654435761 % (1 << 32), int(j)) for d, j in zip(docs, k)]
e, h = crdt_amd.Engine(a.docs, 32), crdt_amd.Engine(a.docs, 32)
t0 = time.perf_counter()
gid, grank = e.agent_intern_dev(docs, names)
t1 = time.perf_counter()
hid = h.agent_intern(docs, names)
t2 = time.perf_counter()
ok = bool(np.array_equal(gid, hid))
print(json.dumps({"metric": "agent names interned/sec (get_or_create_agent_id)", "docs": a.docs,
                  "names_per_doc": a.names, "refs": int(docs.shape[0]),
                  "device_s": t1 - t0, "device_refs_per_s": docs.shape[0] / (t1 - t0),
                  "host_s": t2 - t1, "host_refs_per_s": docs.shape[0] / (t2 - t1),
                  "note": "both include the call's host-side marshalling (Python strings -> C); the device "
                          "time includes upload + kernel + download", "parity_ok": ok}))
