"""Query-kernel A/B (north_star's merge-path sorted-batch queries vs the lockstep LDS kernels):
AP remote documents (bench.py's config 2 state), `--queries` pos->loc and loc->pos queries per
document, each batch random (bench.py's shape) and sorted per document (pos ascending; loc->pos
by (agent, seq)).  Every kernel family answers every batch; answers must equal the LDS kernels'
on the same batch and round-trip.  Times: HIP events on the engine stream, median of --reps."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
import crdt_amd  # noqa: E402
from crdt_amd.traces import load_remote_wire  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=8192)
ap.add_argument("--queries", type=int, default=4096)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
import torch  # noqa: E402

n, q = a.docs, a.queries
e = crdt_amd.Engine(n, 32)
e.device_intern(True)
e.stage_remote_replicated(load_remote_wire("automerge-paper"), 0, ["%08x-c" % ((d * 2654435761) % (1 << 32)) for d in range(n)])
assert (e.run() == 0).all()
e.publish_async()
e.sync()
lens = e.lens()
rng = np.random.default_rng(1234)
qdoc = np.repeat(np.arange(n, dtype=np.uint32), q)
qpos = (rng.random(n * q) * np.repeat(lens, q)).astype(np.uint32)
qpos_sorted = np.sort(qpos.reshape(n, q), axis=1).reshape(-1)
dev = torch.device("cuda", 0)
hip = C.CDLL("libamdhip64.so")
ev = [C.c_void_p() for _ in range(2)]
for x in ev:
    hip.hipEventCreate(C.byref(x))
s_ = C.c_void_p(e.stream())
L = e.L


def t32(x):
    return torch.from_numpy(np.ascontiguousarray(x).view(np.int32)).to(dev)


def timed(fn):
    ms = []
    for _ in range(a.reps):
        hip.hipEventRecord(ev[0], s_)
        fn()
        hip.hipEventRecord(ev[1], s_)
        hip.hipEventSynchronize(ev[1])
        x = C.c_float()
        hip.hipEventElapsedTime(C.byref(x), ev[0], ev[1])
        ms.append(x.value)
    return float(np.median(ms))


d_doc = t32(qdoc)
out = {"metric": "pos->loc and loc->pos queries/sec (AP remote documents)", "docs": n, "queries_per_doc": q,
       "total_queries_each_way": n * q, "kernels": {}}
ref = {}
for batch, pos_np in (("random", qpos), ("sorted", qpos_sorted)):
    d_pos = t32(pos_np)
    # loc->pos inputs: the pos->loc answers (LDS kernels), sorted per document by (agent, seq) for the sorted batch
    e.query_kernel("lds")
    d_ag = torch.zeros(n * q, dtype=torch.int16, device=dev)
    d_sq = torch.zeros(n * q, dtype=torch.int32, device=dev)
    L.crdt_pos_to_loc_dev_async(e.h, n * q, d_doc.data_ptr(), d_pos.data_ptr(), d_ag.data_ptr(), d_sq.data_ptr())
    e.sync()
    ag = d_ag.cpu().numpy().view(np.uint16).astype(np.uint64)
    sq = d_sq.cpu().numpy().view(np.uint32).astype(np.uint64)
    want_pos = pos_np.copy()
    if batch == "sorted":
        key = (np.repeat(np.arange(n, dtype=np.uint64), q) << np.uint64(48)) | (ag << np.uint64(32)) | sq
        perm = np.argsort(key, kind="stable")
        ag, sq, want_pos = ag[perm], sq[perm], pos_np[perm]
    l_ag = torch.from_numpy(ag.astype(np.uint16).view(np.int16)).to(dev)
    l_sq = t32(sq.astype(np.uint32))
    for mode in ("lds", "per_thread", "merge"):
        e.query_kernel(mode)
        o_ag = torch.zeros(n * q, dtype=torch.int16, device=dev)
        o_sq = torch.zeros(n * q, dtype=torch.int32, device=dev)
        o_p = torch.zeros(n * q, dtype=torch.int32, device=dev)
        o_d = torch.zeros(n * q, dtype=torch.uint8, device=dev)
        p2l = timed(lambda: L.crdt_pos_to_loc_dev_async(e.h, n * q, d_doc.data_ptr(), d_pos.data_ptr(), o_ag.data_ptr(), o_sq.data_ptr()))
        l2p = timed(lambda: L.crdt_loc_to_pos_dev_async(e.h, n * q, d_doc.data_ptr(), l_ag.data_ptr(), l_sq.data_ptr(), o_p.data_ptr(), o_d.data_ptr()))
        e.sync()
        got = (o_ag.cpu().numpy().view(np.uint16), o_sq.cpu().numpy().view(np.uint32))
        r = ref.setdefault(batch, got)
        ok = bool(np.array_equal(got[0], r[0]) and np.array_equal(got[1], r[1]))
        ok = ok and bool(np.array_equal(o_p.cpu().numpy().view(np.uint32), want_pos)) and bool((o_d.cpu().numpy() == 0).all())
        out["kernels"][f"{mode}/{batch}"] = {"pos_to_loc_ms": p2l, "loc_to_pos_ms": l2p,
                                             "pos_to_loc_q_per_s": n * q / (p2l * 1e-3), "loc_to_pos_q_per_s": n * q / (l2p * 1e-3),
                                             "answers_ok": ok}
        print(mode, batch, round(p2l, 3), round(l2p, 3), ok, file=sys.stderr)
out["parity_ok"] = all(v["answers_ok"] for v in out["kernels"].values())
print(json.dumps(out))
