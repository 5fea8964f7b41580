#!/usr/bin/env python3
"""Benchmark: CRDT ops remapped+merged per second on MI355X (BASELINE.json metric).

Workload (BASELINE config 2): `--docs` (default 4096) independent copies of the
automerge-paper trace per GPU, delivered as remote txns (apply_remote_txn path) with randomised
client ids (agent name = hex(splitmix64(0xC0FFEE ^ doc))).  One step = reset all documents to
ListCRDT::new(), replay every document's 259,778 remote ops (merge: (agent,seq)->order remap +
integrate + deletes), rebuild the flat position index (publish), and answer one pos->loc and one
loc->pos query per op position sample.  Inputs are staged in HBM before timing.

Multi-GPU: one process per GPU (torchrun); documents shard across ranks with no per-op
communication; the single collective is an all-gather of per-document digests (RCCL) after the
timed region.  `value` = total ops of all ranks / max-over-ranks step time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def doc_name(d):
    return "%016x" % splitmix64(0xC0FFEE ^ d)


def wire_ops(w: bytes):
    """number of RemoteOps and records in a wire batch (ops are what the metric counts)."""
    import struct
    off = 8
    nn = struct.unpack_from("<I", w, 4)[0]
    for _ in range(nn):
        bl = struct.unpack_from("<I", w, off)[0]
        off += 4 + ((bl + 3) & ~3)
    nt = struct.unpack_from("<I", w, off)[0]
    off += 4
    arr = np.frombuffer(w, dtype=np.uint32, offset=off)
    ops = 0
    recs = 0
    i = 0
    for _ in range(nt):
        np_, no = int(arr[i + 2]), int(arr[i + 3])
        ops += no
        recs += 1 + no + np_
        i += 4 + 2 * np_ + 6 * no
    return ops, recs, nt


def cpu_baseline(wire: bytes, n_docs: int, threads: int):
    """The oracle (C++ restatement of the reference B-tree path, leaf 32 / node 16) replaying the
    same remote workload on host cores, one document per task (rayon-equivalent work queue)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    from oracle_lib import lib as olib
    L = olib()
    names = (C.c_char_p * n_docs)(*[doc_name(d).encode() for d in range(n_docs)])
    ck = C.c_uint64()
    secs = L.orc_cpu_baseline_remote(n_docs, threads, wire, len(wire), 0xFFFFFFFF, names, C.byref(ck))
    return secs


def cpu_baseline_sampled(wire: bytes, threads: int, target_s: float, max_docs: int = 16384):
    """Bounded sample: one calibration pass (one document per thread), then as many documents as
    fill about `target_s` seconds.  Returns (docs, seconds)."""
    t_cal = cpu_baseline(wire, 4 * threads, threads)
    per_doc = max(t_cal / (4 * threads), 1e-4)
    n = int(min(max_docs, max(threads, target_s / per_doc)))
    return n, cpu_baseline(wire, n, threads)


def shard(rank: int, world: int, docs_per_rank: int):
    """Weak scaling: rank r owns documents [r*n, (r+1)*n) of the global corpus (no
    per-op communication between ranks)."""
    assert 0 <= rank < world
    return rank * docs_per_rank, docs_per_rank


def reduce_over_ranks(elapsed: float, digests: np.ndarray, dist, device):
    """The only collectives: max of the per-rank elapsed time, and one all-gather of the per-
    document u64 digests (RCCL on the GPU path, gloo in the CPU rehearsal test)."""
    import torch
    if dist is None:
        return elapsed, digests
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    g = torch.from_numpy(np.ascontiguousarray(digests).view(np.int64)).to(device)
    outs = [torch.empty_like(g) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, g)
    return float(t.item()), torch.cat(outs).cpu().numpy().view(np.uint64)


def materialize_leg(eng, trace, n, hip, ev, s_, reps=5):
    """Text materialisation, measured outside the timed step: every document
    shares the trace's order-indexed content stream; k_materialize writes each document's text
    from the published index.  Algorithmic bytes per document: canonical spans read (16 B) + vpos
    read (4 B) per span, content read (4 B) + text written (4 B) per visible char.  Parity: every
    document's text digest == the committed golden text digest (== the trace's endContent)."""
    import ctypes as C
    import json
    from crdt_amd.traces import content_by_order, load_trace
    eng.set_content(list(range(n)), [0] * n, [content_by_order(load_trace(trace))])
    eng.materialize_async()
    eng.sync()
    ms = []
    for _ in range(reps):
        hip.hipEventRecord(ev[2], s_)
        eng.materialize_async()
        hip.hipEventRecord(ev[3], s_)
        hip.hipEventSynchronize(ev[3])
        x = C.c_float()
        hip.hipEventElapsedTime(C.byref(x), ev[2], ev[3])
        ms.append(x.value)
    tdg = eng.text_digests()
    e0 = eng.export(0)
    lens = eng.lens()
    canon_n = e0["canon"].shape[0]
    alg = int(n * canon_n * 20 + int(lens.astype(np.int64).sum()) * 8)
    k_ms = float(np.mean(ms))
    gold = None
    try:
        gold = int(json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_golden.json")))[f"{trace}/L32"]["text_digest"], 16)
    except (OSError, KeyError):
        pass
    return {"kernel": "k_materialize<32>", "kernel_ms": k_ms, "chars_per_s": float(lens.sum()) / (k_ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": alg / (k_ms * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                         "frac": alg / (k_ms * 1e-3) / 1e9 / 8000.0, "alg_bytes_per_launch": alg,
                         "traffic": measured_traffic(n, "k_materialize")},
            "parity_ok": bool(gold is not None and (tdg == np.uint64(gold)).all()),
            "parity": "every document's text digest == committed golden text digest (== endContent FNV, tests/golden)"}


def golden_digest(trace: str):
    """Committed fixture (tests/golden/oracle_golden.json): the oracle's digest of the trace's
    remote replay with the release layout.  Every document of the bench must reproduce it."""
    import json
    p = os.path.join(ROOT, "tests", "golden", "oracle_golden.json")
    try:
        return int(json.load(open(p))[f"{trace}/L32"]["remote_digest"], 16)
    except (OSError, KeyError):
        return None


def measured_traffic(n_docs: int, kernel: str = "k_replay"):
    """HBM bytes per launch of `kernel` from the committed PMC pass (profiles/traffic_<kernel>.json:
    FETCH_SIZE x 2 + WRITE_SIZE per the MI355X guide's gfx950 correction), scaled per document."""
    import json
    p = os.path.join(ROOT, "profiles", f"traffic_{kernel}.json")
    try:
        t = json.load(open(p))
        return t["hbm_bytes_per_launch"] / t["docs"] * n_docs
    except (OSError, KeyError, ZeroDivisionError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--docs", type=int, default=4096, help="documents per GPU")
    ap.add_argument("--trace", default="automerge-paper")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target length of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-text", action="store_true", help="skip the text materialisation leg")
    ap.add_argument("--queries", type=int, default=4096, help="pos->loc and loc->pos queries per document per step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    import torch
    import crdt_amd
    from crdt_amd.traces import load_remote_wire

    wire = load_remote_wire(args.trace)
    n_ops_doc, n_recs_doc, n_txn_doc = wire_ops(wire)
    doc0, n = shard(rank, world, args.docs)
    names = [doc_name(doc0 + i) for i in range(n)]
    # the wire's name table: index 0 is "jeremy" (the trace author); replace it per document
    eng = crdt_amd.Engine(n, 32, device=local_rank if world > 1 else 0)
    t0 = time.time()
    eng.stage_remote_replicated(wire, 0, names)
    stage_s = time.time() - t0
    st = eng.run()  # untimed: sizes capacities (growth) for this workload
    assert (st == 0).all(), np.unique(st)
    eng.publish_async()
    eng.sync()
    lens = eng.lens()
    # query batch (device resident): positions spread over every document
    rng = np.random.default_rng(1234 + rank)
    q = args.queries
    qdoc = np.repeat(np.arange(n, dtype=np.uint32), q)
    qpos = (rng.random(n * q) * np.repeat(lens, q)).astype(np.uint32)
    dev = torch.device("cuda", local_rank if world > 1 else 0)
    d_doc = torch.from_numpy(qdoc.view(np.int32)).to(dev)
    d_pos = torch.from_numpy(qpos.view(np.int32)).to(dev)
    d_ag = torch.zeros(n * q, dtype=torch.int16, device=dev)
    d_seq = torch.zeros(n * q, dtype=torch.int32, device=dev)
    d_p2 = torch.zeros(n * q, dtype=torch.int32, device=dev)
    d_del = torch.zeros(n * q, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    L = eng.L

    def step():
        eng.reset_async()
        eng.run_async()
        eng.publish_async()
        if q:
            L.crdt_pos_to_loc_dev_async(eng.h, n * q, d_doc.data_ptr(), d_pos.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr())
            L.crdt_loc_to_pos_dev_async(eng.h, n * q, d_doc.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr(),
                                        d_p2.data_ptr(), d_del.data_ptr())

    for _ in range(args.warmup):
        step()
    eng.sync()
    torch.cuda.synchronize()
    # HIP events on the engine stream around the replay kernel (dominant kernel)
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    ev = [C.c_void_p() for _ in range(4)]
    for e_ in ev:
        hip.hipEventCreate(C.byref(e_))
    s_ = C.c_void_p(eng.stream())
    replay_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.reset_async()
        hip.hipEventRecord(ev[0], s_)
        eng.run_async()
        hip.hipEventRecord(ev[1], s_)
        eng.publish_async()
        if q:
            L.crdt_pos_to_loc_dev_async(eng.h, n * q, d_doc.data_ptr(), d_pos.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr())
            L.crdt_loc_to_pos_dev_async(eng.h, n * q, d_doc.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr(),
                                        d_p2.data_ptr(), d_del.data_ptr())
        hip.hipEventSynchronize(ev[1])
        ms = C.c_float()
        hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1])
        replay_ms.append(ms.value)
    eng.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st = eng.status()
    ok = bool((st == 0).all())
    dg = eng.digests()
    t_max, all_dg = reduce_over_ranks(elapsed, dg, dist, dev)
    gold = golden_digest(args.trace)
    ok = ok and bool((all_dg == all_dg[0]).all()) and (gold is None or int(all_dg[0]) == gold)
    mat = materialize_leg(eng, args.trace, n, hip, ev, s_) if not args.no_text else None
    total_ops = n_ops_doc * n * world * args.steps
    value = total_ops / t_max
    ms_step = t_max / args.steps * 1e3
    rms = float(np.mean(replay_ms)) if replay_ms else None
    # algorithmic bytes of one replay launch: every record read once (16 B) + the final per-doc
    # state written once (entries 16 B, directory 8 B/slot, order->leaf 4 B/order, RLE tables).
    e0 = eng.export(0)
    state_bytes = e0["raw"].shape[0] * 16 + e0["leaf_sizes"].shape[0] * (8 + 4) + e0["next_order"] * 4 + \
        e0["deletes"].shape[0] * 12 + e0["cwo"].shape[0] * 16 + e0["txns"].shape[0] * 32
    alg_bytes = n * (n_recs_doc * 16 + state_bytes)
    achieved = alg_bytes / (rms * 1e-3) / 1e9 if rms else None
    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            cd, secs = cpu_baseline_sampled(wire, threads, args.cpu_seconds)
            cpu = {"value": n_ops_doc * cd / secs, "unit": "ops/s", "cores": threads, "kind": "port",
                   "sample": f"{cd} docs x {args.trace} remote replay ({n_ops_doc} ops each), oracle C++ "
                             f"restatement of the reference B-tree path (leaf 32/node 16), {threads} threads, "
                             f"one doc per task; {secs:.2f} s"}
        out = {
            "metric": "CRDT ops remapped+merged/sec (whole node)",
            "value": value,
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic-from-trace: benchmark_data/automerge-paper remote form, randomised client ids",
            "config": {"workload": f"config2: {n} docs/GPU x {args.trace} remote txns ({n_ops_doc} ops/doc), "
                                   f"replay+publish+{q} pos->loc & loc->pos queries/doc",
                       "docs_per_gpu": n, "ops_per_doc": n_ops_doc, "parallelism": f"doc-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": (achieved / 8000.0) if achieved else None, "traffic": measured_traffic(n),
                         "kernel": "k_replay<32>", "kernel_ms": rms,
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "parity_ok": ok,
            "parity": "every document's digest == committed oracle golden digest (tests/golden)",
            "stage_s": stage_s,
            "materialize": mat,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
