#!/usr/bin/env python3
"""Benchmark: CRDT ops remapped+merged per second on MI355X (BASELINE.json metric).

Workload (BASELINE config 2): `--docs` (default 8192) independent copies of the
automerge-paper trace per GPU, delivered as remote txns (apply_remote_txn path) with randomised
client ids (agent name = hex(splitmix64(0xC0FFEE ^ doc))).  One step = reset all documents to
ListCRDT::new(), replay every document's 259,778 remote ops (merge: (agent,seq)->order remap +
integrate + deletes), rebuild the flat position index (publish), and answer `--queries` pos->loc
and loc->pos queries per document.  Inputs are staged in HBM before timing.

`--workload config4` (BASELINE config 4, the north star's >= 1 M-document corpus): `--corpus-docs`
(default 1,000,000) random-edit documents of `--gen-ops` ops each, generated inside the replay wave
(make_random_change semantics, /root/reference/src/list/doc.rs:544-569).  The corpus is document-
sharded over the ranks (125,000 documents per rank at N = 8); a rank replays its share in resident
batches of up to `--batch-docs` documents on one engine (8 batches at N = 1).  One step = the whole
corpus: per batch, the generator seeds of its documents are set on the device, then reset +
replay + publish, and the digests are copied out on the device.  `value` = corpus ops / step time.

The default line carries that corpus too: after the config-2 leg (and its engine is freed) the
same config-4 leg runs (`--corpus-steps` timed passes after `--corpus-warmup` untimed ones) and is
reported as the line's `corpus` object, with its own roofline, CPU baseline, parity and collective
check, so `bench.py --gpus N` measures the north star's 1 M-document corpus (strong scaling over N)
without a flag.  `--dist` initialises the RCCL process group even at world size 1.

Multi-GPU: one process per GPU.  `--gpus N` with N > 1 started by hand spawns the N
ranks through torch.distributed.run (the parent never touches a GPU); under torchrun the ranks
read RANK / LOCAL_RANK / WORLD_SIZE.  The global corpus is N x `--docs` documents, sharded into
contiguous ranges balanced by op count; no per-op communication.  The collectives are the max
over ranks of the elapsed time, an all-gather of per-rank times and one all-gather of the per-
document u64 digests (RCCL), all after the timed region.  `value` = total ops of all ranks /
max-over-ranks time.  `--rehearse-cpu` runs the same launch / shard / collective plumbing on CPU
ranks over gloo with no GPU (the per-document results are the committed golden digests).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))

HBM_PEAK_GBS = 8000.0           # MI355X HBM3E (MI355X_MICROARCH.md)
SIMDS = 256 * 4                 # 256 CUs x 4 SIMDs


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def doc_name(d):
    return "%016x" % splitmix64(0xC0FFEE ^ d)


def wire_ops(w: bytes):
    """number of RemoteOps, wire records and txns in a wire batch (ops are what the metric counts)."""
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


# ------------------------------------------------------------------------------------------------
# multi-GPU plumbing
# ------------------------------------------------------------------------------------------------
def shard_balanced(weights, world: int, rank: int):
    """Contiguous document range [lo, lo+n) of `rank`, balanced by the documents' weights (op
    counts): rank r starts at the first document whose weight prefix reaches
    r/world of the total."""
    assert 0 <= rank < world
    w = np.asarray(weights, dtype=np.float64)
    pre = np.concatenate([[0.0], np.cumsum(w)])
    cut = [int(np.searchsorted(pre[1:], pre[-1] * r / world, side="right")) if r else 0 for r in range(world + 1)]
    cut[world] = len(w)
    for r in range(1, world + 1):
        cut[r] = max(cut[r], cut[r - 1])
    return cut[rank], cut[rank + 1] - cut[rank]


def shard(rank: int, world: int, docs_per_rank: int):
    """Weak scaling: the global corpus is world x docs_per_rank documents of equal work (config 2),
    so the balanced ranges are [r*n, (r+1)*n)."""
    return shard_balanced(np.ones(world * docs_per_rank), world, rank)


def reduce_over_ranks(elapsed: float, digests: np.ndarray, dist, device):
    """The only collectives: max of the per-rank elapsed time, all-gather of the per-rank times,
    and one all-gather of the per-document u64 digests (RCCL on the GPU path, gloo in the CPU
    rehearsal).  Returns (max time, per-rank times, all digests in rank order)."""
    import torch
    if dist is None:
        return elapsed, [elapsed], digests
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    ts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(ts, t)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # all_gather needs equal sizes: pad each rank's digests to the largest shard
    n = torch.tensor([len(digests)], device=device, dtype=torch.int64)
    ns = [torch.empty_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(ns, n)
    m = int(max(int(x.item()) for x in ns))
    pad = np.zeros(m, np.uint64)
    pad[:len(digests)] = digests
    g = torch.from_numpy(pad.view(np.int64)).to(device)
    outs = [torch.empty_like(g) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, g)
    alld = np.concatenate([o.cpu().numpy().view(np.uint64)[:int(k.item())] for o, k in zip(outs, ns)])
    return float(t.item()), [float(x.item()) for x in ts], alld


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started by hand: run N ranks under torch.distributed.run, one process per
    GPU, and exit with its status.  The parent process never initialises a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------------------------
# CPU baseline (the oracle's restatement of the reference's B-tree path; cpu_baseline leg only)
# ------------------------------------------------------------------------------------------------
def cpu_share():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota if one is set
    (a GPU box's share can be far below os.cpu_count())."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_baseline_remote(wire: bytes, n_docs: int, threads: int):
    """Config 2 on host cores: the oracle (C++ restatement of the reference B-tree path: leaf 32,
    node 16, SplitList order index with bucket 100) replays the same remote workload, one document
    per task from an atomic work queue (rayon-equivalent)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    from oracle_lib import lib as olib
    L = olib()
    names = (C.c_char_p * n_docs)(*[doc_name(d).encode() for d in range(n_docs)])
    ck = C.c_uint64()
    return L.orc_cpu_baseline_remote(n_docs, threads, wire, len(wire), 0xFFFFFFFF, names, C.byref(ck), 1)


def cpu_baseline_local(trace, n_docs: int, threads: int):
    """Config 1's CPU reference path (benches/yjs.rs:41-48: ListCRDT::new + apply_local_txn per
    txn) on the restatement, `threads` threads, one document per task."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    from oracle_lib import lib as olib
    L = olib()
    c = np.ascontiguousarray(trace.counts, np.uint32)
    p = np.ascontiguousarray(trace.patches, np.uint32)
    ck = C.c_uint64()
    return L.orc_cpu_baseline_local(n_docs, threads, c.shape[0], c.ctypes.data_as(C.POINTER(C.c_uint32)),
                                    p.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(ck), 1)


def sampled(fn, threads: int, target_s: float, max_docs: int = 16384):
    """Bounded sample: one calibration pass (four documents per thread), then as many documents as
    fill about `target_s` seconds.  Returns (docs, seconds)."""
    t_cal = fn(4 * threads)
    per_doc = max(t_cal / (4 * threads), 1e-4)
    n = int(min(max_docs, max(threads, target_s / per_doc)))
    return n, fn(n)


def cpu_baseline(wire, n_ops_doc, target_s):
    from crdt_amd.traces import load_trace
    threads, affinity, quota = cpu_share()
    cd, secs = sampled(lambda k: cpu_baseline_remote(wire, k, threads), threads, target_s)
    ap = load_trace("automerge-paper")
    n1, s1 = sampled(lambda k: cpu_baseline_local(ap, k, 1), 1, max(2.0, target_s / 8), 64)
    return {"value": n_ops_doc * cd / secs, "unit": "ops/s", "cores": threads, "threads_used": threads,
            "host_cores": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "kind": "port",
            "sample": f"{cd} docs x automerge-paper remote replay ({n_ops_doc} ops each) on {threads} threads, "
                      f"one doc per task; {secs:.2f} s.  Oracle C++ restatement of the reference B-tree path "
                      f"(leaf 32 / node 16, SplitList order index, bucket 100), -O3",
            "single_thread": {"config": "config1: automerge-paper as local txns (benches/yjs.rs:41-48), 1 thread",
                              "value": ap.n_patches * n1 / s1, "unit": "ops/s", "docs": n1, "seconds": s1}}


# ------------------------------------------------------------------------------------------------
# measurement helpers
# ------------------------------------------------------------------------------------------------
def golden(trace: str, key: str):
    """Committed fixture (tests/golden/oracle_golden.json) of the oracle's replay of the trace."""
    p = os.path.join(ROOT, "tests", "golden", "oracle_golden.json")
    try:
        return json.load(open(p))[f"{trace}/L32"][key]
    except (OSError, KeyError):
        return None


def golden_pos_seq(trace: str):
    """Committed fixture (tests/golden/ap_remote_pos_seq.delta.gz, made by make_queries.py from the
    oracle): seq of the item at every visible position of the trace's remote replay (one author,
    agent 0), or None."""
    import gzip
    if trace != "automerge-paper":
        return None
    try:
        d = np.frombuffer(gzip.open(os.path.join(ROOT, "tests", "golden", "ap_remote_pos_seq.delta.gz")).read(), np.int32)
    except OSError:
        return None
    return np.cumsum(d.astype(np.int64)).astype(np.uint32)


def golden_seq_pos(trace: str):
    """Committed fixture (tests/golden/ap_remote_seq_pos.delta.gz, made by make_queries.py from the
    oracle): (position, deleted) of every seq of the trace's remote replay (one author, agent 0;
    Cursor::count_pos, cursor.rs:147-190), or None."""
    import gzip
    if trace != "automerge-paper":
        return None
    try:
        b = gzip.open(os.path.join(ROOT, "tests", "golden", "ap_remote_seq_pos.delta.gz")).read()
    except OSError:
        return None
    n = len(b) // 5
    d = np.frombuffer(b[:4 * n], np.int32)
    return np.cumsum(d.astype(np.int64)).astype(np.uint32), np.frombuffer(b[4 * n:], np.uint8).copy()


TRAFFIC_WORKLOAD = {"k_replay": "automerge-paper remote, one clean launch",
                    "k_materialize": "automerge-paper remote, per-document content copies, one launch",
                    "k_replay:config4": "config 4: generated random edits (20,000 ops/doc), one clean launch",
                    "k_replay:config3": "config 3: mixed local corpus, shared record streams, one clean launch",
                    "k_replay:config3_noshare": "config 3: mixed local corpus, per-document record streams, one clean launch",
                    "k_replay:config5": "config 5: concurrent histories (1 M-char base, 16 agents), one clean launch",
                    "k_replay:config5d": "config 5: per-document concurrent histories (1 M-char base, 16 agents), one clean launch"}


def measured_traffic(n_docs: int, kernel: str = "k_replay", workload: str = None):
    """HBM bytes per launch of `kernel` from the committed PMC pass (profiles/traffic_<kernel>.json:
    FETCH_SIZE x 2 + WRITE_SIZE per the MI355X guide's gfx950 correction).  Only a pass of this
    exact workload (TRAFFIC_WORKLOAD) at this document count is reported; anything else is None
    (a pass over another workload says nothing about this launch)."""
    p = os.path.join(ROOT, "profiles", f"traffic_{kernel}{'_' + workload if workload else ''}.json")
    try:
        t = json.load(open(p))
        if t.get("workload") != TRAFFIC_WORKLOAD.get(kernel + (":" + workload if workload else "")) or int(t["docs"]) != n_docs:
            return None
        return t["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def materialize_leg(eng, trace, n, hip, ev, s_, reps=5):
    """Text materialisation, measured outside the timed step.  Every document
    reads its own copy of the trace's order-indexed content (a per-document stream, so the
    content reads come from HBM, not from a shared cache-resident stream); k_materialize writes
    each document's text from the published index.  Algorithmic bytes per document: canonical
    spans read (16 B) + vpos read (4 B) per span, content read (4 B) + text written (4 B) per
    visible char.  Parity: every document's text digest == the committed golden text digest
    (== the trace's endContent)."""
    import ctypes as C
    from crdt_amd.traces import content_by_order, load_trace
    c = content_by_order(load_trace(trace))
    eng.set_content_copies(list(range(n)), c)
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
    canon_n = eng.export_sizes(0)["canon"]
    lens = eng.lens()
    alg = int(n * canon_n * 20 + int(lens.astype(np.int64).sum()) * 8)
    k_ms = float(np.mean(ms))
    gold = golden(trace, "text_digest")
    eng.set_content_copies([], c[:0])  # release the per-document content copies
    return {"kernel": "k_materialize<32>", "kernel_ms": k_ms, "chars_per_s": float(lens.sum()) / (k_ms * 1e-3),
            "content": "one order-indexed content copy per document",
            "roofline": {"bound": "hbm", "achieved": alg / (k_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                         "traffic": measured_traffic(n, "k_materialize")},
            "parity_ok": bool(gold is not None and (tdg == np.uint64(int(gold, 16))).all()),
            "parity": "every document's text digest == committed golden text digest (== endContent FNV, tests/golden)"}


def stated_size_leg(args, wire, n_ops_doc, hip, docs=4096, steps=3):
    """BASELINE config 2 at its stated size (4,096 documents per GPU; the bench line runs 8,192 = 8
    waves per SIMD): the same step (reset + replay + publish + the same per-document queries) on a
    second engine, timed the same way.  Reported beside the line, not as its value."""
    import ctypes as C
    import crdt_amd
    import torch
    e = crdt_amd.Engine(docs, 32)
    e.device_intern(not args.host_intern)
    e.stage_remote_replicated(wire, 0, [doc_name(i) for i in range(docs)])
    assert (e.run() == 0).all()
    e.publish_async()
    e.sync()
    e.fit()
    q = args.queries
    lens = e.lens()
    rng = np.random.default_rng(4321)
    dev = torch.device("cuda", 0)
    d_doc = torch.from_numpy(np.repeat(np.arange(docs, dtype=np.uint32), q).view(np.int32)).to(dev)
    d_pos = torch.from_numpy((rng.random(docs * q) * np.repeat(lens, q)).astype(np.uint32).view(np.int32)).to(dev)
    d_ag = torch.zeros(docs * q, dtype=torch.int16, device=dev)
    d_seq = torch.zeros(docs * q, dtype=torch.int32, device=dev)
    d_p2 = torch.zeros(docs * q, dtype=torch.int32, device=dev)
    d_del = torch.zeros(docs * q, dtype=torch.uint8, device=dev)
    ev = [C.c_void_p() for _ in range(2)]
    for x in ev:
        hip.hipEventCreate(C.byref(x))
    s_ = C.c_void_p(e.stream())
    L = e.L

    def step(ms):
        e.reset_async()
        hip.hipEventRecord(ev[0], s_)
        e.run_async()
        hip.hipEventRecord(ev[1], s_)
        e.publish_async()
        if q:
            L.crdt_pos_to_loc_dev_async(e.h, docs * q, d_doc.data_ptr(), d_pos.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr())
            L.crdt_loc_to_pos_dev_async(e.h, docs * q, d_doc.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr(),
                                        d_p2.data_ptr(), d_del.data_ptr())
        if ms is not None:
            hip.hipEventSynchronize(ev[1])
            x = C.c_float()
            hip.hipEventElapsedTime(C.byref(x), ev[0], ev[1])
            ms.append(x.value)

    step(None)
    e.sync()
    torch.cuda.synchronize()
    ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        step(ms)
    e.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gold = golden(args.trace, "remote_digest")
    ok = bool((e.status() == 0).all()) and (gold is None or bool((e.digests() == np.uint64(int(gold, 16))).all()))
    ok = ok and (not q or bool(((d_p2 == d_pos) & (d_del == 0)).all().item()))
    gseq = golden_pos_seq(args.trace)
    if q and gseq is not None and int(lens.min()) == gseq.shape[0] == int(lens.max()):
        ok = ok and bool((d_seq == torch.from_numpy(gseq.view(np.int32)).to(dev)[d_pos.long()]).all().item())
    e.close()
    return {"docs_per_gpu": docs, "waves_per_simd": docs / SIMDS, "steps": steps, "ms_per_step": el / steps * 1e3,
            "value": docs * n_ops_doc * steps / el, "k_replay_ms": float(np.mean(ms)), "parity_ok": ok,
            "note": "BASELINE config 2's stated size; same step and timing as the line"}


def rehearse_cpu(args, world, rank, dist):
    """--rehearse-cpu: launch, shard and collectives exactly as on the GPU path, on CPU ranks over
    gloo; each document's 'result' is the committed golden digest (no engine, no GPU)."""
    import torch
    doc0, n = shard(rank, world, args.docs)
    gold = int(golden(args.trace, "remote_digest"), 16)
    dg = np.full(n, gold, np.uint64)
    t0 = time.perf_counter()
    elapsed = time.perf_counter() - t0
    t_max, per_rank, all_dg = reduce_over_ranks(elapsed, dg, dist, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"rehearsal": "cpu-gloo", "n_gpus": world, "world_size": dist.get_world_size() if dist else 1,
                          "docs_total": int(all_dg.shape[0]), "shards": [list(shard(r, world, args.docs)) for r in range(world)],
                          "per_rank_s": per_rank, "parity_ok": bool((all_dg == np.uint64(gold)).all()),
                          "value": None}))


# ------------------------------------------------------------------------------------------------
# config 4: the 1 M-document random-edit corpus
# ------------------------------------------------------------------------------------------------
def config4_batches(lo: int, n: int, batch_docs: int):
    """A rank's documents [lo, lo+n) as resident batches of equal size B (the engine's document
    count): [(first global id, documents of the corpus in it)]; the last batch may hold fewer."""
    nb = max(1, -(-n // batch_docs))
    B = -(-n // nb)
    return B, [(lo + k * B, min(B, n - k * B)) for k in range(nb)]


def config4_rehearsal_digest(ids: np.ndarray) -> np.ndarray:
    """--rehearse-cpu stand-in for a document's digest: a hash of its global id (the rehearsal checks
    that the shards and the gather cover every corpus document exactly once, in order)."""
    x = ids.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def cpu_baseline_random(args, threads: int, target_s: float):
    """Config 4 on host cores: the oracle (reference B-tree restatement, SplitList order index)
    replays generated documents 0.. of the corpus, one document per task."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    from oracle_lib import lib as olib

    def run(k):
        seeds = np.array([splitmix64(args.seed ^ d) & 0xFFFFFFFF for d in range(k)], np.uint32)
        ck = C.c_uint64()
        return olib().orc_cpu_baseline_random(k, threads, args.gen_ops, seeds.ctypes.data_as(C.POINTER(C.c_uint32)),
                                              C.byref(ck), 1)
    return sampled(run, threads, target_s, 1 << 20)


def oracle_digests_random(args, ids, threads: int):
    """The oracle's digests of corpus documents `ids` (the checker; test infrastructure)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from concurrent.futures import ThreadPoolExecutor
    from oracle_lib import OracleDoc

    def one(d):
        o = OracleDoc(32, 16, split_index=True)
        assert o.apply_random(o.agent("gen"), args.gen_ops, splitmix64(args.seed ^ int(d)) & 0xFFFFFFFF) == 0
        return o.digest()
    with ThreadPoolExecutor(threads) as ex:
        return np.array(list(ex.map(one, ids)), np.uint64)


def run_config4(args, world: int, rank: int, gpu: int, dist, steps: int = None, warmup: int = None, cpu_s: float = None):
    """BASELINE config 4: the corpus sharded over ranks, each rank's share replayed
    in resident batches on one engine.  Returns the line (rank 0; None elsewhere): the bench line of
    `--workload config4`, and the `corpus` object of the default line (steps / warmup / CPU sample
    given by the caller)."""
    import ctypes as C
    import torch
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    cpu_s = args.cpu_seconds if cpu_s is None else cpu_s
    D = args.corpus_docs
    lo, n = shard_balanced(np.ones(D), world, rank)
    B, batches = config4_batches(lo, n, args.batch_docs)
    if args.rehearse_cpu:
        t0 = time.perf_counter()
        dg = np.concatenate([config4_rehearsal_digest(np.arange(b0, b0 + m, dtype=np.uint64)) for b0, m in batches])
        t_max, per_rank, all_dg = reduce_over_ranks(time.perf_counter() - t0, dg, dist, torch.device("cpu"))
        if rank == 0:
            want = config4_rehearsal_digest(np.arange(D, dtype=np.uint64))
            print(json.dumps({"rehearsal": "cpu-gloo", "workload": "config4", "n_gpus": world,
                              "world_size": dist.get_world_size() if dist else 1, "corpus_docs": D,
                              "docs_total": int(all_dg.shape[0]), "batch_docs": B,
                              "shards": [list(shard_balanced(np.ones(D), world, r)) for r in range(world)],
                              "batches_per_rank": len(batches),
                              "parity_ok": bool(all_dg.shape[0] == D and (all_dg == want).all()), "value": None}))
        return None
    import crdt_amd
    eng = crdt_amd.Engine(B, 32, device=gpu)
    t0 = time.time()
    eng.stage_random(list(range(B)), "gen", args.gen_ops, args.seed)
    dev = torch.device("cuda", gpu)
    d_dg = torch.zeros(len(batches) * B, dtype=torch.int64, device=dev)
    canon = np.zeros(len(batches), np.int64)
    # untimed pass over every batch: capacity growth, then each batch's fitted capacities noted;
    # the engine is then laid out for the maximum over the batches (crdt_fit_note)
    for k, (b0, m) in enumerate(batches):
        eng.reseed_random_async(args.seed, b0)
        eng.reset_async()
        st = eng.run()
        assert (st == 0).all(), np.unique(st)
        eng.publish_async()
        eng.sync()
        canon[k] = int(eng.canon_counts()[:m].astype(np.int64).sum())
        eng.fit_note(False)
    eng.fit_note(True)
    stage_s = time.time() - t0
    mem = eng.mem_bytes()
    hip = C.CDLL("libamdhip64.so")
    ev = [C.c_void_p() for _ in range(2)]
    for e_ in ev:
        hip.hipEventCreate(C.byref(e_))
    s_ = C.c_void_p(eng.stream())

    def step(ms, check=False):
        """one pass over the rank's batches; check (untimed warm-up only): every batch's statuses
        are read back and must all be OK (a batch stopped on capacity still publishes a
        digest, of a partial state)"""
        good = True
        for k, (b0, m) in enumerate(batches):
            eng.reseed_random_async(args.seed, b0)
            eng.reset_async()
            hip.hipEventRecord(ev[0], s_)
            eng.run_async()
            hip.hipEventRecord(ev[1], s_)
            eng.publish_async()
            eng.digests_dev_async(d_dg.data_ptr() + 8 * k * B)
            if check:
                good = good and bool((eng.status() == 0).all())
            if ms is not None:
                hip.hipEventSynchronize(ev[1])
                x = C.c_float()
                hip.hipEventElapsedTime(C.byref(x), ev[0], ev[1])
                ms.append(x.value)
        return good

    warm_ok = True
    for _ in range(warmup):
        warm_ok = step(None, check=True) and warm_ok
    eng.sync()
    torch.cuda.synchronize()
    ref = d_dg.cpu().numpy().view(np.uint64).copy()  # (the warm-up pass's digests)
    d_dg.zero_()
    replay_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(steps):
        step(replay_ms)
    eng.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    got = d_dg.cpu().numpy().view(np.uint64)
    dg = np.concatenate([got[k * B:k * B + m] for k, (b0, m) in enumerate(batches)])
    same = bool(warmup == 0 or np.array_equal(got, ref))
    ok = bool((eng.status() == 0).all()) and same and warm_ok
    # sampled documents of this rank against the oracle (global ids)
    threads, affinity, quota = cpu_share()
    rng = np.random.default_rng(77 + rank)
    pick = sorted(set(rng.integers(0, n, args.check_docs).tolist()) | {0, n - 1})
    odg = oracle_digests_random(args, [lo + i for i in pick], threads)
    ok = ok and bool(np.array_equal(dg[pick], odg))
    cdev = torch.device("cpu") if args.share_gpu else dev  # (gloo rehearsal on one GPU: CPU tensors)
    t_max, per_rank, all_dg = reduce_over_ranks(elapsed, dg, dist, cdev)
    # the gather's own check: this rank's slice of the gathered digests is what it computed
    lo_all = [shard_balanced(np.ones(D), world, r)[0] for r in range(world)]
    gathered_local = bool(np.array_equal(all_dg[lo_all[rank]:lo_all[rank] + n], dg))
    oks = torch.tensor([1.0 if ok else 0.0, 1.0 if gathered_local else 0.0], device=cdev, dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(oks, op=dist.ReduceOp.MIN)
    gathered_local = bool(oks[1].item() == 1.0)
    ok = bool(oks[0].item() == 1.0) and gathered_local and int(all_dg.shape[0]) == D
    nb = len(batches)
    rms = float(np.mean(replay_ms)) if replay_ms else None  # per k_replay launch (one batch)
    docs_done = D * steps
    value = docs_done * args.gen_ops / t_max
    alg_launch = (32 * int(canon.sum()) + 24 * n * args.gen_ops) / nb  # SURVEY 8(d), per launch (batch)
    # compulsory bytes only: the 16 B of op input per op are never read (the ops are generated in
    # the wave), so the state written (32 B per canonical span) + 8 B of result per op remain
    comp_launch = (32 * int(canon.sum()) + 8 * n * args.gen_ops) / nb
    achieved = alg_launch / (rms * 1e-3) / 1e9 if rms else None
    eng.close()
    del d_dg
    torch.cuda.empty_cache()
    line = None
    if rank == 0:
        cpu = None
        if not args.no_cpu:
            cd, csec = cpu_baseline_random(args, threads, cpu_s)
            cpu = {"value": cd * args.gen_ops / csec, "unit": "ops/s", "cores": threads, "threads_used": threads,
                   "host_cores": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "kind": "port",
                   "sample": f"{cd} corpus documents x {args.gen_ops} generated ops on the oracle (reference B-tree "
                             f"restatement, SplitList order index), {threads} threads, one document per task, {csec:.1f} s"}
        line = {
            "metric": "CRDT ops remapped+merged/sec (whole node)", "value": value, "unit": "ops/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": t_max / steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: make_random_change semantics (doc.rs:544-569) generated in the replay wave",
            "config": {"workload": f"config4: {D} docs x {args.gen_ops} random-edit ops, document-sharded over "
                                   f"{world} GPU(s), {nb} resident batch(es) of {B} docs per GPU, replay+publish",
                       "corpus_docs": D, "ops_per_doc": args.gen_ops, "docs_per_gpu": n, "batch_docs": B,
                       "batches_per_gpu": nb, "parallelism": f"doc-sharded x{world}",
                       "waves_per_simd": B / SIMDS, "hbm_bytes_per_batch_doc": mem / B, "hbm_bytes": mem},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None,
                         "frac_compulsory": comp_launch / (rms * 1e-3) / 1e9 / HBM_PEAK_GBS if rms else None,
                         "compulsory_bytes_per_launch": comp_launch,
                         "compulsory_note": "SURVEY 8(d) without the 16 B/op input term: the ops are generated in the "
                                            "wave and never read from HBM",
                         "traffic": measured_traffic(B, "k_replay", "config4"), "kernel": "k_replay<32>",
                         "kernel_ms": rms, "alg_bytes_per_launch": alg_launch,
                         "alg_bytes_formula": "SURVEY 8(d): docs x (32 B x canonical spans + 24 B x ops), per batch launch",
                         "canonical_spans_per_doc": float(canon.sum()) / n},
            "cpu_baseline": cpu,
            "parity_ok": ok,
            "parity": f"all {D} documents' digests equal across the warm-up and timed passes; "
                      f"{len(pick)} sampled documents per rank == the oracle's replay (global document ids)",
            "world_size": dist.get_world_size() if dist is not None else 1,
            "collective": {"backend": dist.get_backend() if dist is not None else None,
                           "gathered_docs": int(all_dg.shape[0]), "gathered_equal_local": gathered_local},
            "per_rank_ops_s": [n * args.gen_ops * steps / t for t in per_rank],
            "build_id": crdt_amd.build_id(), "stage_s": stage_s,
        }
    return line


# ------------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--docs", type=int, default=8192, help="documents per GPU (8 waves per SIMD)")
    ap.add_argument("--trace", default="automerge-paper")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target length of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-text", action="store_true", help="skip the text materialisation leg")
    ap.add_argument("--host-intern", action="store_true",
                    help="intern the per-document client names on the host (default: k_intern on the GPU)")
    ap.add_argument("--queries", type=int, default=4096, help="pos->loc and loc->pos queries per document per step")
    ap.add_argument("--rehearse-cpu", action="store_true", help="CPU/gloo rehearsal of the multi-rank plumbing")
    ap.add_argument("--no-stated-size", action="store_true", help="skip the 4,096-document (BASELINE size) leg")
    ap.add_argument("--workload", choices=["config2", "config4"], default="config2",
                    help="config2 (default, the driver's line): automerge-paper remote copies; config4: the 1 M-document "
                         "random-edit corpus")
    ap.add_argument("--corpus-docs", type=int, default=1_000_000, help="config4: documents in the corpus (all ranks)")
    ap.add_argument("--batch-docs", type=int, default=125_000, help="config4: documents per resident batch")
    ap.add_argument("--gen-ops", type=int, default=20_000, help="config4: generated ops per document")
    ap.add_argument("--seed", type=int, default=0xC0FFEE, help="config4: corpus seed")
    ap.add_argument("--check-docs", type=int, default=64, help="config4: sampled documents per rank checked against the oracle")
    ap.add_argument("--no-corpus", action="store_true",
                    help="config2: skip the corpus leg (the 1 M-document config-4 corpus, the line's `corpus` object)")
    ap.add_argument("--corpus-steps", type=int, default=2, help="config2: timed passes over the corpus in its leg")
    ap.add_argument("--corpus-warmup", type=int, default=1, help="config2: untimed passes over the corpus in its leg")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL (nccl) process group even at world size 1 (under torchrun "
                         "--nproc-per-node=1, or standalone on 127.0.0.1): the digest gather runs over RCCL")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the multi-rank path on one GPU: every rank runs its engine on cuda:0 and "
                         "the collectives go over gloo (CPU tensors); not a scaling measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    import torch
    dist = None
    if args.rehearse_cpu:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        if args.workload == "config4":
            run_config4(args, world, rank, 0, dist)
        else:
            rehearse_cpu(args, world, rank, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    need = world if world > 1 and not args.share_gpu else 1
    if torch.cuda.device_count() < need:  # (counting devices does not initialise them)
        print(f"bench.py: {world} rank(s) need {need} GPU(s); {torch.cuda.device_count()} visible", file=sys.stderr)
        sys.exit(2)
    gpu = 0 if args.share_gpu else local_rank
    if world > 1 or args.dist:
        import torch.distributed as dist
        if world == 1:  # (standalone --dist: a one-rank group on the loopback address)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(gpu)
        dist.init_process_group("gloo" if args.share_gpu else "nccl", device_id=None if args.share_gpu else torch.device("cuda", gpu))
    if args.workload == "config4":
        line = run_config4(args, world, rank, gpu, dist)
        if line is not None:
            print(json.dumps(line))
        if dist is not None:
            dist.destroy_process_group()
        return
    import crdt_amd
    from crdt_amd.traces import load_remote_wire

    wire = load_remote_wire(args.trace)
    n_ops_doc, n_recs_doc, n_txn_doc = wire_ops(wire)
    doc0, n = shard(rank, world, args.docs)
    names = [doc_name(doc0 + i) for i in range(n)]
    # the wire's name table: index 0 is "jeremy" (the trace author); replace it per document
    eng = crdt_amd.Engine(n, 32, device=gpu)
    eng.device_intern(not args.host_intern)  # staging's name interning: k_intern (one wave per document)
    t0 = time.time()
    eng.stage_remote_replicated(wire, 0, names)
    stage_s = time.time() - t0
    st = eng.run()  # untimed: sizes capacities (growth) for this workload
    assert (st == 0).all(), np.unique(st)
    eng.publish_async()
    eng.sync()
    eng.fit()  # capacities = what this stream uses (the timed replays need exactly that)
    mem = eng.mem_bytes()
    lens = eng.lens()
    # query batch (device resident): positions spread over every document
    rng = np.random.default_rng(1234 + rank)
    q = args.queries
    qdoc = np.repeat(np.arange(n, dtype=np.uint32), q)
    qpos = (rng.random(n * q) * np.repeat(lens, q)).astype(np.uint32)
    dev = torch.device("cuda", gpu)
    d_doc = torch.from_numpy(qdoc.view(np.int32)).to(dev)
    d_pos = torch.from_numpy(qpos.view(np.int32)).to(dev)
    d_ag = torch.zeros(n * q, dtype=torch.int16, device=dev)
    d_seq = torch.zeros(n * q, dtype=torch.int32, device=dev)
    d_p2 = torch.zeros(n * q, dtype=torch.int32, device=dev)
    d_del = torch.zeros(n * q, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    L = eng.L

    def queries():
        if q:
            L.crdt_pos_to_loc_dev_async(eng.h, n * q, d_doc.data_ptr(), d_pos.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr())
            L.crdt_loc_to_pos_dev_async(eng.h, n * q, d_doc.data_ptr(), d_ag.data_ptr(), d_seq.data_ptr(),
                                        d_p2.data_ptr(), d_del.data_ptr())

    for _ in range(args.warmup):
        eng.reset_async()
        eng.run_async()
        eng.publish_async()
        queries()
    eng.sync()
    torch.cuda.synchronize()
    # HIP events on the engine stream around the replay kernel (the dominant kernel)
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
        queries()
        hip.hipEventSynchronize(ev[1])
        ms = C.c_float()
        hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1])
        replay_ms.append(ms.value)
    eng.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    # parity: every document's state digest == the committed oracle digest, and every timed query
    # answer round-trips (loc_to_pos(pos_to_loc(p)) == p, visible, by the document's only author)
    st = eng.status()
    ok = bool((st == 0).all())
    q_ok = bool(((d_p2 == d_pos) & (d_del == 0) & (d_ag == 0)).all().item()) if q else True
    gseq = golden_pos_seq(args.trace)  # every timed pos -> loc answer against the oracle's (fixture)
    gpos = golden_seq_pos(args.trace)  # every timed loc -> pos answer against the oracle's (fixture)
    q_gold = q_gold_loc = None
    if q and gseq is not None and int(lens.min()) == gseq.shape[0] == int(lens.max()):
        g = torch.from_numpy(gseq.view(np.int32)).to(dev)
        q_gold = bool((d_seq == g[d_pos.long()]).all().item())
        q_ok = q_ok and q_gold
    if q and gpos is not None:
        gp = torch.from_numpy(gpos[0].view(np.int32)).to(dev)
        gd = torch.from_numpy(gpos[1]).to(dev)
        sq = d_seq.long()
        ix = sq.clamp(0, gp.shape[0] - 1)
        q_gold_loc = bool(((sq >= 0) & (sq < gp.shape[0])).all().item()) and \
            bool(((d_p2 == gp[ix]) & (d_del == gd[ix])).all().item())
        q_ok = q_ok and q_gold_loc
    dg = eng.digests()
    t_max, per_rank, all_dg = reduce_over_ranks(elapsed, dg, dist, torch.device("cpu") if args.share_gpu else dev)
    gold = golden(args.trace, "remote_digest")
    gold = int(gold, 16) if gold else None
    ok = ok and q_ok and bool((all_dg == all_dg[0]).all()) and (gold is None or int(all_dg[0]) == gold)
    mat = materialize_leg(eng, args.trace, n, hip, ev, s_) if not args.no_text else None
    sz = eng.export_sizes(0)
    eng.close()  # (frees the config-2 pools before the other legs allocate theirs)
    torch.cuda.empty_cache()
    stated = None
    if world == 1 and n != 4096 and not args.no_stated_size:
        stated = stated_size_leg(args, wire, n_ops_doc, hip)
    # the north star's corpus (BASELINE config 4: 1 M random-edit documents, document-sharded over
    # the ranks -- strong scaling at N > 1), measured in the same run after the config-2 leg
    corpus = None
    if not args.no_corpus:
        corpus = run_config4(args, world, rank, gpu, dist, steps=args.corpus_steps, warmup=args.corpus_warmup,
                             cpu_s=args.cpu_seconds / 2)
    total_ops = n_ops_doc * int(all_dg.shape[0]) * args.steps
    value = total_ops / t_max
    ms_step = t_max / args.steps * 1e3
    rms = float(np.mean(replay_ms)) if replay_ms else None
    # roofline of k_replay, SURVEY §8(d) algorithmic bytes for one launch = the whole trace per
    # document, starting from empty documents (S = 0): 32 B per final canonical span (16 B span
    # written + 8 B vpos/rpos + 8 B order->span) + 24 B per op (16 B op in + 8 B result out)
    canon = sz["canon"]
    alg_bytes = n * (32 * canon + 24 * n_ops_doc)
    achieved = alg_bytes / (rms * 1e-3) / 1e9 if rms else None
    enc_bytes = n * (n_recs_doc * 16 + sz["raw"] * 16 + sz["leaves"] * 12 + sz["next_order"] * 4)
    out = None
    if rank == 0:
        cpu = cpu_baseline(wire, n_ops_doc, args.cpu_seconds) if not args.no_cpu else None
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
                       "docs_per_gpu": n, "ops_per_doc": n_ops_doc,
                       "parallelism": f"doc-sharded x{world}" + (" (rehearsal: every rank on cuda:0, gloo)" if args.share_gpu else ""),
                       "waves_per_simd": n / SIMDS, "hbm_bytes_per_doc": mem / n},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": measured_traffic(n),
                         "kernel": "k_replay<32>", "kernel_ms": rms, "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_formula": "SURVEY 8(d): docs x (32 B x canonical spans + 24 B x ops)",
                         "canonical_spans_per_doc": canon,
                         "encoding_bytes_per_launch": enc_bytes,
                         "encoding_bytes_note": "the engine's own record stream + final raw state (not algorithmic)"},
            "cpu_baseline": cpu,
            "parity_ok": ok,
            "parity": "every document's digest == committed oracle golden digest (tests/golden); every timed "
                      "pos->loc answer == the oracle's (tests/golden/ap_remote_pos_seq.delta.gz), every timed "
                      "loc->pos answer == the oracle's (tests/golden/ap_remote_seq_pos.delta.gz), and they "
                      "round-trip",
            "queries_vs_oracle_fixture": q_gold,
            "loc_queries_vs_oracle_fixture": q_gold_loc,
            "queries_ok": q_ok,
            "world_size": dist.get_world_size() if dist is not None else 1,
            "per_rank_ops_s": [n_ops_doc * n * args.steps / t for t in per_rank],
            "build_id": crdt_amd.build_id(),
            "stage_s": stage_s,
            "stage_intern": "host" if args.host_intern else "device (k_intern)",
            "materialize": mat,
            "stated_size": stated,
            "corpus": corpus,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
