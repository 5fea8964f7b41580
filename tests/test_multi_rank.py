"""Multi-rank rehearsal (gloo, CPU) of bench.py's multi-GPU path.

Documents shard across ranks by contiguous ranges balanced by op count, with no per-op
communication; the only collectives are the max over ranks of the elapsed time, an all-gather of
per-rank times and one all-gather of the per-document digests.  The same helpers run over RCCL on
the GPU box; here they run over gloo.  Each rank of the world-2 test replays its real shard of a
mixed corpus (the oracle stands in for the GPU engine: this is CPU test infrastructure), and the
gathered digests must equal a single-rank replay of the same global corpus.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus(n_docs):
    """A small mixed corpus: doc d replays a prefix of [AP, RC, SV][splitmix64(d) % 3] (local
    txns), so documents carry different amounts of work (op counts = the shard weights)."""
    import bench
    from crdt_amd.traces import load_trace
    traces = [load_trace(n) for n in ("automerge-paper", "rustcode", "sveltecomponent")]
    docs = []
    for d in range(n_docs):
        t = traces[bench.splitmix64(d) % 3]
        k = 200 + int(bench.splitmix64(d ^ 0x55) % 1500)
        c = t.counts[:k]
        docs.append((c, t.patches[: int(c.sum())]))
    return docs


def _replay_digests(docs):
    from oracle_lib import OracleDoc
    out = []
    for c, p in docs:
        o = OracleDoc()
        assert o.apply_trace(o.agent("jeremy"), c, p) == 0
        out.append(o.digest())
    return np.array(out, dtype=np.uint64)


def _worker(rank, world, port, n_docs, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(ROOT, "text-crdt-rust_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs = _corpus(n_docs)
    weights = [int(p.shape[0]) for _, p in docs]
    doc0, n = bench.shard_balanced(weights, world, rank)
    dg = _replay_digests(docs[doc0:doc0 + n])       # this rank's shard only
    t_max, per_rank, all_dg = bench.reduce_over_ranks(0.25 + rank, dg, dist, torch.device("cpu"))
    q.put((rank, doc0, n, t_max, per_rank, all_dg.tolist()))
    dist.destroy_process_group()


def test_shard_balanced_ranges():
    import bench
    w = [5, 1, 1, 1, 1, 1, 10, 1, 1, 1, 1, 1]
    for world in (1, 2, 3, 4, 8):
        cuts = [bench.shard_balanced(w, world, r) for r in range(world)]
        lo = 0
        for a, n in cuts:                               # contiguous, disjoint, covering
            assert a == lo and n >= 0
            lo += n
        assert lo == len(w)
    # equal weights: the weak-scaling ranges [r*n, (r+1)*n)
    assert [bench.shard(r, 4, 3) for r in range(4)] == [(0, 3), (3, 3), (6, 3), (9, 3)]
    # balance: with 2 ranks the heavy document sits alone with few others
    (a0, n0), (a1, n1) = (bench.shard_balanced(w, 2, r) for r in range(2))
    s0, s1 = sum(w[a0:a0 + n0]), sum(w[a1:a1 + n1])
    assert abs(s0 - s1) <= max(w)


@pytest.mark.parametrize("world", [2])
def test_shards_replay_like_one_rank(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_docs = 10
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_docs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    import bench
    docs = _corpus(n_docs)
    single = _replay_digests(docs).tolist()             # the same global corpus on one rank
    weights = [int(p.shape[0]) for _, p in docs]
    for rank, doc0, n, t_max, per_rank, all_dg in res:
        assert (doc0, n) == bench.shard_balanced(weights, world, rank)
        assert t_max == 0.25 + (world - 1)              # max over ranks
        assert per_rank == [0.25 + r for r in range(world)]
        assert all_dg == single                         # rank-ordered gather == single-rank replay


@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_launches_ranks(gpus):
    # `bench.py --gpus N` started by hand spawns N ranks (torch.distributed.run) before any GPU
    # call; --rehearse-cpu runs the same shard / collective path over gloo without a GPU.
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--rehearse-cpu",
                        "--docs", "6"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["world_size"] == gpus and out["docs_total"] == 6 * gpus and out["parity_ok"]
    assert out["shards"] == [[6 * k, 6] for k in range(gpus)]


def test_bench_without_gpus_fails_cleanly():
    # no rehearsal flag and no GPU: the ranks exit with a message, not a crash
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--docs", "4"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode != 0
    assert "need 2 GPU(s)" in r.stderr


@pytest.mark.parametrize("gpus", [1, 2, 8])
def test_bench_config4_corpus_rehearsal(gpus):
    # `bench.py --gpus N --workload config4`: the 1 M-document corpus sharded into contiguous
    # ranges of 1 M / N, each rank's share in batches of <= 125,000; the rehearsal checks that the
    # shards and the gather cover every corpus document exactly once, in order
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--rehearse-cpu",
                        "--workload", "config4"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert out["parity_ok"] and out["docs_total"] == 1_000_000 and out["world_size"] == gpus
    assert out["shards"] == [[k * (1_000_000 // gpus), 1_000_000 // gpus] for k in range(gpus)]
    assert out["batches_per_rank"] == 8 // gpus and out["batch_docs"] == 125_000


def test_config4_batches_cover_a_ragged_share():
    import bench
    B, batches = bench.config4_batches(10, 333_334, 125_000)
    assert B == 111_112 and [m for _, m in batches] == [111_112, 111_112, 111_110]
    assert batches[0][0] == 10 and batches[-1][0] + batches[-1][1] == 10 + 333_334
