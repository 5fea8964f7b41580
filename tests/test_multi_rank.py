"""World-size-2 rehearsal (gloo, CPU) of bench.py's multi-GPU path.

Documents shard across ranks by contiguous ranges with no per-op communication; the only
collectives are the max over ranks of the elapsed time and one all-gather of the per-document
digests.  The same helpers run over RCCL on the GPU box; here they run over gloo.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, docs_per_rank, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    doc0, n = bench.shard(rank, world, docs_per_rank)
    # stand-in per-document digests: a function of the global document id only
    dg = np.array([bench.splitmix64(doc0 + i) for i in range(n)], dtype=np.uint64)
    t_max, all_dg = bench.reduce_over_ranks(0.25 + rank, dg, dist, torch.device("cpu"))
    q.put((rank, doc0, n, t_max, all_dg.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_shard_and_reduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    per = 5
    ps = [ctx.Process(target=_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    import bench
    expect = [bench.splitmix64(d) for d in range(world * per)]
    for rank, doc0, n, t_max, all_dg in res:
        assert (doc0, n) == (rank * per, per)          # contiguous, disjoint, covering ranges
        assert t_max == 0.25 + (world - 1)              # max over ranks
        assert all_dg == expect                         # rank-ordered all-gather of every document
