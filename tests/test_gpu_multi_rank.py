"""The multi-rank bench path with the real engine (tests/test_multi_rank.py rehearses it on CPU
ranks with the oracle's digests): `bench.py --gpus 2 --share-gpu` launches two ranks through
torch.distributed.run exactly as `--gpus N` does, each rank replays its shard of the config-2
corpus on its own engine (both on cuda:0 of a one-GPU box) and the digests / times meet over gloo.
Every gathered digest must equal the committed golden digest."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_share_one_gpu():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--docs", "48",
           "--steps", "1", "--warmup", "1", "--no-cpu", "--no-text", "--queries", "256",
           "--corpus-docs", "1000", "--batch-docs", "300", "--corpus-steps", "1", "--check-docs", "4", "--gen-ops", "3000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["world_size"] == 2 and out["n_gpus"] == 2
    assert out["parity_ok"] and out["queries_ok"]
    assert len(out["per_rank_ops_s"]) == 2 and out["value"] > 0
    # the corpus leg (config 4) of the same line: 1,000 documents over the two ranks, 2 batches each
    c = out["corpus"]
    assert c["parity_ok"] and c["world_size"] == 2 and c["config"]["batches_per_gpu"] == 2
    assert c["collective"] == {"backend": "gloo", "gathered_docs": 1000, "gathered_equal_local": True}


def test_rccl_world_size_one():
    # RCCL had never run on hardware.  A one-rank process group over the nccl backend
    # (RCCL on ROCm) under torch.distributed.run --nproc-per-node=1, exactly as the driver's N-GPU
    # launch: the corpus leg's time reduction and digest all-gather go through RCCL, and the
    # gathered digests must equal the rank's own.
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           "--master-port=29533", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "--workload", "config4",
           "--corpus-docs", "8192", "--batch-docs", "4096", "--steps", "1", "--warmup", "1", "--no-cpu",
           "--check-docs", "8", "--gen-ops", "4000"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["world_size"] == 1 and out["parity_ok"]
    assert out["collective"] == {"backend": "nccl", "gathered_docs": 8192, "gathered_equal_local": True}
