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
           "--steps", "1", "--warmup", "1", "--no-cpu", "--no-text", "--queries", "256"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["world_size"] == 2 and out["n_gpus"] == 2
    assert out["parity_ok"] and out["queries_ok"]
    assert len(out["per_rank_ops_s"]) == 2 and out["value"] > 0
