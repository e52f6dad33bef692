"""GPU: bench.py's multi-rank path as the driver starts it (`bench.py --gpus N`, no launcher).

Two ranks share the one GPU of a test box over gloo (RCCL refuses two ranks on one device); the
8-GPU scaling run uses the same code path with RCCL."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_bench_gpus_2_starts_two_ranks_and_migrates(gpu_available):
    """BASELINE config[2]'s shape at 64k entities per rank: bench.py starts both ranks itself,
    rank 0 prints one line with n_gpus = 2, and entities crossed shards (SwitchScene, KM:901-951)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--entities", "65536", "--groups", "256", "--steps", "3", "--warmup", "2",
                        "--cpu-baseline", "off"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    assert out["migrations"]["out"] > 0 and out["migrations"]["out"] == out["migrations"]["in"]
    assert out["value"] > 0 and out["config"]["entities_per_gpu"] == 65536
