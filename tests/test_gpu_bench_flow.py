"""bench.py's N-rank flow on the GPU box: `bench.py --gpus 2` launches its own two rank processes
(torchrun's environment), wraps the module in ddp.DataParallel, times with barrier + synchronize on both sides and
takes the max over ranks. Here the collectives go over gloo and both ranks share cuda:0 (MVAE_BENCH_BACKEND=gloo,
MVAE_BENCH_ONE_DEVICE=1 -- the production path is RCCL with one rank per GPU, which this 1-GPU box cannot run), on
the metric's own model (c4 architecture, 927 M parameters) at batch 4 per rank."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_two_rank_flow_c4():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MVAE_BENCH_BACKEND="gloo", MVAE_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c4", "--batch", "4",
           "--steps", "1", "--warmup", "1", "--no-kernel-timing"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8 and out["config"]["per_gpu_batch"] == 4
    assert out["config"]["backend"] == "gloo" and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["scaling"] == "weak"
    assert out["cpu_baseline"] is None  # rank 0 at N = 1 only
    assert abs(out["value"] - 8 / (out["ms_per_step"] * 1e-3)) <= 1e-2 * out["value"]
    assert out["loss"] == out["loss"]  # finite, not NaN


@pytest.mark.timeout(600)
def test_bench_two_rank_flow_c3_graphed():
    """c3 (a captured-graph config) at N = 2: the step is graph-replayed under data parallelism too (gloo: "split"
    capture, two graphs around the eager exchange)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MVAE_BENCH_BACKEND="gloo", MVAE_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c3", "--batch", "64",
           "--steps", "3", "--warmup", "1", "--no-kernel-timing"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 128
    assert out["config"]["step_launch"] == "hip graph (captured step, dp capture split)"
    assert out["value"] > 0 and out["loss"] == out["loss"]
