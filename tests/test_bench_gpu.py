"""bench.py's contract on the GPU: one JSON line with the driver's keys, at
N=1 (C1, the smallest config) and through the N>1 sharded path (2 ranks on
cuda:0 with the gloo exchange: the measured-cost partition, side-stream band
sweep, max-over-ranks timing and slowest-shard roofline all run)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline"}


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_gpu_c1():
    p = subprocess.run([sys.executable, "bench.py", "--config", "c1", "--steps", "5", "--warmup", "1", "--no-cpu"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_line(p.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["value"] > 0
    assert d["config"]["workload"] == "single-chrom-40kb-5000-bins" and d["config"]["resolution_bp"] == 40000
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["achieved"] > 0


def test_bench_two_ranks_sharded_path():
    env = dict(os.environ, HH_DEVICE="0", HH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--standalone",
           "--local-addr", "127.0.0.1", "bench.py", "--gpus", "2", "--nnz", "2e8", "--steps", "3", "--warmup", "1"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    d = _json_line(p.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "sharded x2" in d["config"]["parallelism"]
    assert 0 < d["roofline"]["shard_nnz_upper"] < d["config"]["nnz_upper"]


def test_bench_gpus_flag_launches_ranks_itself():
    """``bench.py --gpus 2`` with no launcher starts its
    own two ranks (here both on cuda:0 with the gloo exchange, HH_DEVICE) and
    reports n_gpus 2 from the sharded path."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HH_DEVICE="0", HH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--nnz", "2e8", "--steps", "3", "--warmup", "1"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    d = _json_line(p.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "sharded x2" in d["config"]["parallelism"]


def test_bench_gpus_flag_refuses_missing_devices():
    """More GPUs asked than the box has: non-zero exit and no JSON line, not a
    one-GPU number labelled n_gpus N."""
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HH_DEVICE")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--config", "c1", "--steps", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "visible GPUs" in p.stderr
