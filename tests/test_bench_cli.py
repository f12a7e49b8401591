"""bench.py's --gpus handling on the CPU (no GPU call is reached): asking for
more GPUs than the node has, or a --gpus that disagrees with the launcher's
WORLD_SIZE, exits non-zero without printing a result line."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HH_DEVICE")}
    e.update(env)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=300)


def test_gpus_without_devices_exits_nonzero():
    p = _run(["--gpus", "2", "--config", "c1"], HIP_VISIBLE_DEVICES="")
    assert p.returncode != 0
    assert "visible GPUs" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_exits_nonzero():
    p = _run(["--gpus", "4", "--config", "c1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2
    assert "disagree" in p.stderr
