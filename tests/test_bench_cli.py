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


def _fake_topology(tmp_path, gfx):
    """A KFD topology tree: one node per entry, gfx_target_version = entry
    (0 = a CPU node)."""
    root = tmp_path / "nodes"
    for i, v in enumerate(gfx):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if v else 8}\nsimd_count {256 if v else 0}\n"
                                      f"gfx_target_version {v}\nmax_waves_per_simd 8\n")
    return str(root)


def test_visible_gpu_count_from_sysfs(tmp_path):
    """The launcher counts GPUs from the KFD topology (nonzero
    gfx_target_version), narrowed by the *_VISIBLE_DEVICES variables."""
    root = _fake_topology(tmp_path, [0, 90500, 90500, 90500])
    code = "import bench; print(bench.visible_gpu_count())"
    base = {k: v for k, v in os.environ.items()
            if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    for extra, want in [({}, 3), ({"HIP_VISIBLE_DEVICES": "0,1"}, 2), ({"ROCR_VISIBLE_DEVICES": ""}, 0)]:
        env = dict(base, HH_KFD_TOPOLOGY=root, **extra)
        p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr
        assert int(p.stdout.strip()) == want, (extra, p.stdout)


def test_launcher_parent_never_loads_hip(tmp_path):
    """``bench.py --gpus N`` decides and spawns its ranks without loading the
    HIP runtime in the parent (an exec or a fork after HIP init is what the
    launcher must never do): with 2 GPUs in the topology it starts 2 ranks
    (here they exit at argument parsing), with 1 it refuses; in both cases
    libamdhip64 is absent from the parent's mappings."""
    code = ("import bench, sys\n"
            "rc = bench.launch_ranks(int(sys.argv[1]), ['--config', 'no-such-config'])\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(rc, 'libamdhip64' in maps, 'torch' in sys.modules)\n")
    base = {k: v for k, v in os.environ.items()
            if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "HH_DEVICE",
                         "WORLD_SIZE", "RANK", "LOCAL_RANK")}
    for ngpu in (2, 1):
        root = _fake_topology(tmp_path / str(ngpu), [0] + [90500] * ngpu)
        p = subprocess.run([sys.executable, "-c", code, "2"], cwd=ROOT, env=dict(base, HH_KFD_TOPOLOGY=root),
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr
        rc, hip, torch_loaded = p.stdout.split()
        assert int(rc) != 0  # children fail on the bad config / the refusal
        assert hip == "False" and torch_loaded == "False"
        if ngpu == 1:
            assert "visible GPUs" in p.stderr
        else:
            assert "exited with" in p.stderr
