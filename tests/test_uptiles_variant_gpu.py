"""The upper-triangle-tile cases against the library build
that has them: libhichap_hip_up.so (4096-column tiles, -DHH_KWBITS=12).  The
default library (8192-column tiles, both triangles: faster on MI355X, §3d)
skips those cases; this test runs them in one child process with HH_LIB
pointing at the variant (one library per process: the tile width is a
compile-time layout constant)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UP_LIB = os.path.join(ROOT, "hichap_master_amd", "libhichap_hip_up.so")


def test_uptiles_cases_on_the_variant_build():
    from hichap_master_amd import _lib
    _lib.require_gpu()
    assert os.path.exists(UP_LIB), "libhichap_hip_up.so missing: run __graft_entry__.build()"
    files = ["tests/test_ice_gpu.py", "tests/test_uband_gpu.py", "tests/test_build_gpu.py", "tests/test_dist_gpu.py"]
    env = dict(os.environ, HH_LIB=UP_LIB)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        "-k", "uptiles", *files], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and "skipped" not in r.stdout.splitlines()[-1], tail
