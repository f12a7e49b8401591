#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r2_dist_tests.log 2>&1
echo "tests rc=$?"
