#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_fullsize_gpu.py > gpurun_out/r2_full_tests.log 2>&1
echo "tests rc=$?"
