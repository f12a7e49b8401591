#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gw_sparse_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r2_gw_tests.log 2>&1
echo "tests rc=$?"
