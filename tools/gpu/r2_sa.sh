#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_structure_gpu.py > gpurun_out/r2_sa_tests.log 2>&1 || exit 1
bash tools/gpu/r2_benchpath.sh
