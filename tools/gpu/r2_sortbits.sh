#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_build_gpu.py tests/test_gw_sparse_gpu.py tests/test_fullsize_gpu.py tests/test_pairs_gpu.py > gpurun_out/r2_sortbits_tests.log 2>&1 || exit 1
HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config dropin --steps 3 --warmup 1 > gpurun_out/r2_sortbits_dropin.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config e2e --steps 3 --warmup 1 > gpurun_out/r2_sortbits_e2e.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config gw --steps 3 --warmup 1 > gpurun_out/r2_sortbits_gw.log 2>&1 || exit 1
