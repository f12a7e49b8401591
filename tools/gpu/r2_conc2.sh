#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ice_gpu.py tests/test_dist_gpu.py > gpurun_out/r2_conc2_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu > gpurun_out/r2_conc2_c3.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2_conc2_c4.log 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/probe_shards.py 8 1 > gpurun_out/r2_conc2_shards.log 2>&1
