#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config gw --steps 2 --warmup 1 --gw-t 2e8 --gw-h 2e8 > gpurun_out/r2_gw_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config gw --steps 3 --warmup 1 >> gpurun_out/r2_gw_bench.log 2>&1
