#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config dropin --steps 3 --warmup 1 --fixed-iters > gpurun_out/r2_dropin.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config dropin --steps 3 --warmup 1 >> gpurun_out/r2_dropin.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config e2e --steps 3 --warmup 1 > gpurun_out/r2_e2e.log 2>&1
