#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 20 "band_rows=0" "band_concurrent=0" "band_rows=0" > gpurun_out/r2_bandvgpr.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kb -o kb -- python3 -u tools/probe_knobs.py --iters 10 "band_concurrent=0" > gpurun_out/r2_bandvgpr_prof.log 2>&1 || exit 1
cp $(find /tmp/kb -name "*kernel_stats.csv" | head -1) gpurun_out/r2_bandvgpr_kernel_stats.csv
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ice_gpu.py > gpurun_out/r2_bandvgpr_tests.log 2>&1
