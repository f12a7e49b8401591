#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config e2e --steps 2 --warmup 1 > gpurun_out/r2_buildphase_e2e.log 2>&1 || exit 1
HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config dropin --steps 2 --warmup 1 > gpurun_out/r2_buildphase_dropin.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kg -o gw -- python3 -u bench.py --config gw --steps 1 --warmup 1 > gpurun_out/r2_gw_prof.log 2>&1 || exit 1
cp $(find /tmp/kg -name "*kernel_stats.csv" | head -1) gpurun_out/r2_gw_kernel_stats.csv
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_build_gpu.py tests/test_ice_gpu.py > gpurun_out/r2_buildgw_tests.log 2>&1
