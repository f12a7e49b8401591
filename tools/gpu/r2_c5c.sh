#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c5_gpu.py tests/test_structure_gpu.py > gpurun_out/r2_c5c_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/r2_c5c_bench.log 2>&1 || exit 1
HH_C5_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k5 -o c5 -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/r2_c5c_prof.log 2>&1 || exit 1
cp $(find /tmp/k5 -name "*kernel_stats.csv" | head -1) gpurun_out/r2_c5c_kernel_stats.csv
