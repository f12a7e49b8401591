#!/bin/bash
# Round-2 final, part 3: the drop-in / pipeline lines after the build and GW fixes
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/final && export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 300 python3 -u bench.py --config dropin --steps 3 --warmup 1 > $O/r2_dropin_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config dropin --steps 3 --warmup 1 --fixed-iters > $O/r2_dropin_fixed_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config e2e --steps 3 --warmup 1 > $O/r2_e2e_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config gw --steps 3 --warmup 1 > $O/r2_gw_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kg -o gw -- python3 -u bench.py --config gw --steps 1 --warmup 1 > $O/r2_gw_prof.log 2>&1 || exit 1
cp $(find /tmp/kg -name "*kernel_stats.csv" | head -1) $O/r2_gw_kernel_stats.csv
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r2_c4_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gw_sparse_gpu.py tests/test_fullsize_gpu.py tests/test_coolio.py > $O/r2_final3_tests.log 2>&1
