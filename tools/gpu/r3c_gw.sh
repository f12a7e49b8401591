#!/bin/bash
# GW statistics with row-bound range tests: GW tests + gw bench line + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gw_sparse_gpu.py > $O/gw_tests.log 2>&1; rc=$?; tail -2 $O/gw_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config gw --no-cpu > $O/gw_bench.log 2>&1 || exit 1
tail -1 $O/gw_bench.log | cut -c1-260
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/gwp -o gw --output-format csv -- python3 -u $R/bench.py --config gw --no-cpu --steps 2 --warmup 1 > $O/gw_prof.log 2>&1 || exit 1
cp $(find /tmp/gwp -name "gw_kernel_stats.csv" | head -1) $O/gw_kernel_stats.csv
head -16 $O/gw_kernel_stats.csv | cut -c1-140
