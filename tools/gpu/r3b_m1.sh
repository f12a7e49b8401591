#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_build_gpu.py -m gpu > $O/m1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/m1_tests.log; grep -m5 "FAILED\|Error" $O/m1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/m1_c4_bench.log 2>&1; echo "bench rc=$?"; tail -1 $O/m1_c4_bench.log | cut -c1-250
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/m1 -o c4 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $GRAFT_REPO_ROOT/$O/m1_prof.log 2>&1; echo "prof rc=$?"
cp $(find /tmp/m1 -name "c4_kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/$O/m1_c4_kernel_stats_1stream.csv; head -7 $GRAFT_REPO_ROOT/$O/m1_c4_kernel_stats_1stream.csv | cut -c1-120
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python3 -u tools/probe_shards.py 2,4,8 1 > $O/m1_shards.log 2>&1; echo "shards rc=$?"; grep "world=.:" $O/m1_shards.log
