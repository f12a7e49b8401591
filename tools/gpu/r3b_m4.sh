#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py tests/test_uband_gpu.py tests/test_dist_gpu.py tests/test_build_gpu.py -m gpu > $O/m4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/m4_tests.log; grep -m5 "FAILED\|Error" $O/m4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu > $O/m4_c3_bench.log 2>&1; echo "c3 rc=$?"; tail -1 $O/m4_c3_bench.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu --steps 200 > $O/m4_c2_bench.log 2>&1; echo "c2 rc=$?"; tail -1 $O/m4_c2_bench.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/m4_c4_bench.log 2>&1; echo "c4 rc=$?"; tail -1 $O/m4_c4_bench.log | cut -c1-200
