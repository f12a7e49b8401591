#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 200 python3 -u tools/probe_uband.py 14637 1 > $O/ub5_probe.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/ub5_probe.log | head -12
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu > $O/ub5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ub5_tests.log; grep -m5 "FAILED\|Error" $O/ub5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/ub5_c4_bench.log 2>&1; echo "bench rc=$?"; tail -1 $O/ub5_c4_bench.log | cut -c1-300
timeout -k 10 400 python3 -u tools/probe_shards.py 2,4,8 1 > $O/ub5_shards.log 2>&1; echo "shards rc=$?"; grep -v amdgpu.ids $O/ub5_shards.log | tail -12
