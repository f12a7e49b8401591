#!/bin/bash
# upper-band sweep v3: its tests + ICE/dist tests, the default C4 bench line, N=8/4/2 shard sweeps
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu > $O/ub3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ub3_tests.log; grep -m5 "FAILED\|Error" $O/ub3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/ub3_c4_bench.log 2>&1; echo "bench rc=$?"; tail -1 $O/ub3_c4_bench.log | cut -c1-400
timeout -k 10 400 python3 -u tools/probe_shards.py 2,4,8 1 > $O/ub3_shards.log 2>&1; echo "shards rc=$?"; grep -v amdgpu.ids $O/ub3_shards.log | tail -12
