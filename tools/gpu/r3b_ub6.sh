#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py -m gpu > $O/ub6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/ub6_tests.log; grep -m5 "FAILED\|Error" $O/ub6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_knobs.py "uband=0" "uband=1" > $O/ub6_c4.log 2>&1; echo "c4 rc=$?"; grep -v amdgpu.ids $O/ub6_c4.log
timeout -k 10 200 python -u tools/probe_knobs.py --config c2 --iters 200 "uband=0" "uband=2" > $O/ub6_c2.log 2>&1; echo "c2 rc=$?"; grep -v amdgpu.ids $O/ub6_c2.log
timeout -k 10 400 python3 -u tools/probe_shards.py 8 1 > $O/ub6_shards.log 2>&1; echo "shards rc=$?"; grep -v amdgpu.ids $O/ub6_shards.log | grep "world=8:"
