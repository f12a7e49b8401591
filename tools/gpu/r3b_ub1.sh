#!/bin/bash
# upper-band sweep: ICE / dist / build GPU tests, then C4 and C2 sweep A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_build_gpu.py -m gpu > $O/ub1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ub1_tests.log; grep -m3 "FAILED\|Error\|error" $O/ub1_tests.log
timeout -k 10 300 python -u tools/probe_knobs.py "uband=0" "uband=1" > $O/ub1_c4.log 2>&1; echo "c4 rc=$?"; cat $O/ub1_c4.log | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/probe_knobs.py --config c2 --iters 200 "uband=0" "uband=1" > $O/ub1_c2.log 2>&1; echo "c2 rc=$?"; grep -v amdgpu.ids $O/ub1_c2.log
