#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py -m gpu -k "flat" > $O/fw1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/fw1_tests.log; grep -m5 "FAILED\|Error" $O/fw1_tests.log; [ $rc -eq 0 ] || exit $rc
for fg in 16 22 33; do
timeout -k 10 300 python -u tools/probe_knobs.py --build flat_group=$fg "flatw_waves=8" "flatw_waves=10" "flatw_waves=11" "flatw_waves=11,flatw_pipe=0" > $O/fw1_c4_g$fg.log 2>&1; echo "c4 g$fg rc=$?"; grep -v amdgpu.ids $O/fw1_c4_g$fg.log | grep "\[1\]"
done
