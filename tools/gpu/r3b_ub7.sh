#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py tests/test_ice_gpu.py -m gpu -k "uband or flat or sharded or band" > $O/ub7_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/ub7_tests.log; grep -m5 "FAILED\|Error" $O/ub7_tests.log; [ $rc -eq 0 ] || exit $rc
for fg in 33 44 66; do
timeout -k 10 300 python -u tools/probe_knobs.py --build flat_group=$fg "uband=1" "uband=0" "band_concurrent=0" > $O/ub7_c4_g$fg.log 2>&1; echo "c4 g$fg rc=$?"; grep -v amdgpu.ids $O/ub7_c4_g$fg.log | grep "\[1\]"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/u7 -o c4 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $GRAFT_REPO_ROOT/$O/ub7_prof.log 2>&1; echo "prof rc=$?"
cp $(find /tmp/u7 -name "c4_kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/$O/ub7_c4_kernel_stats_1stream.csv; head -6 $GRAFT_REPO_ROOT/$O/ub7_c4_kernel_stats_1stream.csv | cut -c1-120
