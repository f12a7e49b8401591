#!/bin/bash
# upper-band sweep v2: its tests + ICE tests, then C4 and C2 sweep A/B, rocprof of the C4 sweep kernels (one stream)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py tests/test_ice_gpu.py -m gpu > $O/ub2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ub2_tests.log; grep -m5 "FAILED\|Error" $O/ub2_tests.log
timeout -k 10 300 python -u tools/probe_knobs.py "uband=0" "uband=1" "uband=1,band_concurrent=0" > $O/ub2_c4.log 2>&1; echo "c4 rc=$?"; grep -v amdgpu.ids $O/ub2_c4.log
timeout -k 10 200 python -u tools/probe_knobs.py --config c2 --iters 200 "uband=0" "uband=2" > $O/ub2_c2.log 2>&1; echo "c2 rc=$?"; grep -v amdgpu.ids $O/ub2_c2.log
cd /tmp && HH_TUNE=band_concurrent=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ub2prof -o c4 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $GRAFT_REPO_ROOT/$O/ub2_prof.log 2>&1; echo "prof rc=$?"
f=$(find /tmp/ub2prof -name "c4_kernel_stats.csv" | head -1); cp $f $GRAFT_REPO_ROOT/$O/ub2_c4_kernel_stats.csv; head -12 $f | cut -c1-200
