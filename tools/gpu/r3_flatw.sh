#!/bin/bash
# column-grouped flat sweep: ICE tests, then C4 A/B (round-2 flat kernel vs k_sweep_flatw, U 8 / 16)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ice_gpu.py tests/test_build_gpu.py -m gpu > $O/r3_flatw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r3_flatw_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r3_flatw_ab.log
for b in "flat_cols=0" "flat_cols=1"; do
  timeout -k 10 240 python3 -u tools/probe_knobs.py --iters 20 --build $b "flatw_u=8" "flatw_u=16" "band_concurrent=0,flatw_u=8" "band_concurrent=0,flatw_u=16" 2>&1 | grep -E "sweep|build" | sed "s/^/[$b] /" >> $O/r3_flatw_ab.log || exit 1
done
cat $O/r3_flatw_ab.log
