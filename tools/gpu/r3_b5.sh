#!/bin/bash
# GW check fix + flat cross-tile prefetch A/B + ICE tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ice_gpu.py -m gpu > $O/r3_b5_ice_tests.log 2>&1
rc=$?; echo "ice tests rc=$rc"; tail -2 $O/r3_b5_ice_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u tools/probe_knobs.py --iters 20 "flatw_pipe=0" "flatw_pipe=1" "flatw_pipe=2" > $O/r3_flatw_pipe_ab.log 2>&1 || exit 1
grep sweep $O/r3_flatw_pipe_ab.log
bash tools/gpu/r3_gwm.sh || exit 1
