#!/bin/bash
# GW merge (fixed) + band DPP A/B + ICE tests + C5 trace + C4 one-stream profile
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
bash tools/gpu/r3_gwm.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ice_gpu.py -m gpu > $O/r3_b4_ice_tests.log 2>&1
rc=$?; echo "ice tests rc=$rc"; tail -2 $O/r3_b4_ice_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u tools/probe_knobs.py --iters 20 "band_dpp=0" "band_dpp=1" "band_dpp=0,band_concurrent=0" "band_dpp=1,band_concurrent=0" > $O/r3_band_dpp_ab.log 2>&1 || exit 1
grep sweep $O/r3_band_dpp_ab.log
timeout -k 10 300 python3 -u tools/pca_trace.py 21 1 --p 8 > $O/r3_pca_trace.log 2>&1 || exit 1
tail -3 $O/r3_pca_trace.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c4prof -o c4 -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --iters 10 "band_concurrent=0" > $GRAFT_REPO_ROOT/$O/r3_c4_prof.log 2>&1 || exit 1
echo c4 prof ok
