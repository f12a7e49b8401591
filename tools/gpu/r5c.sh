#!/bin/bash
# Round-5 upper-triangle tiles: parity tests first, then the per-kernel probe
# and the C4 bench line.  tools/gpu/r5c.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS_EXTRA}"
timeout -k 10 900 $T ${TESTS:-tests/test_uband_gpu.py tests/test_build_gpu.py tests/test_ice_gpu.py tests/test_dist_gpu.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u tools/probe_upper.py "upper_tiles=0" "upper_tiles=-1" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/c4_bench.log 2>&1 || { tail -20 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-600
