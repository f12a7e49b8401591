#!/bin/bash
# GW merge restructure: GW tests, bench line, kernel profile
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gw_sparse_gpu.py -m gpu > $O/r3_gwm_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r3_gwm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config gw --steps 5 --warmup 2 --no-cpu > $O/r3_gwm_bench.log 2>&1 || exit 1
tail -1 $O/r3_gwm_bench.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/gwmprof -o gw -- python3 -u $GRAFT_REPO_ROOT/bench.py --config gw --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/r3_gwm_prof.log 2>&1 || exit 1
echo prof ok
