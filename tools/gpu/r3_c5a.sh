#!/bin/bash
# one-launch orthogonalisation: C5 tests, serial trace, bench line, profile
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c5_gpu.py -m gpu > $O/r3_c5a_tests.log 2>&1
rc=$?; echo "c5 tests rc=$rc"; tail -3 $O/r3_c5a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/pca_trace.py 21 1 --p 8 > $O/r3_c5a_trace.log 2>&1 || exit 1
tail -2 $O/r3_c5a_trace.log
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/r3_c5a_bench.log 2>&1 || exit 1
tail -1 $O/r3_c5a_bench.log | cut -c1-900
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5aprof -o c5 -- python3 -u $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/r3_c5a_prof.log 2>&1 || exit 1
echo prof ok
