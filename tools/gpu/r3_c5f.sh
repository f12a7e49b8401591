#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c5_gpu.py tests/test_structure_gpu.py -m gpu > $O/r3_c5f_tests.log 2>&1
rc=$?; echo "c5 tests rc=$rc"; tail -2 $O/r3_c5f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/pca_trace.py 1 --p 8 --coop 1 --reps 1 --debug 2 > $O/r3_c5f_phases.log 2>&1 || exit 1
grep "mode=0" $O/r3_c5f_phases.log | head -8
grep "mode=1\|mode=3" $O/r3_c5f_phases.log | head -2
grep "cycle=" $O/r3_c5f_phases.log | tail -2
timeout -k 10 300 python3 -u tools/pca_trace.py 1 21 --p 8 --coop 1 --reps 3 > $O/r3_c5f_wall.log 2>&1 || exit 1
grep Get_PCA $O/r3_c5f_wall.log
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/r3_c5f_bench.log 2>&1 || exit 1
tail -1 $O/r3_c5f_bench.log | cut -c1-1300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5fprof -o c5 -- python3 -u $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/r3_c5f_prof.log 2>&1 || exit 1
echo prof ok
