#!/bin/bash
# k_ortho latency fixes: C5 tests / trace / bench / profile; GW windowed T stats; C4 PMC traffic
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
C=${1:-unknown}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_structure_gpu.py -m gpu > $O/r3_distst_tests.log 2>&1
rc=$?; echo "dist/structure tests rc=$rc"; tail -2 $O/r3_distst_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/pca_trace.py 21 1 --p 8 > $O/r3_c5b_trace.log 2>&1 || exit 1
tail -2 $O/r3_c5b_trace.log
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/r3_c5b_bench.log 2>&1 || exit 1
tail -1 $O/r3_c5b_bench.log | cut -c1-1200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5bprof -o c5 -- python3 -u $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/r3_c5b_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
echo c5 prof ok
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gw_sparse_gpu.py -m gpu > $O/r3_gwt_tests.log 2>&1
rc=$?; echo "gw tests rc=$rc"; tail -2 $O/r3_gwt_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config gw --steps 5 --warmup 2 --no-cpu > $O/r3_gwt_bench.log 2>&1 || exit 1
tail -1 $O/r3_gwt_bench.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/gwtprof -o gw -- python3 -u $GRAFT_REPO_ROOT/bench.py --config gw --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/r3_gwt_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
echo gw prof ok
rm -rf /tmp/pf /tmp/pw
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o f --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/r3_pmc_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o w --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/r3_pmc_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) $O/r3_c4_pmc.json "$C" 15202483080 > $O/r3_pmc_summary.log 2>&1 || exit 1
echo pmc ok
