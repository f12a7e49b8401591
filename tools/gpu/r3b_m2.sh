#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py -m gpu -k "flat" > $O/m2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/m2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/probe_shards.py 2,4,8 1 > $O/m2_shards.log 2>&1; echo "shards rc=$?"; grep "world=.:" $O/m2_shards.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/m2_c4_bench.log 2>&1; echo "bench rc=$?"; tail -1 $O/m2_c4_bench.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py --config c4h --no-cpu > $O/m2_c4h_bench.log 2>&1; echo "c4h rc=$?"; tail -1 $O/m2_c4h_bench.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu > $O/m2_c3_bench.log 2>&1; echo "c3 rc=$?"; tail -1 $O/m2_c3_bench.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu --steps 200 > $O/m2_c2_bench.log 2>&1; echo "c2 rc=$?"; tail -1 $O/m2_c2_bench.log | cut -c1-250
