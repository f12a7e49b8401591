#!/bin/bash
# full GPU suite + smoke + default bench line at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/full3_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/full3_gpu_tests.log; grep -m3 "FAILED" $O/full3_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/full3_smoke.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 400 python3 -u bench.py > $O/full3_c4_bench.log 2>&1 || exit 1
tail -1 $O/full3_c4_bench.log | cut -c1-300
