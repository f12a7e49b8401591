#!/bin/bash
# round-3 start: GPU suite + smoke + default C4 bench line at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r3_gpu_tests_head.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r3_gpu_tests_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3_smoke_head.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 300 python3 -u bench.py > $O/r3_c4_bench_head.log 2>&1 || exit 1
tail -1 $O/r3_c4_bench_head.log
