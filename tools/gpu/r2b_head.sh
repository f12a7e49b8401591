#!/bin/bash
# re-entry check of HEAD: GPU suite + smoke + C4 / C2 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/head && export TMPDIR=/tmp
O=gpurun_out/head
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/c4_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c2 --steps 100 --warmup 5 --no-cpu > $O/c2_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c3 --steps 100 --warmup 5 --no-cpu > $O/c3_bench.log 2>&1 || exit 1
echo done
