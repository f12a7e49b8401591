#!/bin/bash
# side streams made on first use: ICE / dist tests, e2e + drop-in phases, C4 line
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/lazy && export TMPDIR=/tmp
O=gpurun_out/lazy
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_bench_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in e2e dropin; do timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 1 --no-cpu > $O/$c.log 2>&1 || exit 1
  tail -1 $O/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],3), d['phases_median'])"; done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', round(d['value'],1), d['ms_per_step'])"
