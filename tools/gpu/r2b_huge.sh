#!/bin/bash
# tile-plan arrays on THP-advised mappings: build/ICE tests, e2e + drop-in phase times
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/huge && export TMPDIR=/tmp
O=gpurun_out/huge
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1
timeout -k 10 600 python -u -m pytest tests/test_build_gpu.py tests/test_ice_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in e2e dropin; do HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 1 --no-cpu > $O/$c.log 2>&1 || exit 1
  tail -1 $O/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],3), d['ms_per_step'], d.get('phases_median'))"; done
grep "\[plan\]\|plan_tiles\|upload plan" $O/e2e.log | tail -6
