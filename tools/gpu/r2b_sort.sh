#!/bin/bash
# radix scatter with wave-private ranking: sort users' tests, pairs / drop-in / gw lines
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/sort && export TMPDIR=/tmp
O=gpurun_out/sort
timeout -k 10 600 python -u -m pytest tests/test_pairs_gpu.py tests/test_build_gpu.py tests/test_gw_sparse_gpu.py tests/test_impute_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in pairs dropin gw e2e; do HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 1 --no-cpu > $O/$c.log 2>&1 || exit 1
  tail -1 $O/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],3), d['ms_per_step'])"; done
grep "radix sort" $O/dropin.log | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kp -o p -- python3 -u bench.py --config pairs --no-cpu --steps 3 --warmup 1 > $O/pairs_prof.log 2>&1 || exit 1
cp $(find /tmp/kp -name "*kernel_stats.csv" | head -1) $O/pairs_kernel_stats.csv
echo done
