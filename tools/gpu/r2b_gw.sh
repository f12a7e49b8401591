#!/bin/bash
# sparse GW with the packed column list: tests, bench line, kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/gw && export TMPDIR=/tmp
O=gpurun_out/gw
timeout -k 10 600 python -u -m pytest tests/test_gw_sparse_gpu.py tests/test_twostep_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config gw --steps 5 --warmup 1 > $O/gw.log 2>&1 || exit 1
tail -1 $O/gw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gw', round(d['value'],3), d['ms_per_step'], d.get('phases_median') or d.get('phases'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kg -o gw -- python3 -u bench.py --config gw --steps 1 --warmup 1 --no-cpu > $O/gw_prof.log 2>&1 || exit 1
cp $(find /tmp/kg -name "*kernel_stats.csv" | head -1) $O/gw_kernel_stats.csv
echo done
