#!/bin/bash
# k_marg with batched band-chunk loads: ICE tests + C2 / C4 kernel times
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/marg && export TMPDIR=/tmp
O=gpurun_out/marg
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k2 -o c2 -- python3 -u bench.py --config c2 --no-cpu --steps 50 --warmup 2 > $O/c2_prof.log 2>&1 || exit 1
cp $(find /tmp/k2 -name "*kernel_stats.csv" | head -1) $O/c2_kernel_stats.csv
tail -1 $O/c2_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'])"
timeout -k 10 300 python3 -u bench.py --config c2 --steps 300 --warmup 10 --no-cpu > $O/c2.log 2>&1 || exit 1
tail -1 $O/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'])"
python3 -c "
import csv
for r in csv.DictReader(open('$O/c2_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('marg','update','sweep')): print(r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
