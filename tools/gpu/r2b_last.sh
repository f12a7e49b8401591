#!/bin/bash
# last check of HEAD: GPU suite + smoke + default C4 bench line + C2/C3
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/last && export TMPDIR=/tmp
O=gpurun_out/last
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r2b_gpu_tests_last.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r2b_gpu_tests_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r2b_smoke_last.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 300 python3 -u bench.py > $O/r2b_c4_bench_last.log 2>&1 || exit 1
for c in c3 c2; do timeout -k 10 300 python3 -u bench.py --config $c --steps 200 --warmup 10 --no-cpu > $O/r2b_${c}_bench_last.log 2>&1 || exit 1; done
for c in c4 c3 c2; do tail -1 $O/r2b_${c}_bench_last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', round(d['value'],1), d['ms_per_step'], r['frac'])"; done
