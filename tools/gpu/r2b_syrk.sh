#!/bin/bash
# double-buffered split-K syrk: compartment tests, then C5 A/B (auto split vs none)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/syrk && export TMPDIR=/tmp
O=gpurun_out/syrk
timeout -k 10 600 python -u -m pytest tests/test_c5_gpu.py tests/test_structure_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for x in -1 0 -1 0; do
  HH_TUNE=syrk_split=$x timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu > $O/c5_s$x.log 2>&1 || exit 1
  tail -1 $O/c5_s$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('split=$x', round(d['value'],2), 'syrk', round(r['achieved'],2) if r['kernel']=='k_syrk' else r['other_kernel']['achieved'], d['config']['serial_step_ms'])"
done
echo done
