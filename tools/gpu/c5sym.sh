#!/bin/bash
# C5: the upper-triangle product kernels A/B (cor_sym 1 vs 2) + the sym tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_c5_gpu.py -k "sym or one_launch or small_autosomes" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 2 1 2; do
  HH_TUNE=cor_sym=$v timeout -k 10 300 python -u bench.py --config c5 --no-cpu > $O/c5_sym$v.log 2>&1 || exit 1
  echo "cor_sym=$v $(tail -1 $O/c5_sym$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value'],1), d['config']['serial_step_ms'], [(k['kernel'][:8], round(k['total_ms'],1), round(k['frac'],3)) for k in [r]+r['other_kernels']])")"
done
