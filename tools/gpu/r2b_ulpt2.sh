#!/bin/bash
# GPU suite at this build, then unit_lpt 1 (cost class) vs 2 (exact cost) A/B, default bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/ulpt2 && export TMPDIR=/tmp
O=gpurun_out/ulpt2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for x in 2 1 2 1; do
  for k in 0 7; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "shard iter" | sed "s/^/unit_lpt=$x shard $k: /" >> $O/ab.log || exit 1; done
  timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/unit_lpt=$x c4: /" >> $O/ab.log || exit 1
  timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 200 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/unit_lpt=$x c3: /" >> $O/ab.log || exit 1
done
sort $O/ab.log
for c in c4 c3 c2; do timeout -k 10 300 python3 -u bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/${c}_bench.log 2>&1 || exit 1
  tail -1 $O/${c}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'], r['frac'])"; done
echo done
