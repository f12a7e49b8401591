#!/bin/bash
# stats modes (auto: fused <= 128 tiles, else 4 launches without tails) + unit_lpt_lists A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/modes && export TMPDIR=/tmp
O=gpurun_out/modes
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for x in 3 1 3 1; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 --build unit_lpt_lists=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/lists=$x c4: /" >> $O/ab.log || exit 1
  timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 200 --build unit_lpt_lists=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/lists=$x c3: /" >> $O/ab.log || exit 1
  for k in 0 7; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 --build unit_lpt_lists=$x "band_lpt=1" 2>&1 | grep "shard iter" | sed "s/^/lists=$x shard $k: /" >> $O/ab.log || exit 1; done
done
sort $O/ab.log
for c in c4 c3 c2; do timeout -k 10 300 python3 -u bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/${c}_bench.log 2>&1 || exit 1
  tail -1 $O/${c}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'])"; done
HH_TUNE=conc_min_bytes=1000000000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k41 -o c41 -- python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $O/c4_prof_1stream.log 2>&1 || exit 1
cp $(find /tmp/k41 -name "*kernel_stats.csv" | head -1) $O/c4_kernel_stats_1stream.csv
echo done
