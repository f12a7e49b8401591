#!/bin/bash
# fused ICE stats: ICE/dist/fullsize tests, then C2/C3/C4 A/B (fuse_stats 1 vs 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/fuse && export TMPDIR=/tmp
O=gpurun_out/fuse
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_build_gpu.py tests/test_bench_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3; do
  for f in 1 0 1; do
    HH_TUNE=fuse_stats=$f timeout -k 10 200 python3 -u bench.py --config $c --steps 200 --warmup 10 --no-cpu > $O/${c}_f$f.log 2>&1 || exit 1
    tail -1 $O/${c}_f$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c fuse=$f', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'])"
  done
done
for f in 1 0; do
  HH_TUNE=fuse_stats=$f timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/c4_f$f.log 2>&1 || exit 1
  tail -1 $O/c4_f$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c4 fuse=$f', round(d['value'],1), r['sweep_ms_avg'], r['iter_ms_avg'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kc2 -o c2 -- python3 -u bench.py --config c2 --steps 100 --warmup 5 --no-cpu > $O/c2_prof.log 2>&1 || exit 1
cp $(find /tmp/kc2 -name "*kernel_stats.csv" | head -1) $O/c2_kernel_stats.csv
echo done
