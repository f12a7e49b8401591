#!/bin/bash
# e2e (sparse 10 kb genome-wide matrix, 22 572 tiles): single-launch sweep vs the three kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/e2es && export TMPDIR=/tmp
O=gpurun_out/e2es
for t in "" "sweep_single=0" "" "sweep_single=0"; do
  HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config e2e --steps 5 --warmup 1 --no-cpu > $O/e2e.log 2>&1 || exit 1
  tail -1 $O/e2e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[${t:-default}]', round(d['value']/1e9,3), d['phases_median'])"
done
