#!/bin/bash
# Every bench.py line at the current build, one after the other, each under
# its own time limit; logs to gpurun_out/$1 (default gpurun_out/lines).
#   tools/gpu/lines.sh [outdir] [config ...]     (default: all configs)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/${1:-lines}; shift
mkdir -p $O
CFGS=${@:-c4 c4h c3 c2 cis c5 gw twostep twostep_genome dropin e2e pairs loops}
for cfg in $CFGS; do
  timeout -k 10 420 python3 -u bench.py --config $cfg > $O/$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 $O/$cfg.log; exit 1; }
  echo "$cfg $(grep '^{"metric"' $O/$cfg.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], round(d['ms_per_step'],3), (d.get('roofline') or {}).get('frac'))")"
done
