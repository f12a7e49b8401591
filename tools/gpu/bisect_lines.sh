#!/bin/bash
# bench lines of older builds (git worktrees under bisect/<commit>, built
# in-tree): tools/gpu/bisect_lines.sh outdir "c3 c2" commit ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=$PWD/gpurun_out/$1; CFGS=$2; shift 2; mkdir -p $O
for c in "$@"; do
  for cfg in $CFGS; do
    (cd bisect/$c && timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu > $O/${c}_$cfg.log 2>&1) || { echo "$c $cfg failed"; tail -3 $O/${c}_$cfg.log; exit 1; }
    echo "$c $cfg $(tail -1 $O/${c}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))")"
  done
done
