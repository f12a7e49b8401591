#!/bin/bash
# the secondary bench lines at the final build: C5, gw, C3, C2, C4 haploid
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
for cfg in c5 gw c3 c2 c4h; do
timeout -k 10 400 python3 -u bench.py --config $cfg --no-cpu > $O/lines_$cfg.log 2>&1 || exit 1
echo "$cfg $(tail -1 $O/lines_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], d['ms_per_step'])")"
done
