#!/bin/bash
# k_sweep_all (C2 / C3 one-launch sweep) at 3 vs 4 blocks per CU
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
for cfg in c3 c2; do for t in "all_minb=3" "all_minb=4"; do
HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu > $O/all_${cfg}_$t.log 2>&1 || exit 1
echo "$cfg $t $(tail -1 $O/all_${cfg}_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
