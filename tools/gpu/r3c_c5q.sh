#!/bin/bash
# C5 with the Cov triangle never split over K (the concurrent streams fill the chip) vs the cost model
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
for t in "syrk_split=0" "syrk_split=-1"; do
HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5q_$t.log 2>&1 || exit 1
echo "$t $(tail -1 $O/c5q_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['config']['serial_step_ms'], [(k['kernel'][:10], round(k['total_ms'],1), k['launches']) for k in [r]+r['other_kernels']])")"
done
