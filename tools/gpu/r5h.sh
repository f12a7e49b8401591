#!/bin/bash
# TwoStep batch stream scaling; the new uband rule on C3 / cis.  tools/gpu/r5h.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python3 -u tools/probe_twostep.py 1 2 4 8 16 > $O/ts_q4.log 2>&1 || { tail -20 $O/ts_q4.log; exit 1; }
cat $O/ts_q4.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python3 -u tools/probe_twostep.py 4 8 16 > $O/ts_q16.log 2>&1 || { tail -20 $O/ts_q16.log; exit 1; }
cat $O/ts_q16.log
for cfg in c3 cis c2; do
timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu > $O/${cfg}_bench.log 2>&1 || { tail -20 $O/${cfg}_bench.log; exit 1; }
grep '^{"metric"' $O/${cfg}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'], round(d['value'],1), round(d['ms_per_step'],4), 'sweep', round(r['sweep_ms_avg'],4), 'iter', round(r['iter_ms_avg'],4))"
done
