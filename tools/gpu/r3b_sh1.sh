#!/bin/bash
# per-kernel times of C4 shards (N = 8) on one stream
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
cd /tmp
for k in 0 7; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/sh$k -o s --output-format csv -- python3 -u $R/tools/probe_knobs.py --shard $k/8 --iters 20 "band_concurrent=0" > $O/sh1_$k.log 2>&1; echo "shard $k rc=$?"; grep "\[1\]\|build" $O/sh1_$k.log
cp $(find /tmp/sh$k -name "s_kernel_stats.csv" | head -1) $O/sh1_${k}_kernel_stats.csv
python3 - <<PY
import csv
for r in csv.DictReader(open('$O/sh1_${k}_kernel_stats.csv')):
    if 'synth' in r['Name'] or 'rocclr' in r['Name']: continue
    print(f"   {r['Name'][:40]:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1000:8.1f} us")
PY
done
