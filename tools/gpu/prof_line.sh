#!/bin/bash
# One bench line under rocprofv3 --kernel-trace --stats: the line's JSON and
# the per-kernel summary (top 12 by total time).
#   tools/gpu/prof_line.sh outdir config [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; CFG=$2; shift 2; mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pl_$CFG -o $CFG --output-format csv -- python3 -u $R/bench.py --no-cpu --config $CFG "$@" > $O/${CFG}_prof.log 2>&1 || { tail -20 $O/${CFG}_prof.log; exit 1; }
cp $(find /tmp/pl_$CFG -name "${CFG}_kernel_stats.csv" | head -1) $O/${CFG}_kernel_stats.csv
tail -1 $O/${CFG}_prof.log | cut -c1-400
python3 - $O/${CFG}_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:9.2f} total_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
