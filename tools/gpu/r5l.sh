#!/bin/bash
# TwoStep shared launches: 32-bit copies on / off, alternating.  tools/gpu/r5l.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
for r in 1 2; do
HH_TS_NARROW=2 timeout -k 10 200 python3 -u tools/probe_twostep.py 0 0 > $O/n2.log 2>&1 || { tail -5 $O/n2.log; exit 1; }
grep n_streams $O/n2.log | sed "s/^/narrow=2 /"
HH_TS_NARROW=1 timeout -k 10 200 python3 -u tools/probe_twostep.py 0 0 > $O/n1.log 2>&1 || { tail -5 $O/n1.log; exit 1; }
grep n_streams $O/n1.log | sed 's/^/narrow=1 /'
HH_TS_NARROW=0 timeout -k 10 200 python3 -u tools/probe_twostep.py 0 0 > $O/n0.log 2>&1 || { tail -5 $O/n0.log; exit 1; }
grep n_streams $O/n0.log | sed 's/^/narrow=0 /'
done
cd /tmp && HH_TS_NARROW=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pts -o ts --output-format csv -- python3 -u $R/tools/probe_twostep.py 0 > $O/ts_prof.log 2>&1 || exit 1
cp $(find /tmp/pts -name "ts_kernel_stats.csv" | head -1) $O/ts_kernel_stats.csv
python3 - $O/ts_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:9.2f} total_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
