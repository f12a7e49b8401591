#!/bin/bash
# TwoStep tests, the twostep lines, kernel stats of the per-genome line.  tools/gpu/twostep_line.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_twostep_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in twostep twostep_genome; do
timeout -k 10 300 python3 -u bench.py --config $c --no-cpu > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
python3 - $O/$c.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][0])
print(d["config"].get("workload"), round(d["value"], 2), d["unit"], round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 3))
PY
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pts -o ts --output-format csv -- python3 $R/bench.py --config twostep_genome --no-cpu > $O/prof.log 2>&1 || exit 1
cp $(find /tmp/pts -name "*kernel_stats.csv" | head -1) $O/ts_kernel_stats.csv
python3 - $O/ts_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    if "hh::" in r["Name"]:
        print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
