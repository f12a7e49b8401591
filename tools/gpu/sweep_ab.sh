#!/bin/bash
# C4 sweep A/B at the current build: GPU tests matching a -k pattern, the
# matrix's own read rates (hh_matrix_stream_probe), sweep times under each
# hh_tune setting, and per-kernel rocprof stats of a one-stream sweep per
# setting.  tools/gpu/sweep_ab.sh outdir "-k pattern" "k=v,..." "k=v,..." ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; K=$2; shift 2; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ice_gpu.py -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python3 -u tools/probe_knobs.py --stream --iters 20 "$@" > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
i=0
for spec in "$@"; do
  i=$((i+1))
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/psab$i -o s --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0,$spec" > $O/prof$i.log 2>&1 || { tail -5 $O/prof$i.log; exit 1; }
  cp $(find /tmp/psab$i -name "s_kernel_stats.csv" | head -1) $O/kstats_$i.csv
  python3 - $O/kstats_$i.csv "$spec" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("[%s]" % sys.argv[2], "  ".join("%s %.3f ms" % (r["Name"].split("<")[0].split("(")[0].replace("void ", ""), float(r["AverageNs"]) / 1e6)
      for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5] if "sweep" in r["Name"] or "marg" in r["Name"]))
PY
  cd $R
done
