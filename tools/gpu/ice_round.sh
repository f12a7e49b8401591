#!/bin/bash
# ICE layout / sweep change: the ICE-side GPU tests, the stream probes and
# sweep times (three streams) under the given hh_tune settings, the C4 bench
# line, and per-kernel rocprof stats of a one-stream sweep.
#   tools/gpu/ice_round.sh outdir "k=v,..." ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_ice_gpu.py tests/test_uband_gpu.py tests/test_build_gpu.py tests/test_uptiles_variant_gpu.py tests/test_dist_gpu.py tests/test_fullsize_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/probe_knobs.py --stream --iters 20 "$@" > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/c4_bench.log 2>&1 || { tail -5 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pir1 -o s --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
cp $(find /tmp/pir1 -name "s_kernel_stats.csv" | head -1) $O/kstats_1stream.csv
python3 - $O/kstats_1stream.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("1-stream:", "  ".join("%s %.3f ms" % (r["Name"].split("<")[0].split("(")[0].replace("void ", ""), float(r["AverageNs"]) / 1e6)
      for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:6] if "sweep" in r["Name"] or "marg" in r["Name"] or "interleave" in r["Name"]))
PY
