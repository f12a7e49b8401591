#!/bin/bash
# TwoStep tests, then the twostep line under each HH_TUNE setting given
# (usage: twostep_ab.sh OUTDIR "symvc_stream=0" "symvc_rows=64" ...)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_twostep_gpu.py tests/test_oracle_golden.py > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
for rep in ${REPS:-0 1}; do
  for t in "$@"; do
    HH_TUNE="$t" timeout -k 10 120 python bench.py --config twostep --steps 50 --warmup 5 > "$out/b.json" 2> "$out/b.err" || { cat "$out/b.err"; exit 1; }
    python - "$t" "$rep" "$out/b.json" <<'PY' | tee -a "$out/ab.log"
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]}] {sys.argv[1]}: {d['value']:.1f} /s  {d['ms_per_step']:.4f} ms  frac {d['roofline']['frac']:.3f}")
PY
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /tmp/tsprof -o run --output-format csv -- python3 bench.py --config twostep --steps 20 --warmup 3 --no-cpu > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
f=$(find /tmp/tsprof -name "*kernel_stats.csv" | head -1); cp "$f" "$out/kernel_stats.csv"
python3 - "$out/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x {int(r['Calls']):5d}  {r['Name'][:70]}")
PY
