#!/bin/bash
# C5 after the AVX2 host Rayleigh-Ritz: tests, line, per-cycle host time.  tools/gpu/r5m.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_c5_gpu.py tests/test_structure_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu > $O/c5_$k.log 2>&1 || { tail -5 $O/c5_$k.log; exit 1; }
echo "c5 $(grep '^{"metric"' $O/c5_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), d['unit'], d['config']['serial_phase_ms'])")"
done
HH_PCA_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 1 --warmup 0 > $O/c5_pcadebug.log 2>&1 || exit 1
python3 - $O/c5_pcadebug.log <<'PY'
import re, sys
h = e = g = 0.0; n = 0
for line in open(sys.argv[1]):
    m = re.search(r"host_ms H=([\d.]+) eig=([\d.]+) gpu_wait_ms=([\d.]+)", line)
    if m:
        h += float(m.group(1)); e += float(m.group(2)); g += float(m.group(3)); n += 1
print(f"pca cycles {n}: host H {h:.1f} ms, host eig {e:.1f} ms, gpu wait {g:.1f} ms (summed over all passes)")
PY
