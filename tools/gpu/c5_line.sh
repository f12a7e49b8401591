#!/bin/bash
# C5 tests, the line and the serial low-synch k_ortho breakdown.  tools/gpu/c5_line.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_c5_gpu.py tests/test_structure_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu > $O/c5_1.log 2>&1 || { tail -5 $O/c5_1.log; exit 1; }
python3 - $O/c5_1.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][0])
r = d["roofline"]
print("c5", round(d["value"], 1), d["config"]["serial_step_ms"], d["config"]["serial_phase_ms"], r["kernel"], round(r["total_ms"], 2),
      [(o["kernel"][:10], round(o["total_ms"], 2)) for o in r["other_kernels"]])
PY
HH_C5_STREAMS=1 HH_PCA_DEBUG=2 timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 1 --warmup 0 > $O/c5_dbg2s.log 2>&1 || exit 1
python3 - $O/c5_dbg2s.log <<'PY'
import re, sys, collections
import numpy as np
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    m = re.match(r"\[ortho-ls\] nb=(\d+) pass=(\d) us: proj ([\d.]+) gram\+reduce ([\d.]+) pyth ([\d.]+) mulq ([\d.]+) chol ([\d.]+) apply ([\d.]+)", l)
    if m:
        d[(int(m.group(1)), int(m.group(2)))].append([float(m.group(i)) for i in range(3, 9)])
print("nb pass count  proj gram+reduce pyth mulq chol apply")
for k in sorted(d):
    a = np.median(np.array(d[k]), 0)
    print("%d %d %4d  " % (k[0], k[1], len(d[k])) + " ".join("%.2f" % x for x in a))
PY
