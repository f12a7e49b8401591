cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_c5_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1 0 1; do
  HH_ORTHO_BAR=$v timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu > $O/c5_bar$v.log 2>&1 || { tail -5 $O/c5_bar$v.log; exit 1; }
  python3 - $O/c5_bar$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print("bar", sys.argv[2], round(d["value"], 2), "chrom/s", "k_ortho", round(r.get("total_ms", 0), 2), "ms", r.get("launches"))
PY
done
