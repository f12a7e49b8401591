#!/bin/bash
# One bench line under several hh_tune settings: tools/gpu/knobs.sh outdir config "k=v,..." "k=v,..." ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; C=$2; shift 2; mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i+1))
  HH_TUNE="$spec" timeout -k 10 300 python3 -u bench.py --config $C --no-cpu > $O/${C}_$i.log 2>&1 || { echo "$spec failed"; tail -3 $O/${C}_$i.log; exit 1; }
  python3 - $O/${C}_$i.log "$spec" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][0])
r = d.get("roofline", {})
print("[%s] %.1f %s sweep %.4f iter %.4f" % (sys.argv[2], d["value"], d["unit"], r.get("sweep_ms_avg") or 0, r.get("iter_ms_avg") or 0))
PY
done
