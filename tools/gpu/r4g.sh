#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_uband_gpu.py tests/test_ice_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for spec in "marg_split=0" ""; do
  HH_TUNE="$spec" timeout -k 10 400 python3 -u tools/probe_shards.py 1,8 0 > "$O/shards_$spec.log" 2>&1 || exit 1
  echo "[$spec]"; grep "max " "$O/shards_$spec.log"
done
