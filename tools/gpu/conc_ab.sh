#!/bin/bash
# three-stream sweep at shard / C3 sizes: probe shards at N = 2, 4, 8 and the
# C3 line with and without conc_min_bytes=0
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for spec in "conc_min_bytes=0" "conc_min_bytes=0,split_tiles=0" ""; do
  HH_TUNE="$spec" timeout -k 10 400 python3 -u tools/probe_shards.py 2,4,8 0 > "$O/shards_${spec//[=,]/_}.log" 2>&1 || exit 1
  echo "[$spec]"; grep "max " "$O/shards_${spec//[=,]/_}.log"
done
for spec in "conc_min_bytes=0" "" "conc_min_bytes=0" ""; do
  HH_TUNE="$spec" timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu > $O/c3.log 2>&1 || exit 1
  echo "c3 [$spec] $(tail -1 $O/c3.log | cut -c1-120)"
done
