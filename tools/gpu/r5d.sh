#!/bin/bash
# Upper-triangle tiles, measured: per-kernel probe (both triangles vs upper
# tiles), the C4 bench line, and the N = 8 / 4 shard sweep times.
#   tools/gpu/r5d.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_upper.py "upper_tiles=0" "upper_tiles=-1" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/c4_bench.log 2>&1 || { tail -20 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-700
timeout -k 10 400 python3 -u tools/probe_shards.py 8,4 > $O/shards.log 2>&1 || { tail -20 $O/shards.log; exit 1; }
grep "max" $O/shards.log
