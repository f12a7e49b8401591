#!/bin/bash
# per-rank C4 shard sweeps of the N = 2 / 4 / 8 partitions (payload, then measured-cost refined), one GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/shards && export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/probe_shards.py 2,4,8 1 > gpurun_out/shards/probe.log 2>&1 || exit 1
grep -E "max|world" gpurun_out/shards/probe.log | grep -E "max" 
