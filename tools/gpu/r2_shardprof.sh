#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for k in 3 7; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sp$k -o s -- python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 "band_concurrent=0,sweep_single=0" > gpurun_out/r2_shardprof_$k.log 2>&1 || exit 1
cp $(find /tmp/sp$k -name "*kernel_stats.csv" | head -1) gpurun_out/r2_shard${k}of8_kernel_stats.csv
done
