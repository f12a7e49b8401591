#!/bin/bash
# XCD dealing of the unit launch lists (bit 1 tiled, bit 2 flat): C4 per-kernel time on one stream
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/xcd && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for d in 0 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kx$d -o k -- python3 -u "$R/tools/probe_knobs.py" --iters 10 --build xcd_deal=$d "conc_min_bytes=1099511627776" "band_rows=0" > gpurun_out/xcd/probe2_d$d.log 2>&1 || exit 1
  cp $(find /tmp/kx$d -name "*kernel_stats.csv" | head -1) gpurun_out/xcd/stats_d$d.csv
done
