#!/bin/bash
# C4 per-kernel ablations on one stream (timing diagnostics): 0 full, 1 no LDS gathers / stream only, 2 no bias staging
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/abl && cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/abl/prof" -o c4abl -- python3 -u "$R/tools/probe_knobs.py" --iters 10 "conc_min_bytes=1099511627776,sweep_ablate=0" "conc_min_bytes=1099511627776,sweep_ablate=1" "conc_min_bytes=1099511627776,sweep_ablate=2" > "$R/gpurun_out/abl/c4abl.log" 2>&1 || exit 1
find "$R/gpurun_out/abl/prof" -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/abl/c4abl_kernel_stats.csv" \;
find "$R/gpurun_out/abl/prof" -name "*kernel_trace.csv" -delete
