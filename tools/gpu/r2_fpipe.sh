#!/bin/bash
# flat-unit tile pipeline A/B (one stream and default launch shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/fp && cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
C="conc_min_bytes=1099511627776"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/fp/prof" -o c4fp -- python3 -u "$R/tools/probe_knobs.py" --iters 10 "$C,flat_pipe=0" "$C,flat_pipe=1" "$C,flat_pipe=2" "flat_pipe=0" "flat_pipe=1" "flat_pipe=2" > "$R/gpurun_out/fp/c4fp.log" 2>&1 || exit 1
find "$R/gpurun_out/fp/prof" -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/fp/c4fp_kernel_stats.csv" \;
find "$R/gpurun_out/fp/prof" -name "*kernel_trace.csv" -delete
timeout -k 10 200 python3 -u "$R/tools/probe_knobs.py" --config c3 --iters 20 "flat_pipe=0" "flat_pipe=1" "flat_pipe=2" > "$R/gpurun_out/fp/c3fp.log" 2>&1 || exit 1
