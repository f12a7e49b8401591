#!/bin/bash
# k_sweep_all block timeline on C2 (diagnostic): flat-tile threshold
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/sweep_trace.py --config c2 --build flat_max=255 "" > gpurun_out/r2_trace_c2_flat255.log 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/sweep_trace.py --config c2 --build flat_max=128 "" > gpurun_out/r2_trace_c2_flat128.log 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/probe_knobs.py --config c2 --iters 50 --build flat_max=255 "sweep_single=1" "sweep_single=0" > gpurun_out/r2_probe_c2_flat255.log 2>&1 || exit 1
