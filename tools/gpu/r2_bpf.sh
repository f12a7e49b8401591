#!/bin/bash
# single-launch sweep block order: bitwise tests + C2 trace / timing
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/bpf
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ice_gpu.py -k "launch_shapes or closed or saturated" > gpurun_out/bpf/tests.log 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/sweep_trace.py --config c2 "" > gpurun_out/bpf/trace_c2.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 "sweep_single=1" "sweep_single=0" > gpurun_out/bpf/probe_c2.log 2>&1 || exit 1
