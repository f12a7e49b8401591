#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ice_gpu.py > gpurun_out/r2_single_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 "sweep_single=1" "sweep_single=0" "sweep_single=0,conc_min_bytes=0,split_tiles=0" "sweep_single=1" > gpurun_out/r2_single_c2.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 20 "sweep_single=1" "sweep_single=0,conc_min_bytes=0" "sweep_single=0,conc_min_bytes=0,split_tiles=0" > gpurun_out/r2_single_c3.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 10 "sweep_single=0" "sweep_single=1" > gpurun_out/r2_single_c4.log 2>&1 || exit 1
