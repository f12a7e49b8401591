#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 30 "band_concurrent=1,split_tiles=1" "band_concurrent=0" "band_concurrent=1,split_tiles=0" "band_concurrent=1,split_tiles=1" "band_concurrent=0" > gpurun_out/r2_conc.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 50 "band_concurrent=1,split_tiles=1" "band_concurrent=0" "band_concurrent=1,split_tiles=0" >> gpurun_out/r2_conc.log 2>&1 || exit 1
