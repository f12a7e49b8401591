#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for k in 3 7; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 "band_rows=256" "band_rows=128" "band_rows=64" "band_rows=256,band_concurrent=0,sweep_single=0" "band_rows=256,split_tiles=0" "sweep_single=1" >> gpurun_out/r2_shard2.log 2>&1 || exit 1; done
