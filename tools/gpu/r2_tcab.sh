#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for tc in 0 32768 0 32768 8192; do timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 20 --build tile_cost=$tc "band_rows=0" >> gpurun_out/r2_tcab.log 2>&1 || exit 1; done
for tc in 0 8192 32768; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard 7/8 --iters 30 --build tile_cost=$tc "band_rows=0" >> gpurun_out/r2_tcab.log 2>&1 || exit 1; done
