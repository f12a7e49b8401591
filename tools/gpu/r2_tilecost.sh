#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for tc in 0 2048 8192 32768; do
for k in 7 3; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 --build tile_cost=$tc "band_rows=0" >> gpurun_out/r2_tilecost.log 2>&1 || exit 1; done
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 10 --build tile_cost=$tc "band_rows=0" >> gpurun_out/r2_tilecost.log 2>&1 || exit 1
done
