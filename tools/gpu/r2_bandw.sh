#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for d in 25 35 45 60; do timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 10 --build band4_density_pct=$d "band_rows=0" >> gpurun_out/r2_bandw.log 2>&1 || exit 1; done
for d in 3 10; do timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 10 --build band8_big_pct=$d "band_rows=0" >> gpurun_out/r2_bandw.log 2>&1 || exit 1; done
