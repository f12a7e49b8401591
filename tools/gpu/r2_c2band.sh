#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for d in 25 15 10 6; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 100 --build band4_density_pct=$d "sweep_single=-1" >> gpurun_out/r2_c2band.log 2>&1 || exit 1; done
for w in 4096 6144 8192; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 100 --build band4_density_pct=2,band_w=$w "sweep_single=-1" >> gpurun_out/r2_c2band.log 2>&1 || exit 1; done
