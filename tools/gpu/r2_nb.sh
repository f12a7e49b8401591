#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for ue in 0 65536 131072; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 --build unit_entries=$ue "sweep_nb=1" "sweep_nb=2" "sweep_nb=4" "sweep_nb=8" "sweep_nb=2,conc_min_bytes=0,split_tiles=0" "sweep_nb=2,conc_min_bytes=0,split_tiles=1" >> gpurun_out/r2_nb_c2.log 2>&1 || exit 1; done
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 20 "sweep_nb=2" "sweep_nb=4" "sweep_nb=2,conc_min_bytes=0" > gpurun_out/r2_nb_c3.log 2>&1 || exit 1
