#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for k in 0 3 7; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 20 "sweep_single=0" "sweep_single=1" >> gpurun_out/r2_single_shard.log 2>&1 || exit 1; done
for ue in 8192 16384 65536; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 --build unit_entries=$ue "sweep_single=1" >> gpurun_out/r2_single_c2u.log 2>&1 || exit 1; done
