#!/bin/bash
# C5 bench with phase timing + rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && cd gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u ../bench.py --config c5 --steps 5 --warmup 1 --no-cpu > r2_c5_phase.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d r2_c5_prof -o c5 -- python -u ../bench.py --config c5 --steps 3 --warmup 1 --no-cpu > r2_c5_prof.log 2>&1
