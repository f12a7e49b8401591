#!/bin/bash
# C5 at HEAD: bench line + rocprof kernel stats (2 timed steps + 1 warmup + 2 serial passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5p -o c5 --output-format csv -- python3 -u $R/bench.py --config c5 --no-cpu --steps 2 --warmup 1 > $O/c5p_prof.log 2>&1 || exit 1
cp $(find /tmp/c5p -name "c5_kernel_stats.csv" | head -1) $O/c5p_kernel_stats.csv
head -30 $O/c5p_kernel_stats.csv | cut -c1-160
tail -1 $O/c5p_prof.log | cut -c1-300
