#!/bin/bash
# Round-2 profiles of the current build: C4 kernel stats, C4 PMC (FETCH / WRITE
# in separate passes), C2 bench + kernel stats.  $1 = commit of the build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out /tmp/pf /tmp/pw && export TMPDIR=/tmp
C=${1:-unknown}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c4k -o c4 -- python3 -u bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r2_c4_prof.log 2>&1 || exit 1
cp $(find /tmp/c4k -name "*kernel_stats.csv" | head -1) gpurun_out/r2_c4_kernel_stats.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o f --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r2_pmc_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o w --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r2_pmc_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) gpurun_out/r2_c4_pmc.json "$C" 15202483080 > gpurun_out/r2_pmc_summary.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu > gpurun_out/r2_c2_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c2k -o c2 -- python3 -u bench.py --config c2 --no-cpu --steps 20 --warmup 2 > gpurun_out/r2_c2_prof.log 2>&1 || exit 1
cp $(find /tmp/c2k -name "*kernel_stats.csv" | head -1) gpurun_out/r2_c2_kernel_stats.csv
