#!/bin/bash
# Round-2 final, part 2 (after the C4 PMC of the same build was committed)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/final && export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 300 python3 -u bench.py > $O/r2_c4_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/r2_c5_bench.log 2>&1 || exit 1
HH_C5_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k5 -o c5 -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $O/r2_c5_prof.log 2>&1 || exit 1
cp $(find /tmp/k5 -name "*kernel_stats.csv" | head -1) $O/r2_c5_kernel_stats.csv
timeout -k 10 300 python3 -u bench.py --config dropin --steps 3 --warmup 1 > $O/r2_dropin_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config e2e --steps 3 --warmup 1 > $O/r2_e2e_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config gw --steps 3 --warmup 1 > $O/r2_gw_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config pairs --steps 5 --warmup 1 > $O/r2_pairs_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config loops --steps 3 --warmup 1 > $O/r2_loops_bench.log 2>&1 || exit 1
