#!/bin/bash
# Round-2 (session b) measurements of the committed build ($1 = commit): C4 PMC first
# (written into profiles/ on the box so the C4 bench line reads this build's traffic),
# C4 bench + rocprof kernel stats / sweep span / one-stream breakdown, then every config.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/final && export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/final
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o f --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/r2b_pmc_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o w --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/r2b_pmc_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) profiles/r2b_c4_pmc.json "$C" 15202483080 > $O/r2b_pmc_summary.log 2>&1 || exit 1
cp profiles/r2b_c4_pmc.json $O/r2b_c4_pmc.json
echo "pmc ok"
timeout -k 10 300 python3 -u bench.py > $O/r2b_c4_bench.log 2>&1 || exit 1
echo "c4 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k4 -o c4 -- python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $O/r2b_c4_prof.log 2>&1 || exit 1
cp $(find /tmp/k4 -name "*kernel_stats.csv" | head -1) $O/r2b_c4_kernel_stats.csv
python3 tools/sweep_span.py $(find /tmp/k4 -name "*kernel_trace.csv" | head -1) $O/r2b_c4_sweep_span.json >> $O/r2b_c4_prof.log 2>&1 || exit 1
HH_TUNE=conc_min_bytes=1000000000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k41 -o c41 -- python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $O/r2b_c4_prof_1stream.log 2>&1 || exit 1
cp $(find /tmp/k41 -name "*kernel_stats.csv" | head -1) $O/r2b_c4_kernel_stats_1stream.csv
echo "c4 prof ok"
timeout -k 10 300 python3 -u bench.py --config c2 --steps 200 --warmup 10 > $O/r2b_c2_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k2 -o c2 -- python3 -u bench.py --config c2 --no-cpu --steps 20 --warmup 2 > $O/r2b_c2_prof.log 2>&1 || exit 1
cp $(find /tmp/k2 -name "*kernel_stats.csv" | head -1) $O/r2b_c2_kernel_stats.csv
timeout -k 10 300 python3 -u bench.py --config c3 --steps 100 --warmup 5 > $O/r2b_c3_bench.log 2>&1 || exit 1
echo "c2 c3 ok"
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/r2b_c5_bench.log 2>&1 || exit 1
HH_C5_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k5 -o c5 -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $O/r2b_c5_prof.log 2>&1 || exit 1
cp $(find /tmp/k5 -name "*kernel_stats.csv" | head -1) $O/r2b_c5_kernel_stats.csv
echo "c5 ok"
timeout -k 10 300 python3 -u bench.py --config dropin --steps 5 --warmup 1 > $O/r2b_dropin_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config e2e --steps 5 --warmup 1 > $O/r2b_e2e_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config gw --steps 3 --warmup 1 > $O/r2b_gw_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config pairs --steps 5 --warmup 1 > $O/r2b_pairs_bench.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --config loops --steps 3 --warmup 1 > $O/r2b_loops_bench.log 2>&1 || exit 1
echo "all ok"
