#!/bin/bash
# C4 at the current build: bench line, rocprof kernel stats (three streams, one stream), PMC traffic
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3d && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3d
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/p2_c4_bench.log 2>&1 || exit 1
tail -1 $O/p2_c4_bench.log | cut -c1-200
RB=$(python3 -c "import json,sys; print(json.loads(open('$O/p2_c4_bench.log').read().strip().splitlines()[-1])['roofline']['real_bytes_per_launch'])")
echo "real bytes $RB"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p3a -o c4 --output-format csv -- python3 -u $R/bench.py --no-cpu > $O/p2_prof3.log 2>&1 || exit 1
cp $(find /tmp/p3a -name "c4_kernel_stats.csv" | head -1) $O/p2_c4_kernel_stats.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf3 -o f --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p2_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw3 -o w --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p2_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pf3 -name "*counter_collection.csv" | head -1) $(find /tmp/pw3 -name "*counter_collection.csv" | head -1) $O/r3d_c4_pmc.json "118f991" $RB > $O/p2_pmc_summary.log 2>&1 || exit 1
cat $O/p2_pmc_summary.log | cut -c1-200
cd $R && timeout -k 10 300 python3 -u bench.py > $O/p2_c4_bench_pmc.log 2>&1 || exit 1
tail -1 $O/p2_c4_bench_pmc.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p3b -o c4 --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $O/p3_prof1.log 2>&1 || exit 1
cp $(find /tmp/p3b -name "c4_kernel_stats.csv" | head -1) $O/p3_c4_kernel_stats_1stream.csv
head -8 $O/p3_c4_kernel_stats_1stream.csv | cut -c1-150
