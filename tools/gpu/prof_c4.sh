#!/bin/bash
# C4 evidence at the current build: the bench line, rocprofv3 kernel stats of
# the same command (three streams) and of a one-stream sweep (per-kernel
# durations), and the PMC traffic of the sweep kernels (FETCH_SIZE and
# WRITE_SIZE in separate passes, summarised by tools/pmc_summary.py with the
# gfx950 corrections of MI355X_MICROARCH.md).  tools/gpu/prof_c4.sh outdir tag commit
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; TAG=${2:-r4}; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/c4_bench.log 2>&1 || exit 1
RB=$(python3 -c "import json; print(json.loads(open('$O/c4_bench.log').read().strip().splitlines()[-1])['roofline']['real_bytes_per_launch'])")
COMMIT=${3:-unknown}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc4a -o c4 --output-format csv -- python3 -u $R/bench.py --no-cpu > $O/c4_prof3.log 2>&1 || exit 1
cp $(find /tmp/pc4a -name "c4_kernel_stats.csv" | head -1) $O/${TAG}_c4_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc4b -o c4 --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $O/c4_prof1.log 2>&1 || exit 1
cp $(find /tmp/pc4b -name "c4_kernel_stats.csv" | head -1) $O/${TAG}_c4_kernel_stats_1stream.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pc4f -o f --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/c4_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pc4w -o w --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/c4_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pc4f -name "*counter_collection.csv" | head -1) $(find /tmp/pc4w -name "*counter_collection.csv" | head -1) $O/${TAG}_c4_pmc.json "$COMMIT" $RB c4 $O/c4_bench.log > $O/c4_pmc_summary.log 2>&1 || exit 1
head -12 $O/c4_pmc_summary.log | cut -c1-200
