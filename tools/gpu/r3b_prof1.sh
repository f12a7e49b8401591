#!/bin/bash
# C4 at HEAD (55c2050): bench line, rocprof kernel stats (three streams + one stream), PMC traffic, flat-kernel SQ counters
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/p1_c4_bench.log 2>&1 || exit 1
tail -1 $O/p1_c4_bench.log | cut -c1-200
RB=$(python3 -c "import json,sys; print(json.loads(open('$O/p1_c4_bench.log').read().strip().splitlines()[-1])['roofline']['real_bytes_per_launch'])")
echo "real bytes $RB"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p1a -o c4 --output-format csv -- python3 -u $R/bench.py --no-cpu > $O/p1_prof3.log 2>&1 || exit 1
cp $(find /tmp/p1a -name "c4_kernel_stats.csv" | head -1) $O/p1_c4_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p1b -o c4 --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $O/p1_prof1.log 2>&1 || exit 1
cp $(find /tmp/p1b -name "c4_kernel_stats.csv" | head -1) $O/p1_c4_kernel_stats_1stream.csv
head -8 $O/p1_c4_kernel_stats_1stream.csv | cut -c1-150
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o f --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p1_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o w --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p1_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) $O/r3b_c4_pmc.json "55c2050" $RB > $O/p1_pmc_summary.log 2>&1 || exit 1
cat $O/p1_pmc_summary.log | cut -c1-200
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES -d /tmp/ps -o s --output-format csv -- python3 $R/tools/probe_knobs.py --iters 4 "band_concurrent=0" > $O/p1_pmc_sq.log 2>&1 || exit 1
python3 $R/tools/pmc_counters.py $(find /tmp/ps -name "*counter_collection.csv" | head -1) $O/p1_sq.json k_sweep_flatw k_sweep_ubands k_sweep_tiled > /dev/null 2>&1 || exit 1
echo sq ok
