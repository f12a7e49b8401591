#!/bin/bash
# C4 at bb68f5f: bench line, rocprof kernel stats (three streams), PMC traffic
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/p2_c4_bench.log 2>&1 || exit 1
tail -1 $O/p2_c4_bench.log | cut -c1-200
RB=$(python3 -c "import json,sys; print(json.loads(open('$O/p2_c4_bench.log').read().strip().splitlines()[-1])['roofline']['real_bytes_per_launch'])")
echo "real bytes $RB"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p2a -o c4 --output-format csv -- python3 -u $R/bench.py --no-cpu > $O/p2_prof3.log 2>&1 || exit 1
cp $(find /tmp/p2a -name "c4_kernel_stats.csv" | head -1) $O/p2_c4_kernel_stats.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf2 -o f --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p2_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw2 -o w --output-format csv -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/p2_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pf2 -name "*counter_collection.csv" | head -1) $(find /tmp/pw2 -name "*counter_collection.csv" | head -1) $O/r3c_c4_pmc.json "bb68f5f" $RB > $O/p2_pmc_summary.log 2>&1 || exit 1
cat $O/p2_pmc_summary.log | cut -c1-200
cd $R && timeout -k 10 300 python3 -u bench.py > $O/p2_c4_bench_pmc.log 2>&1 || exit 1
tail -1 $O/p2_c4_bench_pmc.log | cut -c1-200
