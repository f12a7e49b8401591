#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
for fc in -1 0 1; do
timeout -k 10 200 python -u tools/probe_knobs.py --config c3 --iters 40 --build flat_cols=$fc "uband=1" "uband=0" > $O/m5_c3_fc$fc.log 2>&1; echo "c3 fc=$fc rc=$?"; grep "\[1\]" $O/m5_c3_fc$fc.log
done
timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu > $O/m5_c3_bench.log 2>&1; echo "c3 rc=$?"; tail -1 $O/m5_c3_bench.log | cut -c1-150
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/m5 -o c3 --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --config c3 --iters 40 "uband=1" > $GRAFT_REPO_ROOT/$O/m5_prof.log 2>&1; echo "prof rc=$?"
cp $(find /tmp/m5 -name "c3_kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/$O/m5_c3_kernel_stats.csv; head -8 $GRAFT_REPO_ROOT/$O/m5_c3_kernel_stats.csv | cut -c1-130
