#!/bin/bash
# round 2: C5 trace, bench sweep over the Krylov cycle length, rocprof summary
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pca_trace.py 21 1 --p 8 > gpurun_out/pca_trace.log 2>&1 || exit 1
for p in 6 8; do
  HH_PCA_P=$p timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu >> gpurun_out/r2_c5_bench.log 2>&1 || exit 1
done
cd gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r2prof -o c5 -- python -u ../bench.py --config c5 --steps 3 --warmup 1 --no-cpu > r2_c5_prof.log 2>&1 || exit 1
python ../tools/kstats_db.py /tmp/r2prof/c5_results.db r2_c5_kernel_stats.csv
