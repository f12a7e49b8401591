#!/bin/bash
# symmetric Cor product (k_cor_sym): C5 tests, A/B bench, kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c5_gpu.py tests/test_structure_gpu.py tests/test_fullsize_gpu.py > $O/c5s_tests.log 2>&1; rc=$?; tail -3 $O/c5s_tests.log; [ $rc = 0 ] || exit 1
for t in "cor_sym=1" "cor_sym=2" "cor_sym=0"; do
HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5s_$t.log 2>&1 || exit 1
echo "$t $(tail -1 $O/c5s_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['config']['serial_step_ms'], d['config']['serial_phase_ms'], [(k['kernel'], round(k['total_ms'],1), k['launches']) for k in [r]+r['other_kernels']])")"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5s -o c5 --output-format csv -- python3 -u $R/bench.py --config c5 --no-cpu --steps 2 --warmup 1 > $O/c5s_prof.log 2>&1 || exit 1
cp $(find /tmp/c5s -name "c5_kernel_stats.csv" | head -1) $O/c5s_kernel_stats.csv
head -12 $O/c5s_kernel_stats.csv | cut -c1-130
