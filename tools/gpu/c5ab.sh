cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r4d
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c5_gpu.py -k "not selected_pc" > gpurun_out/r4d/c5tests.log 2>&1 || { tail -30 gpurun_out/r4d/c5tests.log; exit 1; }
tail -3 gpurun_out/r4d/c5tests.log
for ls in 0 1 0 1; do
HH_TUNE=ortho_lowsync=$ls timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/r4d/c5_ls$ls.log 2>&1 || exit 1
echo "ls=$ls $(tail -1 gpurun_out/r4d/c5_ls$ls.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value'],1), d['config']['serial_step_ms'], d['config']['serial_phase_ms'], [(k['kernel'][:8], round(k['total_ms'],1)) for k in [r]+r['other_kernels']], d['config']['pca_products_per_chrom'][1])")"
done
