set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/finalprof -o c4 --output-format csv -- python3 bench.py --no-cpu > gpurun_out/final_prof.log 2>&1 && \
cp $(find /tmp/finalprof -name "c4_kernel_stats.csv" | head -1) gpurun_out/final_c4_kernel_stats.csv
