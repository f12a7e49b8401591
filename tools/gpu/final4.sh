set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/final4_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final4_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/final4_bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/f4prof -o c4 --output-format csv -- python3 bench.py --no-cpu > gpurun_out/final4_prof.log 2>&1 && \
cp $(find /tmp/f4prof -name "c4_kernel_stats.csv" | head -1) gpurun_out/final4_c4_kernel_stats.csv
