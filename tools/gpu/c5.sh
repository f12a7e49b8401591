set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_structure_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/c5_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o c5 --output-format csv -- python3 bench.py --config c5 --no-cpu > gpurun_out/c5_prof.log 2>&1 && \
cp $(find /tmp/c5prof -name "c5_kernel_stats.csv" | head -1) gpurun_out/c5_kernel_stats.csv
