set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_structure_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/c5_bench.log 2>&1
