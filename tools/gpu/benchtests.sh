set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/bench_tests.log 2>&1
