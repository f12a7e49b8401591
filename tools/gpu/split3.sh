set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_bench_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/split_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/split_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/probe_shards.py 8 1 > gpurun_out/split_shards.log 2>&1
