set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gate_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --steps 200 > gpurun_out/r1v8_c2_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r1v8_c3_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/gate_c4_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/probe_shards.py 8 1 > gpurun_out/gate_shards.log 2>&1
