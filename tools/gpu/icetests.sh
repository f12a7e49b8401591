set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ice_tests.log 2>&1
