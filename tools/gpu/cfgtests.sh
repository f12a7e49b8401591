set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ice_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c1_config or config_size" > gpurun_out/cfg_tests.log 2>&1
