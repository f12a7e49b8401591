set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ice_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/ice_c4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --no-cpu > gpurun_out/ice_c3.log 2>&1 && \
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_marg -o c3 --output-format csv -- python3 bench.py --config c3 --no-cpu --steps 10 > gpurun_out/ice_c3_prof.log 2>&1
