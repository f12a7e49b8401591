set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r1v8_distgpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --no-cpu > gpurun_out/r1v8_c3_prof.log 2>&1
