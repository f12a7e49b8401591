set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r1v8_c3_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --steps 200 > gpurun_out/r1v8_c2_bench.log 2>&1
