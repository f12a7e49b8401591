set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/spprof -o c4 --output-format csv -- python3 bench.py --no-cpu > gpurun_out/span_bench.log 2>&1 && \
python3 tools/sweep_span.py $(find /tmp/spprof -name "c4_kernel_trace.csv" | head -1) gpurun_out/r1v8_c4_sweep_span.json > gpurun_out/span.log 2>&1 && \
cp $(find /tmp/spprof -name "c4_kernel_stats.csv" | head -1) gpurun_out/span_c4_kernel_stats.csv
