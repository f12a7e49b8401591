set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/final5_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final5_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/final5_bench.log 2>&1
