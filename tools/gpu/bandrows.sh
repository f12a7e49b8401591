set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ice_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "band" > gpurun_out/bandrows_tests.log 2>&1 && \
HH_TUNE=band_rows=256 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_br256.log 2>&1 && \
HH_TUNE=band_rows=128 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_br128.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_knobs.py "band_rows=256" "band_rows=128" > gpurun_out/knobs_br.log 2>&1
