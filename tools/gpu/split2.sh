set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/probe_knobs.py --iters 30 "band_concurrent=0,split_tiles=0" "band_concurrent=1,split_tiles=0" "band_concurrent=1,split_tiles=1" "band_concurrent=0,split_tiles=0" "band_concurrent=1,split_tiles=1" > gpurun_out/knobs_split2.log 2>&1
