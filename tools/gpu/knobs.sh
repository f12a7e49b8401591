set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/probe_knobs.py "band_concurrent=0,flat_lds_pad=0" "band_concurrent=1,flat_lds_pad=0" \
  "band_concurrent=1,flat_lds_pad=16384" "band_concurrent=1,flat_lds_pad=40960" "band_concurrent=0,flat_lds_pad=16384" \
  > gpurun_out/knobs_flatpad.log 2>&1
