#!/bin/bash
# fused / 64-row band launches: C2 and C4 sweep times under the knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 "band_fused=0,band_rows=256" "band_fused=1,band_rows=256" "band_fused=1,band_rows=64" "band_fused=0,band_rows=64" "band_fused=1,band_rows=64,conc_min_bytes=0" "band_fused=1,band_rows=64,conc_min_bytes=0,split_tiles=0" > gpurun_out/r2_band_c2.log 2>&1 || exit 1
for ue in 8192 16384; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 50 --build unit_entries=$ue "band_fused=1,band_rows=64" "band_fused=1,band_rows=64,conc_min_bytes=0" >> gpurun_out/r2_band_c2.log 2>&1 || exit 1; done
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 10 "band_fused=0,band_rows=256" "band_fused=1,band_rows=256" "band_fused=1,band_rows=64" > gpurun_out/r2_band_c4.log 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ice_gpu.py > gpurun_out/r2_band_tests.log 2>&1
