#!/bin/bash
# Default build (8192 columns, both triangles) vs the upper-tile variant:
# the variant's parity cases, the C4 line on the default build, the
# per-kernel probe on each build.   tools/gpu/r5e.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 900 $T tests/test_uptiles_variant_gpu.py tests/test_uband_gpu.py tests/test_build_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/c4_bench.log 2>&1 || { tail -20 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-300
timeout -k 10 300 python3 -u tools/probe_upper.py "upper_tiles=0" > $O/probe_default.log 2>&1 || { tail -20 $O/probe_default.log; exit 1; }
HH_LIB=$R/hichap_master_amd/libhichap_hip_up.so timeout -k 10 300 python3 -u tools/probe_upper.py "upper_tiles=0" "upper_tiles=1" > $O/probe_up.log 2>&1 || { tail -20 $O/probe_up.log; exit 1; }
cat $O/probe_default.log $O/probe_up.log
