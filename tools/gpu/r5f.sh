#!/bin/bash
# cis / c2 sweep knobs, the batched TwoStep tests.   tools/gpu/r5f.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_twostep_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/probe_knobs.py --config cis --iters 20 "uband=0" "uband=0,conc_min_bytes=0" "uband=2" "uband=2,conc_min_bytes=0,conc_ub_min_bytes=0" > $O/cis_knobs.log 2>&1 || { tail -20 $O/cis_knobs.log; exit 1; }
cat $O/cis_knobs.log
timeout -k 10 300 python3 -u tools/probe_knobs.py --config c2 --iters 50 "uband=0" "uband=0,sweep_single=0" "uband=0,sweep_single=0,conc_min_bytes=0" > $O/c2_knobs.log 2>&1 || { tail -20 $O/c2_knobs.log; exit 1; }
cat $O/c2_knobs.log
timeout -k 10 400 python3 -u bench.py --config twostep_genome --steps 10 --warmup 2 > $O/twostep_genome.log 2>&1 || { tail -20 $O/twostep_genome.log; exit 1; }
grep '^{"metric"' $O/twostep_genome.log | cut -c1-900
