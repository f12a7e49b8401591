#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_uband_gpu.py -m gpu > $O/x1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/x1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_knobs.py "ub_xcd=0" "ub_xcd=1" "ub_xcd=0,band_concurrent=0" "ub_xcd=1,band_concurrent=0" > $O/x1_c4.log 2>&1; echo "c4 rc=$?"; grep "\[1\]" $O/x1_c4.log
cd /tmp
for x in 0 1; do
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d /tmp/xf$x -o f --output-format csv -- python3 $R/tools/probe_knobs.py --iters 4 "ub_xcd=$x,band_concurrent=0" > $O/x1_pmc$x.log 2>&1 || exit 1
python3 $R/tools/pmc_counters.py $(find /tmp/xf$x -name "*counter_collection.csv" | head -1) $O/x1_fetch$x.json k_sweep_ubands > /dev/null 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$O/x1_fetch$x.json')); print('xcd=$x', {k: v['FETCH_SIZE']['per_dispatch'] for k, v in d.items()})"
done
