#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py -m gpu -k "flat or sharded or full_size or config" > $O/fr1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/fr1_tests.log; grep -m3 "FAILED" $O/fr1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_knobs.py "band_concurrent=1" "band_concurrent=0" > $O/fr1_c4.log 2>&1; echo "c4 rc=$?"; grep "\[1\]" $O/fr1_c4.log
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d /tmp/ff -o f --output-format csv -- python3 $R/tools/probe_knobs.py --iters 4 "band_concurrent=0" > $O/fr1_pmc.log 2>&1 || exit 1
python3 $R/tools/pmc_counters.py $(find /tmp/ff -name "*counter_collection.csv" | head -1) $O/fr1_fetch.json k_sweep > /dev/null 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$O/fr1_fetch.json')); print({k[:24]: round(v['FETCH_SIZE']['per_dispatch']*1024/1e9,3) for k, v in d.items()})"
