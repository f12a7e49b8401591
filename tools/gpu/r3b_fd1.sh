#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ice_gpu.py tests/test_uband_gpu.py tests/test_build_gpu.py -m gpu > $O/fd1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/fd1_tests.log; grep -m3 "FAILED" $O/fd1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_knobs.py "band_concurrent=1" "band_concurrent=0" > $O/fd1_c4.log 2>&1; echo "c4 rc=$?"; grep "\[1\]" $O/fd1_c4.log
timeout -k 10 300 python -u tools/probe_knobs.py --shard 0/8 "band_concurrent=0" > $O/fd1_sh0.log 2>&1; echo "sh0 rc=$?"; grep "\[1\]" $O/fd1_sh0.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fd1 -o c4 --output-format csv -- python3 -u $R/tools/probe_knobs.py --iters 20 "band_concurrent=0" > $O/fd1_prof.log 2>&1; echo "prof rc=$?"
python3 - <<PY
import csv, glob
f = glob.glob('/tmp/fd1/**/c4_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'synth' in r['Name'] or 'rocclr' in r['Name']: continue
    print(f"   {r['Name'][:40]:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1000:8.1f} us")
PY
