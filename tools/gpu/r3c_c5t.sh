#!/bin/bash
# symmetric Cor product: the C5 / structure / fullsize GPU tests + bench line at the build
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_c5_gpu.py tests/test_structure_gpu.py tests/test_fullsize_gpu.py > $O/c5t_tests.log 2>&1; rc=$?; tail -3 $O/c5t_tests.log; grep -i "upper_triangle" $O/c5t_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5t_bench.log 2>&1 || exit 1
tail -1 $O/c5t_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['config']['serial_step_ms'], [(k['kernel'], round(k['total_ms'],1), k['launches'], round(k['frac'],3)) for k in [r]+r['other_kernels']])"
