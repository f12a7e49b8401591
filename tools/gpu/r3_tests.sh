#!/bin/bash
# run selected GPU tests: r3_tests.sh <log name> <pytest args...>
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
name=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/r3/$name.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3/$name.log; exit $rc
