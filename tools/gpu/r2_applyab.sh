#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
cp hichap_master_amd/libhichap_hip.so /tmp/lib64.so
for v in 64 128 256 64; do
  if [ $v = 64 ]; then cp /tmp/lib64.so hichap_master_amd/libhichap_hip.so; else cp tools/ab/lib_apply$v.so hichap_master_amd/libhichap_hip.so; fi
  echo "== $v" >> gpurun_out/r2_applyab.log
  timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu 2>&1 | grep '^{' >> gpurun_out/r2_applyab.log || exit 1
done
