#!/bin/bash
# C5 MFMA counters for split-K k_syrk / k_cor_mul_part / k_ortho at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c /tmp/c5pmc && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES -d /tmp/c5pmc -o c5 --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu > $R/gpurun_out/r3c/c5pmc.log 2>&1 || exit 1
python3 $R/tools/pmc_counters.py $(find /tmp/c5pmc -name "*counter_collection.csv" | head -1) $R/gpurun_out/r3c/r3c_c5_mfma_pmc.json k_syrk k_cor_mul k_ortho > $R/gpurun_out/r3c/c5pmc_summary.log 2>&1 || exit 1
cat $R/gpurun_out/r3c/c5pmc_summary.log | cut -c1-300
