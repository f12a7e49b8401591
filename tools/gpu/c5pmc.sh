set -o pipefail
mkdir -p gpurun_out /tmp/c5pmc
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES -d /tmp/c5pmc -o c5 --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu > gpurun_out/c5pmc.log 2>&1 && \
python3 tools/pmc_counters.py $(find /tmp/c5pmc -name "*counter_collection.csv" | head -1) gpurun_out/c5_mfma_pmc.json k_syrk k_cor_mul > gpurun_out/c5pmc_summary.log 2>&1
