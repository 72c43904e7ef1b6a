#!/bin/bash
# Counters of the gridded interpolation kernels on C2 (tools/pmc_passes.sh + pmc_summary.py).
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_passes.sh gpurun_out/pmc_sparse \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_IFETCH" \
  "FETCH_SIZE" "WRITE_SIZE" \
  -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 "$@" || exit 1
python tools/pmc_summary.py gpurun_out/pmc_sparse --match interp > gpurun_out/pmc_sparse.txt 2>&1 || exit 1
cat gpurun_out/pmc_sparse.txt
