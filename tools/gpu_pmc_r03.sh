#!/bin/bash
# PMC of every shipped config kernel with the kernels serialised (one stream), so each dispatch's counters are its own:
# C2 (k_grid_dft_gen, k_gen_mix, k_grid_interp_ws), C3 (k_grid_dft_mfma, fused-checksum interpolation), C5 (white
# epilogue interpolation, k_epoch_normals).
#   bash tools/gpu_pmc_r03.sh <tag>
set -o pipefail
tag=${1:-r03c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
run() {  # <name> <cmd...>
  local name=$1; shift
  bash tools/pmc_passes.sh gpurun_out/${tag}_$name "$P0" "$P1" "$P2" "$P3" "$P4" -- "$@" || { echo "pmc $name failed"; tail -20 gpurun_out/${tag}_$name/pass*.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/${tag}_$name > gpurun_out/${tag}_$name.txt 2>&1 || exit 1
}
run c2 python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0
run c3 python bench.py --config c3 --steps 1 --warmup 0 --cpu-sample 0 --overlap 0 --c3-real 20000
run c5 python tools/bench_configs.py c5
grep -E "^==|duration|MFMA_BUSY|wait_inst|valu_busy|hbm_|TCC_HIT|TCC_MISS|LDS_BANK" gpurun_out/${tag}_c2.txt
