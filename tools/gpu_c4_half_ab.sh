#!/bin/bash
# C4: half-chunk bands forced (FPTA_OPT_INTERP_FUSED 3) vs the automatic choice (whole-chunk bands on C4); PMC of the
# C4 fused kernel at HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh R6w "" c4 "" "INTERP_FUSED=3" || exit 1
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
bash tools/pmc_passes.sh gpurun_out/R6w_pmc_c4 "$P0" "$P1" "$P2" -- python tools/bench_configs.py c4 || exit 1
python tools/pmc_dispatch.py gpurun_out/R6w_pmc_c4 > gpurun_out/R6w_pmc_dispatch_c4.txt 2>&1 || exit 1
echo done
