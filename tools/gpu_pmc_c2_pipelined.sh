#!/bin/bash
# Per-dispatch PMC of the shipped C2 step (pipelined blocks: the next block's mix inside k_grid_fused, no co-running
# kernel), as tools/gpu_evidence6.sh's passes.   bash tools/gpu_pmc_c2_pipelined.sh <tag>
set -o pipefail
tag=${1:-R6q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
bash tools/pmc_passes.sh ${o}_pmc_c2p "$P0" "$P1" "$P2" -- python bench.py --steps 6 --warmup 3 --cpu-sample 0 --exact-launches 0 --sub-configs 0 || exit 1
python tools/pmc_dispatch.py ${o}_pmc_c2p > ${o}_pmc_dispatch_c2p.txt 2>&1 || exit 1
echo done
