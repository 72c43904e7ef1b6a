#!/bin/bash
set -o pipefail
tag=${1:-WRP}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
bash tools/pmc_passes.sh ${o}_pmc "$P0" "$P1" "$P2" "$P3" "$P4" -- python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0 --sub-configs 0 --opt INTERP_WR=1 || { echo "pmc failed"; tail -20 ${o}_pmc/pass*.log; exit 1; }
python tools/pmc_dispatch.py ${o}_pmc --match interp > ${o}_pmc_dispatch.txt 2>&1 || exit 1
cat ${o}_pmc_dispatch.txt
