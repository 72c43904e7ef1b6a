#!/bin/bash
# C3 evidence at HEAD: rocprofv3 kernel statistics of bench.py --config c3, and per-dispatch PMC (one pass per counter
# group) of the C3 kernels (k_grid_interp_psr, k_gen_mix, partial reductions).   bash tools/gpu_r5_c3_evidence.sh <tag>
set -o pipefail
tag=${1:-R5f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_part_final --last 20 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
bash tools/pmc_passes.sh ${o}_pmc_c3 "$P0" "$P1" "$P2" "$P3" "$P4" -- python bench.py --config c3 --steps 1 --warmup 1 --cpu-sample 0 --sub-configs 0 --overlap 0 || { echo "pmc failed"; tail -20 ${o}_pmc_c3/pass*.log; exit 1; }
python tools/pmc_dispatch.py ${o}_pmc_c3 --match interp,gen_mix,part > ${o}_pmc_dispatch_c3.txt 2>&1 || exit 1
head -60 ${o}_pmc_dispatch_c3.txt
