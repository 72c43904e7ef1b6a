#!/bin/bash
# Kernel counters of the gridded path (k_grid_interp_mfma, k_grid_dft_mfma) on a short C2 bench: issue /
# wait / MFMA-busy / address-unit passes and the HBM FETCH_SIZE / WRITE_SIZE passes, one rocprofv3 run each.
#   bash tools/gpu_pmc_interp.sh <tag>   -> gpurun_out/pmc_<tag>/ and gpurun_out/pmc_<tag>.txt
set -o pipefail
tag=${1:-interp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmc_$tag
mkdir -p $out
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR TA_TA_BUSY TD_TD_BUSY GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES GRBM_GUI_ACTIVE"
i=0
for p in "$P0" "$P1" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $out/pass$i -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 > $out/pass$i.log 2>&1 || exit 1
  i=$((i+1))
done
python tools/pmc_summary.py $out --match grid > gpurun_out/pmc_$tag.txt 2>&1 || exit 1
cat gpurun_out/pmc_$tag.txt
