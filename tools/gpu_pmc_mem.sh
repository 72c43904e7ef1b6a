#!/bin/bash
# Memory-pipeline PMC passes over a short bench (gridded path), MFMA and VALU interpolation.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_mem
A="TCC_HIT TCC_MISS TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TCC_WRITE_REQ_LATENCY TA_TA_BUSY TD_TD_BUSY SQ_LEVEL_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_TAG_STALL TCC_BUSY TCC_EA0_WRREQ_LEVEL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES GRBM_GUI_ACTIVE"
for m in 3 1; do
  i=0
  for p in "$A" "$B"; do
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d gpurun_out/pmc_mem/m$m/pass$i -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --grid-mfma $m > gpurun_out/pmc_mem/m$m.pass$i.log 2>&1 || exit 1
    i=$((i+1))
  done
  python tools/pmc_summary.py gpurun_out/pmc_mem/m$m --match grid_interp > gpurun_out/pmc_mem/m$m.txt 2>&1 || exit 1
  echo "== mask $m"; cat gpurun_out/pmc_mem/m$m.txt
done
