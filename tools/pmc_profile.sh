#!/bin/bash
# PMC passes over a command (run on the GPU box). Usage: tools/pmc_profile.sh <outdir> -- <cmd...>
# One rocprofv3 run per counter group (no trace domains combined with --pmc).
set -o pipefail
out=$1; shift; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_SMEM GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_THREAD_CYCLES_VALU"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$out/pass$i" -o run -- "$@" > "$out/pass$i.log" 2>&1 || exit $?
  i=$((i+1))
done
