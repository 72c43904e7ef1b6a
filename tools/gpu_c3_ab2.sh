#!/bin/bash
set -o pipefail
tag=${1:-PG2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_c3_trace.sh || exit 1
python tools/trace_steps.py gpurun_out/C3T_prof/run_kernel_trace.csv --marker k_part_final --last 20 > gpurun_out/${tag}_c3_trace.txt || exit 1
cat gpurun_out/${tag}_c3_trace.txt
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "ASYNC_SUMS=1" "PART_GROUP=16" "PART_GROUP=8" || exit 1
