#!/bin/bash
set -o pipefail
tag=${1:-PG4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "LIB=build/diag/lib_pwpc1.so" "PART_GROUP=16" "LIB=build/diag/lib_pwpc1.so PART_GROUP=16" || exit 1
