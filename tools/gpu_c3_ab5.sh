#!/bin/bash
set -o pipefail
tag=${1:-PG5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "LIB=build/diag/lib_pwg14.so" "LIB=build/diag/lib_pwg12.so" || exit 1
