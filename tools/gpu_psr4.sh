#!/bin/bash
set -o pipefail
tag=${1:-PSR6}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "GEN_MIX=1" "LIB=build/diag/lib_nokeep.so" "LIB=build/diag/lib_nokeep.so GEN_MIX=1" "LIB=build/diag/lib_head.so" || exit 1
