#!/bin/bash
set -o pipefail
tag=${1:-C5A}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c5 "" "LIB=build/diag/lib_rw4w3.so" "LIB=build/diag/lib_rw4w2.so" || exit 1
