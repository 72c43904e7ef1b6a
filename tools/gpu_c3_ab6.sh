#!/bin/bash
set -o pipefail
tag=${1:-PSR4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "ASYNC_SUMS=1" "GEN_MIX=3" || exit 1
