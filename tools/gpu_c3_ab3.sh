#!/bin/bash
set -o pipefail
tag=${1:-PG3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "INTERP_WS=2" "PART_GROUP=16" "INTERP_WS=2 PART_GROUP=16" || exit 1
