#!/bin/bash
set -o pipefail
tag=${1:-PSR7}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr or c4 or pipelined" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c4 "" "INTERP_PSR=0" || exit 1
