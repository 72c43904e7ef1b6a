#!/bin/bash
# Window-ring interpolation (FPTA_OPT_INTERP_WR): bitwise tests, then C2 A/B (on vs off) on one box.
set -o pipefail
tag=${1:-WR1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "window_ring" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c2 "" "INTERP_WR=1" || exit 1
