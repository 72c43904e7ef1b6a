#!/bin/bash
# Per-pulsar interpolation (FPTA_OPT_INTERP_PSR): its bitwise tests, the C3 and gridded suites, then C3 A/B against
# the two-kernel path.   bash tools/gpu_psr.sh <tag>
set -o pipefail
tag=${1:-PSR}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr" > ${o}_psr_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_psr_tests.log | head -20; tail -40 ${o}_psr_tests.log; exit 1; }
tail -1 ${o}_psr_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_grid.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_tests.log | head; tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "INTERP_PSR=0" || exit 1
