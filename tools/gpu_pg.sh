#!/bin/bash
# Partial-checksum groups (FPTA_OPT_PART_GROUP): the checksum / interpolation tests, the diagnostic-kernel tests on the
# variant build, then C3 A/B of group sizes against the previous HEAD's library.
#   bash tools/gpu_pg.sh <tag>
set -o pipefail
tag=${1:-PG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_grid.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_tests.log | head; tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
FAKEPTA_AMD_LIB=build/diag/lib_diag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "storer or union or interpolation_is_bitwise or partial_realization or lds" > ${o}_diag_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_diag_tests.log | head; tail -30 ${o}_diag_tests.log; exit 1; }
tail -1 ${o}_diag_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "PART_GROUP=4" "LIB=build/diag/lib_head.so" || exit 1
