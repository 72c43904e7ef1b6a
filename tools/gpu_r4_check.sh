#!/bin/bash
# Round-4 validation in one GPU call: the full GPU suite on the product library, the diagnostic-kernel tests on the
# variant build (make variant NAME=diag DEFS=-DFPTA_DIAG_KERNELS), smoke, and the default bench.py line.
#   bash tools/gpu_r4_check.sh <tag>
set -o pipefail
tag=${1:-R4t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_gpu_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_gpu_tests.log | head; tail -30 ${o}_gpu_tests.log; exit 1; }
tail -2 ${o}_gpu_tests.log
FAKEPTA_AMD_LIB=build/diag/lib_diag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "storer or union or interpolation_is_bitwise or partial_realization or lds or window_ring" > ${o}_diag_tests.log 2>&1 || { tail -30 ${o}_diag_tests.log; exit 1; }
tail -2 ${o}_diag_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
tail -3 ${o}_smoke.log
timeout -k 10 600 python -u bench.py > ${o}_bench.log 2>&1 || { tail -30 ${o}_bench.log; exit 1; }
tail -c 3000 ${o}_bench.log
