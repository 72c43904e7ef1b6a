#!/bin/bash
# C5: the ECORR epoch normals of pipelined blocks on a stream of their own (make variant NAME=zside
# DEFS=-DFPTA_EPOCH_SIDE=1) vs the shipped library; the white / ECORR GPU tests on the variant first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAKEPTA_AMD_LIB=build/diag/lib_zside.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "white or ecorr or c5 or pipelined" > gpurun_out/R6v_tests.log 2>&1 || { tail -30 gpurun_out/R6v_tests.log; exit 1; }
tail -1 gpurun_out/R6v_tests.log
bash tools/gpu_ab_cfg.sh R6v "" c5 "" "LIB=build/diag/lib_zside.so" || exit 1
