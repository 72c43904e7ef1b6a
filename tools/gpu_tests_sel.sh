#!/bin/bash
# Selected GPU tests (verbose log under gpurun_out/<tag>_tests.log).   bash tools/gpu_tests_sel.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -40
exit $rc
