#!/bin/bash
# The round's GPU evidence in one call: the GPU suite on the product library and on the variant build (the
# diagnostic kernels and the variant-only option values), smoke(), and the default bench line.
#   bash tools/gpu_suite.sh <tag>      (outputs gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-R5a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_gpu_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_gpu_tests.log | head; tail -5 ${o}_gpu_tests.log; exit 1; }
tail -1 ${o}_gpu_tests.log
FAKEPTA_AMD_LIB=build/diag/lib_diag.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_diag_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_diag_tests.log | head; tail -5 ${o}_diag_tests.log; exit 1; }
tail -1 ${o}_diag_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
tail -1 ${o}_smoke.log
timeout -k 10 400 python -u bench.py > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
grep '^{' ${o}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('isolated'), r.get('fp64_pipe'), d.get('c5',{}).get('ms_per_step'), d.get('c3',{}).get('ms_per_job'), d.get('c4_per_gpu',{}).get('ms_per_step'))"
