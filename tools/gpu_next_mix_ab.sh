#!/bin/bash
# FPTA_OPT_FUSED_NEXT_MIX A/B on C2 (one box): the shipped library with the option on and off, and variant builds of
# FusedMix::min_left (make variant NAME=ml<v> DEFS=-DFPTA_FUSED_MIX_MIN_LEFT=<v>), each twice in turn; then kernel
# traces of on / off.
#   bash tools/gpu_next_mix_ab.sh <tag> [variant names...]
set -o pipefail
tag=${1:-R6h}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 420 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_next_mix.py tests/test_gpu_fused.py > ${o}_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --cpu-sample 0 --sub-configs 0"
for i in 1 2; do
  timeout -k 10 300 $B > ${o}_bench_on$i.log 2>&1 || exit 1
  timeout -k 10 300 $B --opt fused_next_mix=0 > ${o}_bench_off$i.log 2>&1 || exit 1
  for v in "$@"; do
    FAKEPTA_AMD_LIB=build/diag/lib_$v.so timeout -k 10 300 $B > ${o}_bench_${v}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d ${o}_tr_on -o run -- python bench.py --steps 10 --cpu-sample 0 --exact-launches 0 --sub-configs 0 > ${o}_tr_on.log 2>&1 || exit 1
echo done
