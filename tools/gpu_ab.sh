#!/bin/bash
# A/B of library options on one box: each variant runs bench.py (C2 or C3) twice, alternating.
#   bash tools/gpu_ab.sh <tag> <c2|c3> "<variant args 1>" "<variant args 2>" ...
set -o pipefail
tag=$1; cfg=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    if [ "$cfg" = c3 ]; then extra="--config c3 --steps 2 --warmup 1"; else extra="--steps 30 --exact-launches 0"; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 $extra $v > gpurun_out/${tag}_v$i.log 2>&1 || { tail -20 gpurun_out/${tag}_v$i.log; exit 1; }
    grep '^{' gpurun_out/${tag}_v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep $rep', '$cfg', repr('$v'), round(d['ms_per_step'],4), 'ms/step', '%.3e' % d['value'])" | tee -a $out
    i=$((i+1))
  done
done
