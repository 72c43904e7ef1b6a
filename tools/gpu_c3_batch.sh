#!/bin/bash
# C3 job time by batch size (bench.py --config c3 --c3-batch B), same box, alternating sizes.
#   bash tools/gpu_c3_batch.sh <tag> [reps] [sizes ...]
set -o pipefail
tag=${1:-C3B}; reps=${2:-2}; shift 2; sizes=${*:-4096 8192 12500 16384}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in $(seq 1 $reps); do
  for b in $sizes; do
    log=gpurun_out/${tag}_b${b}_r$rep.log
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c3 --steps 4 --warmup 2 --sub-configs 0 --c3-batch $b > $log 2>&1 || { tail -20 $log; exit 1; }
    grep '^{' $log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('rep $rep batch $b', round(d['ms_per_step'],3), 'ms/job', 'interp', round(d['roofline']['avg_launch_ms'],4))" | tee -a $out
  done
done
