#!/bin/bash
# C2 (k_grid_fused): pipelined (OVERLAP 1, k_gen_mix of the next block on the side stream) vs one-stream (OVERLAP 0)
# blocks, alternating, four repetitions at W 30 / K 50 and at the driver's W 5 / K 20.
set -o pipefail
tag=${1:-r5ov}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt; : > $out
for wk in "30 50" "5 20"; do
  set -- $wk
  for rep in 1 2 3 4; do
    for ov in 1 0; do
      timeout -k 10 120 python bench.py --cpu-sample 0 --sub-configs 0 --warmup $1 --steps $2 --overlap $ov > gpurun_out/${tag}_o$ov.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_o$ov.json').read().strip().splitlines()[-1]); print('W $1 K $2 rep $rep overlap $ov', round(d['ms_per_step'],4), 'fused launch', round(d['roofline'].get('avg_launch_ms'),4))" | tee -a $out
    done
  done
done
