#!/bin/bash
# C2 step with / without the bench's per-kernel HIP timing events, pipelined (OVERLAP 1) and one-stream (OVERLAP 0)
# blocks, alternating, two repetitions; then kernel traces of the one-stream step with and without events.
set -o pipefail
tag=${1:-r5ev}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_grid.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused or gen_mix" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
out=gpurun_out/${tag}_ab.txt; : > $out
for rep in 1 2; do
  for ov in 1 0; do
    for ev in on off; do
      fl=""; [ $ev = off ] && fl="--no-kernel-events"
      timeout -k 10 120 python bench.py --cpu-sample 0 --sub-configs 0 --steps 50 --warmup 30 --overlap $ov $fl > gpurun_out/${tag}_o${ov}_$ev.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_o${ov}_$ev.json').read().strip().splitlines()[-1]); print('rep $rep overlap $ov events $ev', round(d['ms_per_step'],4), 'fused launch (events)', d['roofline'].get('avg_launch_ms'))" | tee -a $out
    done
  done
done
for ev in on off; do
  fl=""; [ $ev = off ] && fl="--no-kernel-events"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_tr0_$ev -o run -- python3 bench.py --cpu-sample 0 --sub-configs 0 --steps 20 --warmup 30 --overlap 0 $fl > gpurun_out/${tag}_tr0_$ev.log 2>&1 || exit 1
done
