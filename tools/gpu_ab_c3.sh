#!/bin/bash
# C3 A/B: pipelined blocks on/off x interpolation kernel (bench.py --config c3, 5 jobs each, alternating).
mkdir -p gpurun_out
for rep in 1 2; do for ov in 0 1; do for ws in 0 1; do
  timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 --interp-ws $ws --overlap $ov > gpurun_out/abc3_ov${ov}_ws${ws}_$rep.log 2>&1 || exit 1
done; done; done
for f in gpurun_out/abc3_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), '%.3e'%d['value'])"; done
