#!/bin/bash
# C3 and C2 A/B of the interpolation kernels, 3 alternating repetitions each (box noise is ~5 %).
mkdir -p gpurun_out
for rep in 1 2 3; do for ws in 0 1; do
  timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 --interp-ws $ws > gpurun_out/abw_c3_ws${ws}_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 30 --cpu-sample 0 --exact-launches 0 --interp-ws $ws > gpurun_out/abw_c2_ws${ws}_$rep.log 2>&1 || exit 1
done; done
for f in gpurun_out/abw_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), '%.3e'%d['value'])"; done
