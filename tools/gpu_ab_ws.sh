#!/bin/bash
# A/B of the two gridded interpolation kernels in the driver's bench (C2 and C3), alternating, 2 runs each.
mkdir -p gpurun_out
for rep in 1 2; do for ws in 0 1; do
  timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 0 --interp-ws $ws > gpurun_out/ab_c2_ws${ws}_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config c3 --steps 2 --cpu-sample 0 --interp-ws $ws > gpurun_out/ab_c3_ws${ws}_$rep.log 2>&1 || exit 1
done; done
for f in gpurun_out/ab_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(d['roofline']['avg_launch_ms'],4), d['roofline']['kernel'])"; done
