#!/bin/bash
# C2 throughput against realizations per step (bench.py --real): whether smaller blocks (grid values resident in
# the 256 MB Infinity Cache between the DFT and the interpolation) pay.
set -o pipefail
mkdir -p gpurun_out
for r in 256 512 1024 2048 4096; do
  timeout -k 10 200 python -u bench.py --real $r --steps 20 --cpu-sample 0 --exact-launches 0 > gpurun_out/bs_$r.log 2>&1 || exit 1
  grep "^{" gpurun_out/bs_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($r, d['value'], d['ms_per_step'], d['kernels_ms_per_step'])"
done
