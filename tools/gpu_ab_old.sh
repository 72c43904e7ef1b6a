#!/bin/bash
# Same-box comparison against the tree in build/oldtree (an earlier commit, built in place): C2 and C3 benches.
mkdir -p gpurun_out
for rep in 1 2; do
  (cd build/oldtree && timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 0 > ../../gpurun_out/old_c2_$rep.log 2>&1) || exit 1
  timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 0 > gpurun_out/new_c2_$rep.log 2>&1 || exit 1
  (cd build/oldtree && timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 > ../../gpurun_out/old_c3_$rep.log 2>&1) || exit 1
  timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 > gpurun_out/new_c3_$rep.log 2>&1 || exit 1
done
for f in gpurun_out/old_c*.log gpurun_out/new_c*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), '%.3e'%d['value'])"; done
