#!/bin/bash
# Quick GPU pass while iterating: gridded / C3 tests, bench C2 and C3, and a 2-rank gloo rehearsal of both on one
# card (the driver runs the real N-GPU benches).   bash tools/gpu_quick.sh <tag>
set -o pipefail
tag=${1:-quick}
o=gpurun_out/$tag
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_grid.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_tests.log 2>&1 || { tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > ${o}_c3.log 2>&1 || { tail -20 ${o}_c3.log; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-sample 0 --exact-launches 0 > ${o}_c2.log 2>&1 || { tail -20 ${o}_c2.log; exit 1; }
if [ -n "$REHEARSE" ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --cpu-sample 0 --exact-launches 0 > ${o}_rehearsal_c2.log 2>&1 || { tail -20 ${o}_rehearsal_c2.log; exit 1; }
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --config c3 --dist-backend gloo --cpu-sample 0 > ${o}_rehearsal_c3.log 2>&1 || { tail -20 ${o}_rehearsal_c3.log; exit 1; }
fi
for f in ${o}_c3 ${o}_c2 ${o}_rehearsal_c2 ${o}_rehearsal_c3; do
  [ -f $f.log ] && grep "^{" $f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['n_gpus'], d['kernels_ms_per_step'])"
done
exit 0
