#!/bin/bash
# Same-box C2 A/B of the product library against throwaway builds (LIBS, default build/diag/lib_prev.so), alternating,
# REPS rounds; prints ms/step, samples/s, the interpolation's co-run launch time and the per-kernel side-stream times.
mkdir -p gpurun_out
TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-3}); do for lib in fakepta_amd/lib/libfakepta_amd.so ${LIBS:-build/diag/lib_prev.so}; do
  n=$(basename $lib .so)
  FAKEPTA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 1 > gpurun_out/${TAG}_c2_${n}_$rep.log 2>&1 || exit 1
done; done
for f in gpurun_out/${TAG}_c2_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; k=d['kernels_ms_per_step']; print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['avg_launch_ms'],4), {a: round(b, 3) for a, b in k.items()})"; done
