#!/bin/bash
# Same-box A/B: the product library against build/diag/lib_prev.so (an earlier commit's build), C2 and C3, alternating.
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in fakepta_amd/lib/libfakepta_amd.so build/diag/lib_prev.so; do
  n=$(basename $lib .so)
  FAKEPTA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 3 > gpurun_out/abp_c2_${n}_$rep.log 2>&1 || exit 1
done; done
for rep in 1 2; do for lib in fakepta_amd/lib/libfakepta_amd.so build/diag/lib_prev.so; do
  n=$(basename $lib .so)
  FAKEPTA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 > gpurun_out/abp_c3_${n}_$rep.log 2>&1 || exit 1
done; done
for f in gpurun_out/abp_c*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; i=r.get('isolated') or {}; print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['avg_launch_ms'],4), i.get('avg_launch_ms'))"; done
