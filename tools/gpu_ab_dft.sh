#!/bin/bash
# DFT wave tile A/B: product (32 rows x 64 realizations) vs build/diag/lib_dft4.so (64 x 32), grid tests + C2/C3.
mkdir -p gpurun_out
FAKEPTA_AMD_LIB=build/diag/lib_dft4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abd_tests.log 2>&1 || { tail -20 gpurun_out/abd_tests.log; exit 1; }
tail -1 gpurun_out/abd_tests.log
for rep in 1 2; do for lib in fakepta_amd/lib/libfakepta_amd.so build/diag/lib_dft4.so; do
  n=$(basename $lib .so)
  FAKEPTA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 3 > gpurun_out/abd_c2_${n}_$rep.log 2>&1 || exit 1
  FAKEPTA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 > gpurun_out/abd_c3_${n}_$rep.log 2>&1 || exit 1
done; done
for f in gpurun_out/abd_c*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; i=r.get('isolated') or {}; print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], i.get('avg_launch_ms'), i.get('dft_avg_launch_ms'), r['dft']['avg_launch_ms'], r['grid']['band_rows_per_chunk'])"; done
