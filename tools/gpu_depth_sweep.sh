#!/bin/bash
# k_grid_interp_mfma prefetch depth 2 (product) vs 3 (build/diag/lib_depth3.so), kernels alone and pipelined.
mkdir -p gpurun_out
for lib in fakepta_amd/lib/libfakepta_amd.so build/diag/lib_depth3.so; do
  for ov in 0 1; do
    FAKEPTA_AMD_LIB=$lib timeout -k 5 120 python tools/interp_diag.py --ws 0 --overlap $ov --label "$(basename $lib)-ws0-ov$ov" || exit 1
  done
done
