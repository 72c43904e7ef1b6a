mkdir -p gpurun_out
for lib in fakepta_amd/lib/libfakepta_amd.so build/diag/lib_lead7.so; do
  for ws in 0 1; do for ov in 0 1; do
    FAKEPTA_AMD_LIB=$lib timeout -k 5 120 python tools/interp_diag.py --ws $ws --overlap $ov --label "$(basename $lib)-ws$ws-ov$ov" || exit 1
  done; done
done
