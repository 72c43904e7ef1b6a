#!/bin/bash
# NOTE (round 4): the FPTA_INTERP_DIAG cuts below were removed from the product source; this
# script reproduces the round-2/3 records only on a checkout of revision 059c9cc or earlier.
# Build (build) or time (run) compile-time variants of k_grid_interp_mfma: realization tiles per wave (RW),
# persistent workgroups per CU (WPC), diagnostic cuts (DIAG 1: grid loads from one L1-resident row; 2: no
# stores; 3: non-temporal stores; 4: no band loop, the store stream alone; 5: every other workgroup starts
# ~7 us late; 6: k_grid_interp_ws producers load nothing; 7: 1 and 2 together, the MFMA stream alone; 8: accumulators in AGPRs; 9: waves of a CU staggered by 0..7 x 3.4 us). WS selects FPTA_OPT_INTERP_WS values to time. VARIANTS entries are RW:WPC:DIAG. Throwaway libraries in build/diag, loaded by tools/interp_diag.py
# through FAKEPTA_AMD_LIB; never the product or the bench. Results: profiles/r02_interp_diag*.txt (a single
# operand set at 3 workgroups per CU measured 0.70 ms against 0.66 for the shipped 2-deep pipeline at 2).
S=fakepta_amd/csrc
D=build/diag
VARIANTS=${VARIANTS:-"8:2:0 8:2:2 8:2:4 8:2:6"}
if [ "$1" = build ]; then
  mkdir -p $D
  for v in $VARIANTS; do
    IFS=: read rw wpc dg <<< "$v"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result -ffp-contract=fast \
      -fno-gpu-rdc -DFPTA_INTERP_RW=$rw -DFPTA_INTERP_WPC=$wpc -DFPTA_INTERP_DIAG=$dg ${EXTRA:-} $S/kernels.hip $S/dense.hip $S/grid.hip \
      $S/grid_mfma.hip $S/capi.hip -o $D/lib_rw${rw}_wpc${wpc}_d${dg}.so &
  done
  wait
  exit 0
fi
set -o pipefail
for v in $VARIANTS; do
  IFS=: read rw wpc dg <<< "$v"
  for ws in ${WS:-0 1}; do
    FAKEPTA_AMD_LIB=$D/lib_rw${rw}_wpc${wpc}_d${dg}.so timeout -k 5 120 python tools/interp_diag.py --ws $ws --label "rw$rw-wpc$wpc-d$dg-ws$ws" || exit 1
  done
done
