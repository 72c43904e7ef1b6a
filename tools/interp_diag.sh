#!/bin/bash
# Build diagnostic variants of k_grid_interp_sparse (throwaway copies of grid_sparse.hip in build/diag, never
# shipped) and time each on C2: d0 unchanged, d1 no FMA chain, d2 no output stores, d3 no grid-row loads.
# Build here (no GPU needed): bash tools/interp_diag.sh build ; run on the GPU box: bash tools/interp_diag.sh run
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
D=build/diag
if [ "$1" = "build" ]; then
  mkdir -p $D
  S=fakepta_amd/csrc
  F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -fno-gpu-rdc -I$S"
  for v in 0 1 2 3; do
    cp $S/grid_sparse.hip $D/gs$v.hip
    case $v in
      1) sed -i 's/^\(\s*\)window_dot<WS>(acc, acc1, wa, wb, win);/\1acc1 = wa + wb;/' $D/gs$v.hip ;;
      2) sed -i 's/if (r < a.n_real) ocol\[(int64_t)r \* a.ldo\] = Tw\[tt\]\[rr\];/if (r < a.n_real \&\& Tw[tt][rr] == 1.2345e300) ocol[(int64_t)r * a.ldo] = 0.0;/' $D/gs$v.hip ;;
      3) sed -i 's/win\[i\] = G\[(int64_t)j \* R_pad\];/win[i] = G[(int64_t)(i \& 1) * R_pad];/' $D/gs$v.hip ;;
    esac
    /opt/rocm/bin/hipcc $F -c $D/gs$v.hip -mllvm -sink-common-insts=false -o $D/gs$v.o || exit 1
    /opt/rocm/bin/hipcc $F -shared $S/kernels.hip $S/dense.hip $S/grid.hip $S/grid_mfma.hip $S/capi.hip -x none $D/gs$v.o -o $D/lib_d$v.so || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out
for v in 0 1 2 3; do
  FAKEPTA_AMD_LIB=$D/lib_d$v.so timeout -k 5 120 python tools/interp_diag.py --label d$v || exit 1
done
timeout -k 5 120 python tools/interp_diag.py --label mfma --grid-mfma 3 || exit 1
