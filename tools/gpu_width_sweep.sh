#!/bin/bash
# C2 gridded-path timing per (interpolation kernel, width) at sigma 1.5 (tools/sweep_grid.py --params-style):
# bench.py lines for the MFMA and the sparse VALU interpolation at widths 14, 15, 16.
set -o pipefail
mkdir -p gpurun_out
for w in 14 15 16; do
  for m in 3 1; do
    timeout -k 5 120 python tools/interp_diag.py --label "w$w-mask$m" --grid-mfma $m --width $w || exit 1
  done
done
