#!/bin/bash
# C2 gridded-path timing of k_grid_interp_mfma and k_grid_dft_mfma per kernel width at sigma 1.5
# (tools/interp_diag.py: HIP-event averages over 10 batches of 1024 realizations).
set -o pipefail
mkdir -p gpurun_out
for w in 14 15 16; do
  timeout -k 5 120 python tools/interp_diag.py --label "w$w" --width $w || exit 1
done
