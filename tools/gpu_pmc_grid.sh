#!/bin/bash
# PMC passes over a short gridded-path bench (kernel-level counters of k_grid_dft*/k_grid_interp*).
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_profile.sh gpurun_out/pmc_grid -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 "$@" || exit 1
python tools/pmc_summary.py gpurun_out/pmc_grid --match grid > gpurun_out/pmc_grid.txt 2>&1 || exit 1
cat gpurun_out/pmc_grid.txt
