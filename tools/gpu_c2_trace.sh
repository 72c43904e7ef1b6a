#!/bin/bash
# Kernel trace of the C2 bench (short run, no CPU legs, no sub-records) and its per-step timeline.
#   bash tools/gpu_c2_trace.sh <tag> [bench options ...]
set -o pipefail
tag=${1:-C2T}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --cpu-sample 0 --steps 20 --sub-configs 0 --exact-launches 0 "$@" > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_grid_interp --last 8 > ${o}_steps.txt; cat ${o}_steps.txt; true

