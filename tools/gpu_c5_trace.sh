#!/bin/bash
set -o pipefail
tag=${1:-C5T}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python tools/bench_configs.py c5 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_grid_interp --last 10 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
