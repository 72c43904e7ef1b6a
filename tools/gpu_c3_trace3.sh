#!/bin/bash
# C3 kernel trace: per-batch statistics and the launch timeline of the last batches (tools/trace_steps.py)
set -o pipefail
tag=${1:-C3T3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_part_sums --last 20 --timeline 4 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
