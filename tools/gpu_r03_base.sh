#!/bin/bash
# Round-3 starting point: GPU tests, smoke, bench C2/C3, configs, rocprof kernel stats of C2, C3 and C5.
#   bash tools/gpu_r03_base.sh <tag>
set -o pipefail
tag=${1:-r03a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > ${o}_gpu_tests.log 2>&1 || { tail -40 ${o}_gpu_tests.log; exit 1; }
tail -2 ${o}_gpu_tests.log
timeout -k 10 300 python -u bench.py --cpu-sample 0 > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
grep '^{' ${o}_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > ${o}_bench_c3.log 2>&1 || { tail -20 ${o}_bench_c3.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py c5 > ${o}_configs.jsonl 2>&1 || { tail -20 ${o}_configs.jsonl; exit 1; }
cut -c1-300 ${o}_configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c2 -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 > ${o}_prof_c2.log 2>&1 || { tail -20 ${o}_prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c3 -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 > ${o}_prof_c3.log 2>&1 || { tail -20 ${o}_prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c5 -o run -- python tools/bench_configs.py c5 > ${o}_prof_c5.log 2>&1 || { tail -20 ${o}_prof_c5.log; exit 1; }
find ${o}_prof_* -name "*kernel_stats.csv"
