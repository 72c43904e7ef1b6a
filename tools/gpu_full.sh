#!/bin/bash
# Full GPU validation + measurement pass (round evidence): tests, smoke, bench (+CPU baseline), configs, rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --path 3 --cpu-sample 0 > gpurun_out/bench_exact.log 2>&1 || { tail -20 gpurun_out/bench_exact.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py c1 c3 c4 c5 > gpurun_out/configs.jsonl 2>&1 || { tail -20 gpurun_out/configs.jsonl; exit 1; }
cat gpurun_out/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 20 --cpu-sample 0 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
