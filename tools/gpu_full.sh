#!/bin/bash
# Full GPU validation + measurement pass (round evidence): tests, smoke, HBM traffic of the gridded interpolation,
# bench C2 (+ CPU baseline) and C3, exact-path bench, configs, rocprof kernel stats.
#   bash tools/gpu_full.sh <tag>     (outputs under gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > ${o}_gpu_tests.log 2>&1 || { tail -40 ${o}_gpu_tests.log; exit 1; }
  tail -3 ${o}_gpu_tests.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
  cat ${o}_smoke.log
fi
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d ${o}_traffic/pass$i -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 > ${o}_traffic_$p.log 2>&1 || { tail -20 ${o}_traffic_$p.log; exit 1; }
  i=$((i+1))
done
python tools/collect_traffic.py ${o}_traffic ${o}_grid_traffic.json 320 200000 1024 k_grid_interp_ws band32c || exit 1
timeout -k 10 300 python -u bench.py --traffic ${o}_grid_traffic.json > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
cat ${o}_bench.log
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $p --output-format csv -d ${o}_traffic_c3/pass$i -o run -- python bench.py --config c3 --steps 1 --warmup 1 --cpu-sample 0 > ${o}_traffic_c3_$p.log 2>&1 || { tail -20 ${o}_traffic_c3_$p.log; exit 1; }
  i=$((i+1))
done
python tools/collect_traffic.py ${o}_traffic_c3 ${o}_grid_traffic_c3.json 60 200000 4096 k_grid_interp_mfma band32c || exit 1
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --traffic ${o}_grid_traffic_c3.json > ${o}_bench_c3.log 2>&1 || { tail -20 ${o}_bench_c3.log; exit 1; }
cat ${o}_bench_c3.log
timeout -k 10 300 python -u bench.py --path 3 --cpu-sample 0 > ${o}_bench_exact.log 2>&1 || { tail -20 ${o}_bench_exact.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py c1 c3 c4 c5 > ${o}_configs.jsonl 2>&1 || { tail -20 ${o}_configs.jsonl; exit 1; }
cat ${o}_configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
find ${o}_prof -name "*kernel_stats.csv"
