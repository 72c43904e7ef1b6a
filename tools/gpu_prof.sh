#!/bin/bash
# rocprofv3 kernel-trace stats + FETCH/WRITE passes over the default bench (profiles/ evidence).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc_traffic
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --cpu-sample 0 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_traffic/pass0 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/pmc_traffic0.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_traffic/pass1 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/pmc_traffic1.log 2>&1 || exit 1
python tools/collect_traffic.py gpurun_out/pmc_traffic gpurun_out/traffic.json 320 200000 1024 k_grid_interp_mfma
