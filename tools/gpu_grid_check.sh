#!/bin/bash
# GPU-box check of the gridded path: parity tests, kernel A/B sweep, bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -2 gpurun_out/grid_tests.log
timeout -k 10 240 python -u tools/sweep_grid.py --rounds 3 --reps 5 --masks 1,3 > gpurun_out/sweep_grid.log 2>&1 || { tail -20 gpurun_out/sweep_grid.log; exit 1; }
echo "LDS"; cat gpurun_out/sweep_grid.log
FPTA_INTERP_DIRECT=1 timeout -k 10 240 python -u tools/sweep_grid.py --rounds 3 --reps 5 --masks 3 > gpurun_out/sweep_grid_direct.log 2>&1 || { tail -20 gpurun_out/sweep_grid_direct.log; exit 1; }
echo "DIRECT"; cat gpurun_out/sweep_grid_direct.log
timeout -k 10 240 python -u bench.py --cpu-sample 0 > gpurun_out/bench_grid.log 2>&1 || { tail -20 gpurun_out/bench_grid.log; exit 1; }
cat gpurun_out/bench_grid.log
