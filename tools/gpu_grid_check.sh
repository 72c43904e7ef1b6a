set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_c3.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_grid_sparse.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r02_grid_sparse.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.err
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --grid-mfma 3 --exact-launches 0 > gpurun_out/r02_bench3_mfma.json 2>> gpurun_out/r02_bench3.err
echo done
