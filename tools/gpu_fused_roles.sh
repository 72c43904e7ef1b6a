set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5fx_tests.log 2>&1 || { tail -5 gpurun_out/r5fx_tests.log; exit 1; }
tail -1 gpurun_out/r5fx_tests.log
for v in "" cut1 cut2; do
  lib=fakepta_amd/lib/libfakepta_amd.so; [ -n "$v" ] && lib=build/diag/lib_$v.so
  FAKEPTA_AMD_LIB=$lib timeout -k 10 60 python -u bench.py --steps 30 --cpu-sample 0 --exact-launches 3 --sub-configs 0 > gpurun_out/r5fx_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r5fx_$v.log; exit 1; }
  grep -h '^{' gpurun_out/r5fx_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['isolated']['avg_launch_ms'])"
done
