set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5tr1 -o run -- python bench.py --steps 10 --cpu-sample 0 --exact-launches 0 --sub-configs 0 > gpurun_out/r5tr1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5tr0 -o run -- python bench.py --steps 10 --cpu-sample 0 --exact-launches 0 --sub-configs 0 --overlap 0 > gpurun_out/r5tr0.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r5tr1.log gpurun_out/r5tr0.log | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])"
