set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/R6k
B="python bench.py --steps 20 --warmup 5 --cpu-sample 0 --sub-configs 0"
for i in 1 2; do
  timeout -k 10 300 $B > ${o}_ev$i.log 2>&1 || exit 1
  timeout -k 10 300 $B --no-kernel-events > ${o}_noev$i.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d ${o}_tr_noev -o run -- python bench.py --steps 10 --cpu-sample 0 --exact-launches 0 --sub-configs 0 --no-kernel-events > ${o}_tr_noev.log 2>&1 || exit 1
echo done
