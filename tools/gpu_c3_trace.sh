set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/C3T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
grep '^{' ${o}_prof.log | head -c 600
find ${o}_prof -name "*.csv"
