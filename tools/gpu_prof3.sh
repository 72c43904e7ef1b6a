#!/bin/bash
# Kernel traces of C2 (pipelined and one-stream), C3 and C5 with per-step summaries (tools/trace_steps.py).
#   bash tools/gpu_prof3.sh <tag> [extra bench.py args for C2]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 "$@" > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
grep '^{' ${o}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C2', d['value'], d['ms_per_step'], 'interp', r['avg_launch_ms'], 'iso', r.get('isolated',{}).get('avg_launch_ms'), r.get('isolated',{}).get('dft_ms_per_block'))"
for ov in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${o}_c2ov$ov -o run -- python bench.py --steps 12 --cpu-sample 0 --exact-launches 0 --overlap $ov "$@" > ${o}_c2ov$ov.log 2>&1 || { tail -20 ${o}_c2ov$ov.log; exit 1; }
  echo "== C2 overlap $ov"; python tools/trace_steps.py ${o}_c2ov$ov/run_kernel_trace.csv --last 8
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${o}_c3 -o run -- python bench.py --config c3 --steps 1 --warmup 1 --cpu-sample 0 > ${o}_c3.log 2>&1 || { tail -20 ${o}_c3.log; exit 1; }
grep '^{' ${o}_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 (under rocprof)', d['value'], d['ms_per_step'])"
echo "== C3"; python tools/trace_steps.py ${o}_c3/run_kernel_trace.csv --marker k_part_final --last 12
timeout -k 10 300 python -u tools/bench_configs.py c5 > ${o}_c5.jsonl 2>&1 || { tail -20 ${o}_c5.jsonl; exit 1; }
cut -c1-400 ${o}_c5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${o}_c5 -o run -- python tools/bench_configs.py c5 > ${o}_c5p.log 2>&1 || { tail -20 ${o}_c5p.log; exit 1; }
echo "== C5"; python tools/trace_steps.py ${o}_c5/run_kernel_trace.csv --last 6
