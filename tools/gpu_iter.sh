#!/bin/bash
# Iteration pass: selected GPU tests, then C2 (and optionally C3 / C5) wall times and a kernel trace of C2.
#   bash tools/gpu_iter.sh <tag> "<pytest -k expr or empty>" [c3] [c5]
set -o pipefail
tag=$1; kexpr=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
if [ -n "$kexpr" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "$kexpr" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -30 ${o}_tests.log; exit 1; }
  tail -1 ${o}_tests.log
fi
timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
python - ${o}_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]
print("C2", round(d["value"] / 1e11, 3), "e11 samples/s", round(d["ms_per_step"], 4), "ms/step; interp", round(r["avg_launch_ms"], 4),
      "iso", r.get("isolated", {}).get("avg_launch_ms"), "dft iso", r.get("isolated", {}).get("dft_ms_per_block"))
PY
for c in "$@"; do
  if [ "$c" = c3 ]; then
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --steps 2 > ${o}_bench_c3.log 2>&1 || { tail -20 ${o}_bench_c3.log; exit 1; }
    grep '^{' ${o}_bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'])"
  fi
  if [ "$c" = c5 ]; then
    timeout -k 10 300 python -u tools/bench_configs.py c5 > ${o}_c5.jsonl 2>&1 || { tail -20 ${o}_c5.jsonl; exit 1; }
    cut -c1-300 ${o}_c5.jsonl
  fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c2 -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 > ${o}_prof_c2.log 2>&1 || { tail -20 ${o}_prof_c2.log; exit 1; }
python tools/trace_steps.py ${o}_prof_c2/run_kernel_trace.csv --last 15
