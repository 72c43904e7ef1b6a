#!/bin/bash
# A/B of library options on one box, for C2 / C3 (bench.py) and C4 / C5 (tools/bench_configs.py), alternating variants,
# two repetitions; optional GPU test selection first.
#   bash tools/gpu_ab_cfg.sh <tag> "<pytest -k expr or empty>" <c2|c3|c4|c5> "<opts 1>" "<opts 2>" ...
# opts are NAME=VALUE library options separated by spaces ("" = the library defaults); LIB=<path.so> runs that variant
# on another build of the library (make -C fakepta_amd/csrc variant ...).
set -o pipefail
tag=$1; kexpr=$2; cfg=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$kexpr" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "$kexpr" > gpurun_out/${tag}_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/${tag}_tests.log | head -20; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    flags=""
    lib=fakepta_amd/lib/libfakepta_amd.so
    for kv in $v; do
      case $kv in LIB=*) lib=${kv#LIB=} ;; *) flags="$flags --opt $kv" ;; esac
    done
    export FAKEPTA_AMD_LIB=$lib
    log=gpurun_out/${tag}_${cfg}_v${i}_r$rep.log
    case $cfg in
      c2) timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 --exact-launches 3 $flags > $log 2>&1 ;;
      c3) timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c3 --steps 4 --warmup 2 --sub-configs 0 $flags > $log 2>&1 ;;
      *) timeout -k 10 300 python -u tools/bench_configs.py $cfg $flags > $log 2>&1 ;;
    esac || { tail -20 $log; exit 1; }
    grep '^{' $log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
ms=d.get('ms_per_step')
r=d.get('roofline',{})
print('rep $rep', '$cfg', repr('$v'), round(ms,4), 'ms/step', 'interp', r.get('avg_launch_ms'), 'iso', r.get('isolated',{}).get('avg_launch_ms'), 'dft_iso', r.get('isolated',{}).get('dft_ms_per_block'), 'k', d.get('isolated_kernels_ms_per_step'))" | tee -a $out
    i=$((i+1))
  done
done
