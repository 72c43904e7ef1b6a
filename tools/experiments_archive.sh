#!/bin/bash
# Archive of the one-off GPU experiment command lines of rounds 2-6 (formerly tools/gpu_<name>.sh or tools/<name>.sh,
# one file each; exp_<name> without the gpu_ prefix).
# Each is a function named after its old file (bodies unindented: some hold here-documents); the records they
# produced are under profiles/ (the tags in the bodies). Kept for provenance only, NOT runnable: several bodies call
# the tools/gpu_*.sh files this archive replaced (gpu_c3_trace.sh, gpu_c3_trace3.sh, gpu_c3_batch.sh, gpu_full.sh,
# ...), and variant libraries (build/diag/lib_*.so) of revisions long gone. New A/B runs go through
# tools/gpu_ab_cfg.sh configurations.
#   bash tools/experiments_archive.sh <name>   # prints the archived body of exp_<name> (e.g. psr3, c3_ab2)

exp_c2_trace() {
# Kernel trace of the C2 bench (short run, no CPU legs, no sub-records) and its per-step timeline.
#   bash tools/gpu_c2_trace.sh <tag> [bench options ...]
set -o pipefail
tag=${1:-C2T}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --cpu-sample 0 --steps 20 --sub-configs 0 --exact-launches 0 "$@" > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_grid_interp --last 8 > ${o}_steps.txt; cat ${o}_steps.txt; true

}

exp_c3_ab2() {
set -o pipefail
tag=${1:-PG2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_c3_trace.sh || exit 1
python tools/trace_steps.py gpurun_out/C3T_prof/run_kernel_trace.csv --marker k_part_final --last 20 > gpurun_out/${tag}_c3_trace.txt || exit 1
cat gpurun_out/${tag}_c3_trace.txt
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "ASYNC_SUMS=1" "PART_GROUP=16" "PART_GROUP=8" || exit 1
}

exp_c3_ab3() {
set -o pipefail
tag=${1:-PG3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "INTERP_WS=2" "PART_GROUP=16" "INTERP_WS=2 PART_GROUP=16" || exit 1
}

exp_c3_ab4() {
set -o pipefail
tag=${1:-PG4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "LIB=build/diag/lib_pwpc1.so" "PART_GROUP=16" "LIB=build/diag/lib_pwpc1.so PART_GROUP=16" || exit 1
}

exp_c3_ab5() {
set -o pipefail
tag=${1:-PG5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "LIB=build/diag/lib_pwg14.so" "LIB=build/diag/lib_pwg12.so" || exit 1
}

exp_c3_ab6() {
set -o pipefail
tag=${1:-PSR4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "ASYNC_SUMS=1" "GEN_MIX=3" || exit 1
}

exp_c3_ab7() {
# C3: checksum / pipelining tests, the A/B of the deferred ev_gfree record, and the timeline with it
set -o pipefail
tag=${1:-R5u}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh $tag "c3 or checksum or rccl or multi or pipelined or coalesced or psr" c3 "" "LIB=build/diag/lib_early.so" && bash tools/gpu_c3_trace3.sh ${tag}T
}

exp_c3_batch() {
# C3 job time by batch size (bench.py --config c3 --c3-batch B), same box, alternating sizes.
#   bash tools/gpu_c3_batch.sh <tag> [reps] [sizes ...]
set -o pipefail
tag=${1:-C3B}; reps=${2:-2}; shift 2; sizes=${*:-4096 8192 12500 16384}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in $(seq 1 $reps); do
  for b in $sizes; do
    log=gpurun_out/${tag}_b${b}_r$rep.log
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c3 --steps 4 --warmup 2 --sub-configs 0 --c3-batch $b > $log 2>&1 || { tail -20 $log; exit 1; }
    grep '^{' $log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('rep $rep batch $b', round(d['ms_per_step'],3), 'ms/job', 'interp', round(d['roofline']['avg_launch_ms'],4))" | tee -a $out
  done
done
}

exp_c3_trace() {
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/C3T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
grep '^{' ${o}_prof.log | head -c 600
find ${o}_prof -name "*.csv"
}

exp_c3_trace2() {
# C3 kernel trace + per-batch timeline (tools/trace_steps.py and the last batches' launches)
set -o pipefail
tag=${1:-C3T2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_part_final --last 20 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
}

exp_c3_trace3() {
# C3 kernel trace: per-batch statistics and the launch timeline of the last batches (tools/trace_steps.py)
set -o pipefail
tag=${1:-C3T3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_part_sums --last 20 --timeline 4 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
}

exp_c5_ab() {
set -o pipefail
tag=${1:-C5A}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c5 "" "LIB=build/diag/lib_rw4w3.so" "LIB=build/diag/lib_rw4w2.so" || exit 1
}

exp_c5_trace() {
set -o pipefail
tag=${1:-C5T}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python tools/bench_configs.py c5 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_grid_interp --last 10 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
}

exp_full() {
# Full GPU validation + measurement pass (round evidence): tests, smoke, HBM traffic of the gridded interpolation,
# bench C2 (+ CPU baseline) and C3, exact-path bench, configs, rocprof kernel stats.
#   bash tools/gpu_full.sh <tag>     (outputs under gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > ${o}_gpu_tests.log 2>&1 || { tail -40 ${o}_gpu_tests.log; exit 1; }
  tail -3 ${o}_gpu_tests.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
  cat ${o}_smoke.log
fi
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d ${o}_traffic/pass$i -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 > ${o}_traffic_$p.log 2>&1 || { tail -20 ${o}_traffic_$p.log; exit 1; }
  i=$((i+1))
done
python tools/collect_traffic.py ${o}_traffic ${o}_grid_traffic.json 320 200000 1024 k_grid_interp_ws band32c || exit 1
timeout -k 10 300 python -u bench.py --traffic ${o}_grid_traffic.json > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
cat ${o}_bench.log
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $p --output-format csv -d ${o}_traffic_c3/pass$i -o run -- python bench.py --config c3 --steps 1 --warmup 1 --cpu-sample 0 > ${o}_traffic_c3_$p.log 2>&1 || { tail -20 ${o}_traffic_c3_$p.log; exit 1; }
  i=$((i+1))
done
python tools/collect_traffic.py ${o}_traffic_c3 ${o}_grid_traffic_c3.json 60 200000 4096 k_grid_interp_mfma band32c || exit 1
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --traffic ${o}_grid_traffic_c3.json > ${o}_bench_c3.log 2>&1 || { tail -20 ${o}_bench_c3.log; exit 1; }
cat ${o}_bench_c3.log
timeout -k 10 300 python -u bench.py --path 3 --cpu-sample 0 > ${o}_bench_exact.log 2>&1 || { tail -20 ${o}_bench_exact.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py c1 c3 c4 c5 > ${o}_configs.jsonl 2>&1 || { tail -20 ${o}_configs.jsonl; exit 1; }
cat ${o}_configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
find ${o}_prof -name "*kernel_stats.csv"
}

exp_iter() {
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
}

exp_pg() {
# Partial-checksum groups (FPTA_OPT_PART_GROUP): the checksum / interpolation tests, the diagnostic-kernel tests on the
# variant build, then C3 A/B of group sizes against the previous HEAD's library.
#   bash tools/gpu_pg.sh <tag>
set -o pipefail
tag=${1:-PG}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_grid.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_tests.log | head; tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
FAKEPTA_AMD_LIB=build/diag/lib_diag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "storer or union or interpolation_is_bitwise or partial_realization or lds" > ${o}_diag_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_diag_tests.log | head; tail -30 ${o}_diag_tests.log; exit 1; }
tail -1 ${o}_diag_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "PART_GROUP=4" "LIB=build/diag/lib_head.so" || exit 1
}

exp_pmc_grid() {
# PMC passes over a short gridded-path bench (kernel-level counters of k_grid_dft*/k_grid_interp*).
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_profile.sh gpurun_out/pmc_grid -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 "$@" || exit 1
python tools/pmc_summary.py gpurun_out/pmc_grid --match grid > gpurun_out/pmc_grid.txt 2>&1 || exit 1
cat gpurun_out/pmc_grid.txt
}

exp_pmc_r03() {
# PMC of every shipped config kernel with the kernels serialised (one stream), so each dispatch's counters are its own:
# C2 (k_grid_dft_gen, k_gen_mix, k_grid_interp_ws), C3 (k_grid_dft_mfma, fused-checksum interpolation), C5 (white
# epilogue interpolation, k_epoch_normals).
#   bash tools/gpu_pmc_r03.sh <tag>
set -o pipefail
tag=${1:-r03c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
run() {  # <name> <cmd...>
  local name=$1; shift
  bash tools/pmc_passes.sh gpurun_out/${tag}_$name "$P0" "$P1" "$P2" "$P3" "$P4" -- "$@" || { echo "pmc $name failed"; tail -20 gpurun_out/${tag}_$name/pass*.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/${tag}_$name > gpurun_out/${tag}_$name.txt 2>&1 || exit 1
}
run c2 python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0
run c3 python bench.py --config c3 --steps 1 --warmup 0 --cpu-sample 0 --overlap 0 --c3-real 20000
run c5 python tools/bench_configs.py c5
grep -E "^==|duration|MFMA_BUSY|wait_inst|valu_busy|hbm_|TCC_HIT|TCC_MISS|LDS_BANK" gpurun_out/${tag}_c2.txt
}

exp_prof3() {
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
}

exp_psr() {
# Per-pulsar interpolation (FPTA_OPT_INTERP_PSR): its bitwise tests, the C3 and gridded suites, then C3 A/B against
# the two-kernel path.   bash tools/gpu_psr.sh <tag>
set -o pipefail
tag=${1:-PSR}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr" > ${o}_psr_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_psr_tests.log | head -20; tail -40 ${o}_psr_tests.log; exit 1; }
tail -1 ${o}_psr_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_grid.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_tests.log | head; tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "INTERP_PSR=0" || exit 1
}

exp_psr2() {
set -o pipefail
tag=${1:-PSR3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_c3.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr or gen_mix or pipelined or c3 or checksums" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "GEN_MIX=1" "INTERP_PSR=0" || exit 1
bash tools/gpu_c3_trace2.sh ${tag}T || exit 1
}

exp_psr3() {
set -o pipefail
tag=${1:-PSR5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_c3.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr or pipelined or c3 or checksums or warp_spec or partial_real" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "LIB=build/diag/lib_head.so" || exit 1
}

exp_psr4() {
set -o pipefail
tag=${1:-PSR6}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh ${tag} "" c3 "" "GEN_MIX=1" "LIB=build/diag/lib_nokeep.so" "LIB=build/diag/lib_nokeep.so GEN_MIX=1" "LIB=build/diag/lib_head.so" || exit 1
}

exp_psr5() {
set -o pipefail
tag=${1:-PSR7}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "psr or c4 or pipelined" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c4 "" "INTERP_PSR=0" || exit 1
}

exp_r03_base() {
# Round-3 starting point: GPU tests, smoke, bench C2/C3, configs, rocprof kernel stats of C2, C3 and C5.
#   bash tools/gpu_r03_base.sh <tag>
set -o pipefail
tag=${1:-r03a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > ${o}_gpu_tests.log 2>&1 || { tail -40 ${o}_gpu_tests.log; exit 1; }
tail -2 ${o}_gpu_tests.log
timeout -k 10 300 python -u bench.py --cpu-sample 0 > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
grep '^{' ${o}_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > ${o}_bench_c3.log 2>&1 || { tail -20 ${o}_bench_c3.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py c5 > ${o}_configs.jsonl 2>&1 || { tail -20 ${o}_configs.jsonl; exit 1; }
cut -c1-300 ${o}_configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c2 -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 > ${o}_prof_c2.log 2>&1 || { tail -20 ${o}_prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c3 -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 > ${o}_prof_c3.log 2>&1 || { tail -20 ${o}_prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof_c5 -o run -- python tools/bench_configs.py c5 > ${o}_prof_c5.log 2>&1 || { tail -20 ${o}_prof_c5.log; exit 1; }
find ${o}_prof_* -name "*kernel_stats.csv"
}

exp_r06() {
# One GPU call: the full GPU test suite, same-box A/B of the shipped library against a variant build on C5 and C2,
# then the round evidence pass (tools/gpu_full.sh without its tests).
#   bash tools/gpu_r06.sh <tag> <variant .so>
set -o pipefail
tag=${1:-r06}; var=${2:-build/diag/lib_oldbm.so}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh ${tag}b "test" c5 "" "LIB=$var" || exit 1
bash tools/gpu_ab_cfg.sh ${tag}c "" c2 "" "LIB=$var" || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}a_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}a_smoke.log; exit 1; }
SKIP_TESTS=1 bash tools/gpu_full.sh ${tag}a
}

exp_r4_check() {
# Round-4 validation in one GPU call: the full GPU suite on the product library, the diagnostic-kernel tests on the
# variant build (make variant NAME=diag DEFS=-DFPTA_DIAG_KERNELS), smoke, and the default bench.py line.
#   bash tools/gpu_r4_check.sh <tag>
set -o pipefail
tag=${1:-R4t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${o}_gpu_tests.log 2>&1 || { grep -E "FAILED|Error" ${o}_gpu_tests.log | head; tail -30 ${o}_gpu_tests.log; exit 1; }
tail -2 ${o}_gpu_tests.log
FAKEPTA_AMD_LIB=build/diag/lib_diag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "storer or union or interpolation_is_bitwise or partial_realization or lds or window_ring" > ${o}_diag_tests.log 2>&1 || { tail -30 ${o}_diag_tests.log; exit 1; }
tail -2 ${o}_diag_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
tail -3 ${o}_smoke.log
timeout -k 10 600 python -u bench.py > ${o}_bench.log 2>&1 || { tail -30 ${o}_bench.log; exit 1; }
tail -c 3000 ${o}_bench.log
}

exp_r5_c3_evidence() {
# C3 evidence at HEAD: rocprofv3 kernel statistics of bench.py --config c3, and per-dispatch PMC (one pass per counter
# group) of the C3 kernels (k_grid_interp_psr, k_gen_mix, partial reductions).   bash tools/gpu_r5_c3_evidence.sh <tag>
set -o pipefail
tag=${1:-R5f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
python tools/trace_steps.py ${o}_prof/run_kernel_trace.csv --marker k_part_final --last 20 > ${o}_steps.txt || exit 1
cat ${o}_steps.txt
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
bash tools/pmc_passes.sh ${o}_pmc_c3 "$P0" "$P1" "$P2" "$P3" "$P4" -- python bench.py --config c3 --steps 1 --warmup 1 --cpu-sample 0 --sub-configs 0 --overlap 0 || { echo "pmc failed"; tail -20 ${o}_pmc_c3/pass*.log; exit 1; }
python tools/pmc_dispatch.py ${o}_pmc_c3 --match interp,gen_mix,part > ${o}_pmc_dispatch_c3.txt 2>&1 || exit 1
head -60 ${o}_pmc_dispatch_c3.txt
}

exp_tests_sel() {
# Selected GPU tests (verbose log under gpurun_out/<tag>_tests.log).   bash tools/gpu_tests_sel.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -40
exit $rc
}

exp_wr() {
# Window-ring interpolation (FPTA_OPT_INTERP_WR): bitwise tests, then C2 A/B (on vs off) on one box.
set -o pipefail
tag=${1:-WR1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "window_ring" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|error" ${o}_tests.log | head -20; tail -40 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/gpu_ab_cfg.sh ${tag} "" c2 "" "INTERP_WR=1" || exit 1
}

exp_wr_pmc() {
set -o pipefail
tag=${1:-WRP}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
bash tools/pmc_passes.sh ${o}_pmc "$P0" "$P1" "$P2" "$P3" "$P4" -- python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0 --sub-configs 0 --opt INTERP_WR=1 || { echo "pmc failed"; tail -20 ${o}_pmc/pass*.log; exit 1; }
python tools/pmc_dispatch.py ${o}_pmc --match interp > ${o}_pmc_dispatch.txt 2>&1 || exit 1
cat ${o}_pmc_dispatch.txt
}

exp_ab_kernel_events() {
# (formerly tools/ab_kernel_events.sh)
# C2 step with / without the bench's per-kernel HIP timing events, pipelined (OVERLAP 1) and one-stream (OVERLAP 0)
# blocks, alternating, two repetitions; then kernel traces of the one-stream step with and without events.
set -o pipefail
tag=${1:-r5ev}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_grid.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused or gen_mix" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
out=gpurun_out/${tag}_ab.txt; : > $out
for rep in 1 2; do
  for ov in 1 0; do
    for ev in on off; do
      fl=""; [ $ev = off ] && fl="--no-kernel-events"
      timeout -k 10 120 python bench.py --cpu-sample 0 --sub-configs 0 --steps 50 --warmup 30 --overlap $ov $fl > gpurun_out/${tag}_o${ov}_$ev.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_o${ov}_$ev.json').read().strip().splitlines()[-1]); print('rep $rep overlap $ov events $ev', round(d['ms_per_step'],4), 'fused launch (events)', d['roofline'].get('avg_launch_ms'))" | tee -a $out
    done
  done
done
for ev in on off; do
  fl=""; [ $ev = off ] && fl="--no-kernel-events"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_tr0_$ev -o run -- python3 bench.py --cpu-sample 0 --sub-configs 0 --steps 20 --warmup 30 --overlap 0 $fl > gpurun_out/${tag}_tr0_$ev.log 2>&1 || exit 1
done
}

exp_ab_overlap_fused() {
# (formerly tools/ab_overlap_fused.sh)
# C2 (k_grid_fused): pipelined (OVERLAP 1, k_gen_mix of the next block on the side stream) vs one-stream (OVERLAP 0)
# blocks, alternating, four repetitions at W 30 / K 50 and at the driver's W 5 / K 20.
set -o pipefail
tag=${1:-r5ov}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt; : > $out
for wk in "30 50" "5 20"; do
  set -- $wk
  for rep in 1 2 3 4; do
    for ov in 1 0; do
      timeout -k 10 120 python bench.py --cpu-sample 0 --sub-configs 0 --warmup $1 --steps $2 --overlap $ov > gpurun_out/${tag}_o$ov.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_o$ov.json').read().strip().splitlines()[-1]); print('W $1 K $2 rep $rep overlap $ov', round(d['ms_per_step'],4), 'fused launch', round(d['roofline'].get('avg_launch_ms'),4))" | tee -a $out
    done
  done
done
}

exp_evidence() {
# (formerly tools/gpu_evidence.sh)
# Evidence at HEAD in one GPU call: rocprofv3 kernel statistics of the default bench command (C2), HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes) of the C2 interpolation, per-dispatch PMC of the C2 and C5 kernels (one stream).
#   bash tools/gpu_evidence.sh <tag> [traffic kernel]       (outputs under gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-R5e}; kern=${2:-k_grid_fused}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_prof -o run -- python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 --sub-configs 0 > ${o}_prof.log 2>&1 || { tail -20 ${o}_prof.log; exit 1; }
grep '^{' ${o}_prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d ${o}_traffic/pass$i -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 --sub-configs 0 > ${o}_traffic_$p.log 2>&1 || { tail -20 ${o}_traffic_$p.log; exit 1; }
  i=$((i+1))
done
python tools/collect_traffic.py ${o}_traffic ${o}_grid_traffic.json 320 200000 1024 $kern band32c || exit 1
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
run() {  # <name> <cmd...>
  local name=$1; shift
  bash tools/pmc_passes.sh ${o}_pmc_$name "$P0" "$P1" "$P2" "$P3" "$P4" -- "$@" || { echo "pmc $name failed"; tail -20 ${o}_pmc_$name/pass*.log; exit 1; }
  python tools/pmc_dispatch.py ${o}_pmc_$name > ${o}_pmc_dispatch_$name.txt 2>&1 || python tools/pmc_summary.py ${o}_pmc_$name > ${o}_pmc_dispatch_$name.txt 2>&1 || exit 1
}
run c2 python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0 --sub-configs 0
run c5 python tools/bench_configs.py c5
find ${o}_prof -name "*kernel_stats.csv"
}

exp_interp_variants() {
# (formerly tools/interp_variants.sh)
# NOTE (round 4): the FPTA_INTERP_DIAG cuts below were removed from the product source; this
# script reproduces the round-2/3 records only on a checkout of revision 059c9cc or earlier.
# Build (build) or time (run) compile-time variants of k_grid_interp_mfma: realization tiles per wave (RW),
# persistent workgroups per CU (WPC), diagnostic cuts (DIAG 1: grid loads from one L1-resident row; 2: no
# stores; 3: non-temporal stores; 4: no band loop, the store stream alone; 5: every other workgroup starts
# ~7 us late; 6: k_grid_interp_ws producers load nothing; 7: 1 and 2 together, the MFMA stream alone; 8: accumulators in AGPRs; 9: waves of a CU staggered by 0..7 x 3.4 us). WS selects FPTA_OPT_INTERP_WS values to time. VARIANTS entries are RW:WPC:DIAG. Throwaway libraries in build/diag, loaded by tools/interp_diag.py
# through FAKEPTA_AMD_LIB; never the product or the bench. Results: profiles/r02_interp_diag*.txt (a single
# operand set at 3 workgroups per CU measured 0.70 ms against 0.66 for the shipped 2-deep pipeline at 2).
S=fakepta_amd/csrc
D=build/diag
VARIANTS=${VARIANTS:-"8:2:0 8:2:2 8:2:4 8:2:6"}
if [ "$1" = build ]; then
  mkdir -p $D
  for v in $VARIANTS; do
    IFS=: read rw wpc dg <<< "$v"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result -ffp-contract=fast \
      -fno-gpu-rdc -DFPTA_INTERP_RW=$rw -DFPTA_INTERP_WPC=$wpc -DFPTA_INTERP_DIAG=$dg ${EXTRA:-} $S/kernels.hip $S/dense.hip $S/grid.hip \
      $S/grid_mfma.hip $S/capi.hip -o $D/lib_rw${rw}_wpc${wpc}_d${dg}.so &
  done
  wait
  exit 0
fi
set -o pipefail
for v in $VARIANTS; do
  IFS=: read rw wpc dg <<< "$v"
  for ws in ${WS:-0 1}; do
    FAKEPTA_AMD_LIB=$D/lib_rw${rw}_wpc${wpc}_d${dg}.so timeout -k 5 120 python tools/interp_diag.py --ws $ws --label "rw$rw-wpc$wpc-d$dg-ws$ws" || exit 1
  done
done
}

exp_fused_roles() {
# (formerly tools/gpu_fused_roles.sh)
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
}

exp_epoch_side_ab() {
# (formerly tools/gpu_epoch_side_ab.sh)
# C5: the ECORR epoch normals of pipelined blocks on a stream of their own (make variant NAME=zside
# DEFS=-DFPTA_EPOCH_SIDE=1) vs the shipped library; the white / ECORR GPU tests on the variant first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FAKEPTA_AMD_LIB=build/diag/lib_zside.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "white or ecorr or c5 or pipelined" > gpurun_out/R6v_tests.log 2>&1 || { tail -30 gpurun_out/R6v_tests.log; exit 1; }
tail -1 gpurun_out/R6v_tests.log
bash tools/gpu_ab_cfg.sh R6v "" c5 "" "LIB=build/diag/lib_zside.so" || exit 1
}

exp_c5_white_wpc_ab() {
# (formerly tools/gpu_c5_white_wpc_ab.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh R6t "" c5 "" "LIB=build/diag/lib_wwpc3.so" "LIB=build/diag/lib_wwpc4.so" || exit 1
}

exp_c4_half_ab() {
# (formerly tools/gpu_c4_half_ab.sh)
# C4: half-chunk bands forced (FPTA_OPT_INTERP_FUSED 3) vs the automatic choice (whole-chunk bands on C4); PMC of the
# C4 fused kernel at HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh R6w "" c4 "" "INTERP_FUSED=3" || exit 1
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
bash tools/pmc_passes.sh gpurun_out/R6w_pmc_c4 "$P0" "$P1" "$P2" -- python tools/bench_configs.py c4 || exit 1
python tools/pmc_dispatch.py gpurun_out/R6w_pmc_c4 > gpurun_out/R6w_pmc_dispatch_c4.txt 2>&1 || exit 1
echo done
}

exp_events_ab() {
# (formerly tools/gpu_events_ab.sh)
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
}

exp_next_mix_ab() {
# (formerly tools/gpu_next_mix_ab.sh)
# FPTA_OPT_FUSED_NEXT_MIX A/B on C2 (one box): the shipped library with the option on and off, and variant builds of
# FusedMix::min_left (make variant NAME=ml<v> DEFS=-DFPTA_FUSED_MIX_MIN_LEFT=<v>), each twice in turn; then kernel
# traces of on / off.
#   bash tools/gpu_next_mix_ab.sh <tag> [variant names...]
set -o pipefail
tag=${1:-R6h}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
timeout -k 10 420 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_next_mix.py tests/test_gpu_fused.py > ${o}_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --cpu-sample 0 --sub-configs 0"
for i in 1 2; do
  timeout -k 10 300 $B > ${o}_bench_on$i.log 2>&1 || exit 1
  timeout -k 10 300 $B --opt fused_next_mix=0 > ${o}_bench_off$i.log 2>&1 || exit 1
  for v in "$@"; do
    FAKEPTA_AMD_LIB=build/diag/lib_$v.so timeout -k 10 300 $B > ${o}_bench_${v}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d ${o}_tr_on -o run -- python bench.py --steps 10 --cpu-sample 0 --exact-launches 0 --sub-configs 0 > ${o}_tr_on.log 2>&1 || exit 1
echo done
}

exp_ab_prev_rev() {
# (formerly tools/gpu_ab_prev_rev.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh R6m "" c4 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6m "" c5 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6n "" c3 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6o "" c2 "" "LIB=build/diag/lib_r6f.so" || exit 1
}

exp_mix_early_ab() {
# (formerly tools/gpu_mix_early_ab.sh; the variant switch FPTA_FUSED_MIX_EARLY was removed)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FAKEPTA_AMD_LIB=build/diag/lib_early3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_next_mix.py > gpurun_out/R6bb_tests.log 2>&1 || { tail -20 gpurun_out/R6bb_tests.log; exit 1; }
tail -1 gpurun_out/R6bb_tests.log
bash tools/gpu_ab_cfg.sh R6bb "" c2 "" "LIB=build/diag/lib_early3.so" "LIB=build/diag/lib_early5.so" || exit 1
}

fn="exp_$1"
if ! declare -F "$fn" > /dev/null; then echo "unknown experiment: $fn" >&2; exit 2; fi
echo "# archived experiment (provenance only, not runnable: it may call removed scripts):" >&2
declare -f "$fn"
