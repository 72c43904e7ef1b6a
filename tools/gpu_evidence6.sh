#!/bin/bash
# Evidence at HEAD for every BASELINE config's dominant kernel in one GPU call (round 6):
#  * rocprofv3 kernel statistics of C2 (bench.py), C3 (bench.py --config c3), C4 and C5 (tools/bench_configs.py);
#  * HBM traffic (FETCH_SIZE / WRITE_SIZE passes, each its own run) of each config's dominant kernel ->
#    <tag>_<cfg>_traffic.json (tools/collect_traffic.py: FETCH_SIZE doubled per MI355X_MICROARCH.md);
#  * per-dispatch PMC of the C2 and C5 dominant kernels (one stream).
#   bash tools/gpu_evidence6.sh <tag>          (outputs under gpurun_out/<tag>_*)
set -o pipefail
tag=${1:-R6e}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/$tag
C2="python bench.py --steps 20 --cpu-sample 0 --exact-launches 0 --sub-configs 0"
C2S="python bench.py --steps 5 --warmup 2 --cpu-sample 0 --exact-launches 0 --sub-configs 0"
C3="python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --exact-launches 0 --sub-configs 0"
C4="python tools/bench_configs.py c4"
C5="python tools/bench_configs.py c5"
for cfg in c2 c3 c4 c5; do
  case $cfg in c2) cmd=$C2 ;; c3) cmd=$C3 ;; c4) cmd=$C4 ;; c5) cmd=$C5 ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${o}_${cfg}_prof -o run -- $cmd > ${o}_${cfg}_prof.log 2>&1 || { tail -20 ${o}_${cfg}_prof.log; exit 1; }
  echo "kernel stats $cfg done"
done
# traffic: one counter per run; the shapes and kernels collect_traffic.py matches
traffic() {  # <cfg> <K> <n_toa> <n_real> <kernel> [layout] -- <cmd...>
  local cfg=$1 K=$2 n=$3 R=$4 kern=$5 lay=$6; shift 6; shift
  local i=0
  for p in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d ${o}_${cfg}_traffic/pass$i -o run -- "$@" > ${o}_${cfg}_traffic_$p.log 2>&1 || { tail -20 ${o}_${cfg}_traffic_$p.log; return 1; }
    i=$((i+1))
  done
  python tools/collect_traffic.py ${o}_${cfg}_traffic ${o}_${cfg}_traffic.json $K $n $R "$kern" $lay
}
traffic c2 320 200000 1024 "k_grid_fused<8, false, true, true>" band32c -- $C2S || exit 1
traffic c3 60 200000 7168 "k_grid_interp_psr<true, 4>" "" -- $C3 || exit 1
traffic c4 200 10000000 256 "k_grid_fused<8, false, false, false>" "" -- $C4 || exit 1
traffic c5 640 200000 1024 "k_grid_interp_mfma<true, false, 8>" "" -- $C5 || exit 1
P0="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
run() {  # <name> <cmd...>
  local name=$1; shift
  bash tools/pmc_passes.sh ${o}_pmc_$name "$P0" "$P1" "$P2" -- "$@" || { echo "pmc $name failed"; tail -20 ${o}_pmc_$name/pass*.log; exit 1; }
  python tools/pmc_dispatch.py ${o}_pmc_$name > ${o}_pmc_dispatch_$name.txt 2>&1 || python tools/pmc_summary.py ${o}_pmc_$name > ${o}_pmc_dispatch_$name.txt 2>&1 || exit 1
}
run c2 python bench.py --steps 4 --warmup 2 --cpu-sample 0 --exact-launches 0 --overlap 0 --sub-configs 0
run c5 python tools/bench_configs.py c5
find gpurun_out -path "*${tag}_*" -name "*kernel_stats.csv"
