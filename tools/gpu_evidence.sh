#!/bin/bash
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
