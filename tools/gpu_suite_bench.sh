#!/bin/bash
# Whole GPU suite, then C2 (3 runs) and C3 (2 runs) benches.   bash tools/gpu_suite_bench.sh <tag>
mkdir -p gpurun_out
o=gpurun_out/${1:-sb}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > ${o}_tests.log 2>&1 || { tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 3 > ${o}_c2_$rep.log 2>&1 || { tail ${o}_c2_$rep.log; exit 1; }
done
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 > ${o}_c3_$rep.log 2>&1 || { tail ${o}_c3_$rep.log; exit 1; }
done
for f in ${o}_c2_1 ${o}_c2_2 ${o}_c2_3 ${o}_c3_1 ${o}_c3_2; do grep "^{" $f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['avg_launch_ms'],4), r.get('isolated',{}).get('avg_launch_ms'), r['grid'].get('band_rows_per_chunk'), (d.get('pcie_inclusive') or {}).get('samples_per_s'))"; done
