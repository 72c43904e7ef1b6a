#!/bin/bash
# Gridded tests, then the interpolation kernels alone and pipelined (tools/interp_diag.py), then the C2 and C3 benches.
mkdir -p gpurun_out
o=gpurun_out/${1:-q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > ${o}_tests.log 2>&1 || { tail -30 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for ws in 0 1; do for ov in 0 1; do
  timeout -k 5 120 python tools/interp_diag.py --ws $ws --overlap $ov --label "ws$ws-ov$ov" >> ${o}_diag.log 2>&1 || { tail ${o}_diag.log; exit 1; }
done; done
python -c "
import json
for l in open('${o}_diag.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['label'], round(d['interp_ms'],4), round(d['dft_ms'],4), round(d['step_ms'],4))
"
for ws in 0 1; do
  timeout -k 10 200 python -u bench.py --cpu-sample 0 --exact-launches 3 --interp-ws $ws > ${o}_c2_ws$ws.log 2>&1 || { tail ${o}_c2_ws$ws.log; exit 1; }
  timeout -k 10 200 python -u bench.py --config c3 --steps 5 --cpu-sample 0 --interp-ws $ws > ${o}_c3_ws$ws.log 2>&1 || { tail ${o}_c3_ws$ws.log; exit 1; }
done
for f in ${o}_c2_ws0 ${o}_c2_ws1 ${o}_c3_ws0 ${o}_c3_ws1; do grep "^{" $f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['avg_launch_ms'],4), r.get('isolated',{}).get('avg_launch_ms'))"; done
