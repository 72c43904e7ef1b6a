#!/bin/bash
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
