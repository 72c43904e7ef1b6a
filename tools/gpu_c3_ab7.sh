#!/bin/bash
# C3: checksum / pipelining tests, the A/B of the deferred ev_gfree record, and the timeline with it
set -o pipefail
tag=${1:-R5u}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh $tag "c3 or checksum or rccl or multi or pipelined or coalesced or psr" c3 "" "LIB=build/diag/lib_early.so" && bash tools/gpu_c3_trace3.sh ${tag}T
