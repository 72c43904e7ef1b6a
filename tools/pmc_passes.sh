#!/bin/bash
# rocprofv3 PMC passes (one run per counter group) over a command, on the GPU box.
#   tools/pmc_passes.sh <outdir> "<counters pass 0>" ["<counters pass 1>" ...] -- <cmd...>
# Each pass stays within gfx950's per-block limits (8 SQ, 4 TCC, 4 TCP, 2 TA/TD/GRBM); no trace domains.
set -o pipefail
out=$1; shift
passes=()
while [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
i=0
for p in "${passes[@]}"; do
  timeout -k 10 120 rocprofv3 --pmc $p --output-format csv -d "$out/pass$i" -o run -- "$@" > "$out/pass$i.log" 2>&1 || exit $?
  i=$((i+1))
done
