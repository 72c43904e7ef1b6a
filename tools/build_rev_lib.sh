#!/bin/bash
# Build the library of an earlier git revision as a same-box A/B baseline (tools/gpu_ab_cfg.sh "LIB=<out>"), e.g. the
# previous normal map: bash tools/build_rev_lib.sh a0c8a10^ build/diag/lib_oldbm.so  (profiles/round4/R4w, R4x);
# round 3's HEAD: bash tools/build_rev_lib.sh 059c9cc build/diag/lib_r3.so  (R4q, R4r, R4s). Runs here (no GPU).
set -e -o pipefail
rev=$1; out=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" fakepta_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$(dirname "$root/$out")"
make -C "$tmp/fakepta_amd/csrc" -j8 > /dev/null  # the revision's own source list and flags
cp "$tmp/fakepta_amd/lib/libfakepta_amd.so" "$root/$out"
rm -rf "$tmp"
echo "$out <- $rev"
