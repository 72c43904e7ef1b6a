set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh R6t "" c5 "" "LIB=build/diag/lib_wwpc3.so" "LIB=build/diag/lib_wwpc4.so" || exit 1
