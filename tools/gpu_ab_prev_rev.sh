set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_cfg.sh R6m "" c4 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6m "" c5 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6n "" c3 "" "LIB=build/diag/lib_r6f.so" || exit 1
bash tools/gpu_ab_cfg.sh R6o "" c2 "" "LIB=build/diag/lib_r6f.so" || exit 1
