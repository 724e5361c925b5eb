set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
for e in "X=1" "GGML_MI355X_GEMV_WGS4=0" "GGML_MI355X_GEMV_WGS4=1024" "GGML_MI355X_GEMV_R4W=1" "X=1"; do
  env $e timeout -k 10 120 python scripts/probe_geom.py || exit 1
done
