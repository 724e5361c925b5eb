# round 4: in-graph kernel timeline, engine off / on
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
for v in 0 1; do
  echo "== GGML_MI355X_GEMV_ENG=$v"
  GGML_MI355X_GEMV_ENG=$v timeout -k 10 300 python -u scripts/ktrace.py --tokens 8 --csv gpurun_out/ktrace_e$v.csv 2>&1 | tail -12 || exit 1
done
