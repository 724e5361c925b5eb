# one-shot GEMV: parity first (kernels + model greedy), then the geometry probe and the in-graph timeline
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-mul_mat or greedy_tiny or greedy_llama3_8b_2layer_q4km or fused_and_graph or 70b_2layer_q4km}" > $OUT/pytest_os.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_os.log | head -30; tail -30 $OUT/pytest_os.log; exit 1; }
tail -2 $OUT/pytest_os.log
timeout -k 10 120 python scripts/probe_geom.py > $OUT/probe_geom_os.txt 2>&1 && GGML_MI355X_GEMV_OS=0 timeout -k 10 120 python scripts/probe_geom.py >> $OUT/probe_geom_os.txt 2>&1; cat $OUT/probe_geom_os.txt
VARIANTS="${VARIANTS:-base}" bash scripts/gpu_ktrace.sh
