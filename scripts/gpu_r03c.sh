# parity of the decode path (kernels + model greedy incl. 70B shapes, virtual-device splits), then the timeline
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 600 --timeout-method thread -k "${TESTK:-mul_mat or greedy or fused_and_graph or flash_attn}" > $OUT/pytest_c.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_c.log | head -30; tail -30 $OUT/pytest_c.log; exit 1; }
tail -2 $OUT/pytest_c.log
VARIANTS="${VARIANTS:-base}" bash scripts/gpu_ktrace.sh
