# decode FA (two heads per workgroup): parity, depth probe, in-graph timeline
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-flash_attn or greedy_tiny or greedy_llama3_8b_2layer or 70b_2layer_q4km}" > $OUT/pytest_fa2.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_fa2.log | head -30; tail -30 $OUT/pytest_fa2.log; exit 1; }
tail -2 $OUT/pytest_fa2.log
timeout -k 10 120 python -u scripts/probe_fa_depth.py 256:16 256:136 1024:1024 4096:4096 > $OUT/probe_fa2.txt 2>&1 && GGML_MI355X_FA_DEC2=0 timeout -k 10 120 python -u scripts/probe_fa_depth.py 256:16 256:136 1024:1024 4096:4096 >> $OUT/probe_fa2.txt 2>&1; cat $OUT/probe_fa2.txt | grep -v phases
VARIANTS="${VARIANTS:-base}" bash scripts/gpu_ktrace.sh
