# round 4: mat-vec (engine on) + flash-attention kernel parity, quantized-KV depth greedy runs,
# then the engine and long-context FA microbenchmarks
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
GGML_MI355X_GEMV_ENG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "(mul_mat and not prefill and not mul_mat_id) or flash_attn" > gpurun_out/pytest_r04b_k.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r04b_k.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r04b_k.log | head -20; exit $rc; }
timeout -k 10 400 python -u scripts/probe_fal.py 2>&1 | tee gpurun_out/probe_fal.txt || exit 1
timeout -k 10 400 python -u scripts/probe_eng.py 2>&1 | tee gpurun_out/probe_eng.txt || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "depth1536" > gpurun_out/pytest_r04b_m.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_r04b_m.log; exit $rc
