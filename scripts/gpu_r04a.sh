# round 4, first engine call: mat-vec parity subset, then the engine / one-shot microbenchmark
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
GGML_MI355X_GEMV_ENG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "${TESTK:-mul_mat and not prefill and not mul_mat_id}" > gpurun_out/pytest_r04a.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_r04a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/probe_eng.py 2>&1 | tee gpurun_out/probe_eng.txt
