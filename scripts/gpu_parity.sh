# parity iteration on one MI355X: kernel tests then model tests (all reported, not -x)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_gpu_kernels.py -q -rf --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/pytest_kernels.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_kernels.log
[ $rc -gt 1 ] && { echo "kernel tests rc=$rc"; tail -30 gpurun_out/pytest_kernels.log; exit 1; }
[ -n "$NOMODEL" ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -q -rf --timeout 300 --timeout-method thread ${MODELK:+-k "$MODELK"} > gpurun_out/pytest_model.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_model.log
exit 0
