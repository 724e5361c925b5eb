# round 3, first pass: the mixlo rounding probe, the new config-4 / virtual-device / concurrency
# tests, then the tg + pp bench with a kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/r03
timeout -k 10 60 tools/bin/ubench_mixlo > gpurun_out/r03/mixlo.txt 2>&1; cat gpurun_out/r03/mixlo.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-70b or virtual or concurrent or stage_handoff}" > gpurun_out/r03/pytest_new.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_new.log | head -30; tail -30 gpurun_out/r03/pytest_new.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/r03/pytest_new.log | tail -20
NOTEST=1 PP=512 TRACE=1 bash scripts/gpu_iter.sh
