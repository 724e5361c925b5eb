# one iteration on one box (round 6): the GPU tests selected by K (a pytest -k expression; none if
# unset), then interleaved tg A/B runs over VARIANTS (scripts/gpu_ab5.sh: ';'-separated env
# settings, "base" = none, MI355X_PLUGIN=<path> another build of the plugin)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=${OUT:-r06/iter}
mkdir -p gpurun_out/$OUT
if [ -n "$K" ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -x -q -rA --timeout 600 --timeout-method thread -k "$K" > gpurun_out/$OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" gpurun_out/$OUT/pytest.log | head; tail -5 gpurun_out/$OUT/pytest.log; exit 1; }
  grep -E "passed|failed" gpurun_out/$OUT/pytest.log | tail -1
fi
if [ -n "$VARIANTS" ]; then OUT=$OUT/ab bash scripts/gpu_ab5.sh || exit 1; fi
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || exit 1; fi
