# the whole GPU suite (full-depth 8B / Mixtral / 70B included) and smoke() on one box
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r06/tests}
mkdir -p $OUT
(rocm-smi --showclocks --showpower --showperflevel > $OUT/devinfo.txt 2>&1 || true)
(df -h /tmp >> $OUT/devinfo.txt 2>&1 || true)
timeout -k 10 1080 python -u -m pytest tests -m gpu -q -rA --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; tail -5 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
timeout -k 10 100 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
