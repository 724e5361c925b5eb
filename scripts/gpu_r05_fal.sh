# long-context flash attention: parity (kernel oracle tests, 1536-position greedy) and the
# per-call times of the long pair vs the per-head kernels (scripts/probe_fal.py)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/fal}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py -k "flash_attn or depth1536" > $OUT/pytest_fa.log 2>&1 || { echo "fa tests rc=$?"; grep -E "FAILED|Error" $OUT/pytest_fa.log | head; tail -5 $OUT/pytest_fa.log; exit 1; }
tail -1 $OUT/pytest_fa.log
timeout -k 10 600 python scripts/probe_fal.py > $OUT/probe_fal.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_fal.txt; exit 1; }
grep -A7 "long pair" $OUT/probe_fal.txt
