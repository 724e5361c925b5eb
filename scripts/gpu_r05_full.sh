# the whole GPU suite (without the full-depth models), then the full-depth parity tests one by one
# (timed), then the Mixtral tg A/B of the MoE expert kernels and the 8B line on the same box
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread -k "not full_depth" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; tail -5 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
for t in ${FULL:-llama3_8b mixtral}; do
  s=$(date +%s)
  timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -q -rA --timeout 850 --timeout-method thread -k "full_depth and $t" > $OUT/pytest_full_$t.log 2>&1 || { echo "full $t rc=$?"; tail -15 $OUT/pytest_full_$t.log; exit 1; }
  echo "full_depth $t: $(tail -1 $OUT/pytest_full_$t.log) ($(( $(date +%s) - s )) s)"
done
if [ -n "$MIX" ]; then
  for v in "GGML_MI355X_MMID_OS=0" "GGML_MI355X_MMID_OS=1"; do
    env $v timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --pp 0 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/mix_$v.json 2> $OUT/mix_$v.err || { echo "mix bench rc=$?"; tail -5 $OUT/mix_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('mixtral', sys.argv[2], 'tg', round(d['value'],1))" $OUT/mix_$v.json $v
  done
fi
