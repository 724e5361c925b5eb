# the whole GPU suite (without the full-depth models), then the full-depth parity tests one by one
# (timed), then the Mixtral tg A/B of the MoE expert kernels and the 8B line on the same box
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread -k "${PYK:-not full_depth}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; tail -5 $OUT/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
for t in ${FULL:-llama3_8b mixtral}; do
  s=$(date +%s)
  timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -q -rA --timeout 850 --timeout-method thread -k "full_depth and $t" > $OUT/pytest_full_$t.log 2>&1 || { echo "full $t rc=$?"; tail -15 $OUT/pytest_full_$t.log; exit 1; }
  echo "full_depth $t: $(tail -1 $OUT/pytest_full_$t.log) ($(( $(date +%s) - s )) s)"
done
if [ -n "$MIX" ]; then
  # MIXV: ';'-separated env settings ("base" = none), e.g. MI355X_PLUGIN=build_ab/c2/libggml-mi355x.so
  IFS=';' read -ra MV <<< "${MIXV:-GGML_MI355X_MMID_OS=0;GGML_MI355X_MMID_OS=1}"
  for rep in $(seq 1 ${MIXREPS:-1}); do
  for v in "${MV[@]}"; do
    e=""; [ "$v" != "base" ] && e="$v"
    tag=$(echo "$v" | tr ' =/' '_-_' | cut -c1-60)
    env $e timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --pp 0 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/mix_${tag}_$rep.json 2> $OUT/mix_${tag}_$rep.err || { echo "mix bench rc=$?"; tail -5 $OUT/mix_${tag}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('mixtral', sys.argv[2], 'tg', round(d['value'],1))" $OUT/mix_${tag}_$rep.json "$v"
  done
  done
fi
if [ -n "${OPS:-}" ]; then
  timeout -k 10 400 python scripts/dbg_ops.py $OPS > $OUT/ops.txt 2>&1 || { echo "ops rc=$?"; tail -5 $OUT/ops.txt; exit 1; }
  grep -c "\[ops\]" $OUT/ops.txt
fi
