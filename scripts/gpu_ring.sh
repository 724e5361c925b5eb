# ring GEMV round: decode parity (kernels + model greedy, ring on), tg A/B over variants, timeline, MMQ probe
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-mul_mat or greedy_tiny_q4km or greedy_llama3_8b or fused_and_graph or 70b_2layer_q4km}" > $OUT/pytest_ring.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_ring.log | head -30; tail -30 $OUT/pytest_ring.log; exit 1; }
tail -2 $OUT/pytest_ring.log
IFS=';' read -ra VS <<< "${VARIANTS:-base;GGML_MI355X_GEMV_RING=0;GGML_MI355X_GEMV_RING=2;GGML_MI355X_TAILS=1;base}"
for v in "${VS[@]}"; do
  e=""; [ "$v" != "base" ] && e="$v"
  env $e timeout -k 10 300 python bench.py --pp ${PP:-0} --no-cpu-baseline --roofline-steps 8 --no-split-series > $OUT/bench_v.json 2> $OUT/bench_v.err || { echo "bench $v rc=$?"; tail -20 $OUT/bench_v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/bench_v.json'));print(sys.argv[1], 'tg', d['value'], 'ms', d['ms_per_step'], 'pp', d.get('pp_tok_s'), 'gemv', d['roofline']['achieved'], d['roofline']['avg_launch_us'])" "$v"
done
VARIANTS="${KVARIANTS:-base}" bash scripts/gpu_ktrace.sh
[ -n "$MMQ" ] && { timeout -k 10 200 bash scripts/gpu_mmq_probe.sh 2>&1 | grep -v "mmq probe M=" | tee $OUT/mmq_probe.txt; }
true
