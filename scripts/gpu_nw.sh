# prefill Q4_K tile, 4 vs 8 waves: parity with 8 forced, the MMQ probe and pp512 for both
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
GGML_MI355X_MMQ_NW=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "prefill or prompt512" > $OUT/pytest_nw8.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_nw8.log | head -30; tail -30 $OUT/pytest_nw8.log; exit 1; }
tail -1 $OUT/pytest_nw8.log
VARIANTS="base;GGML_MI355X_MMQ_NW=8;base;GGML_MI355X_MMQ_NW=8" timeout -k 10 300 bash scripts/gpu_mmq_probe.sh 2>&1 | grep -v "mmq probe M=" | tee $OUT/mmq_probe_nw.txt
for v in base GGML_MI355X_MMQ_NW=8 base GGML_MI355X_MMQ_NW=8; do
  e=""; [ "$v" != "base" ] && e="$v"
  env $e timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/bench_nw.json 2> $OUT/bench_nw.err || { echo "bench rc=$?"; tail -5 $OUT/bench_nw.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/bench_nw.json'));print(sys.argv[1], 'pp', d['pp_tok_s'], 'tg', d['value'])" "$v"
done
