set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out/fav
GGML_MI355X_FA_PREFILL_CH=128 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flash_attn or model" > gpurun_out/fav/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/fav/pytest.log; exit 1; }
tail -1 gpurun_out/fav/pytest.log
for v in "X=1" "GGML_MI355X_FA_PREFILL_CH=128" "GGML_MI355X_FA_PREFILL_CH=128 GGML_MI355X_FA_PREFILL_OCC=3" "GGML_MI355X_FA_PREFILL_CH=128 GGML_MI355X_FA_PREFILL_OCC=4"; do
  env $v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --pp 512 --no-cpu-baseline --roofline-steps 0 > gpurun_out/fav/b.json 2> gpurun_out/fav/b.err || { echo "bench rc=$?"; tail -20 gpurun_out/fav/b.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/fav/b.json'));print(sys.argv[1], 'tg', d['value'], 'pp', d['pp_tok_s'])" "$v"
done
