# prefill MMQ tests, then pp512 with the XCD-aware tile order off / on
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out/xcd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "prefill or mul_mat_id or model" > gpurun_out/xcd/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/xcd/pytest.log; exit 1; }
tail -1 gpurun_out/xcd/pytest.log
for v in "GGML_MI355X_MMQ_XCD=0" "GGML_MI355X_MMQ_XCD=1" "GGML_MI355X_MMQ_XCD=0" "GGML_MI355X_MMQ_XCD=1"; do
  env $v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --pp 512 --no-cpu-baseline --roofline-steps 0 > gpurun_out/xcd/b.json 2> gpurun_out/xcd/b.err || { echo "bench rc=$?"; tail -20 gpurun_out/xcd/b.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/xcd/b.json'));print(sys.argv[1], 'tg', d['value'], 'pp', d['pp_tok_s'])" "$v"
done
