# prefill FA round: parity (flash-attention goldens incl. prefill rows, 512-token greedy, fused), probe, pp512
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flash_attn or prompt512 or fused_and_graph or backend_ops or greedy_tiny" > $OUT/pytest_fapf.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_fapf.log | head -30; tail -30 $OUT/pytest_fapf.log; exit 1; }
tail -1 $OUT/pytest_fapf.log
timeout -k 10 120 python -u scripts/probe_fa_pf.py > $OUT/probe_fa_pf.txt 2>&1; cat $OUT/probe_fa_pf.txt
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/bench_fapf.json 2> $OUT/bench_fapf.err || { echo "bench rc=$?"; tail -5 $OUT/bench_fapf.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_fapf.json'));print('pp', d['pp_tok_s'], 'tg', d['value'])"
done
