# MoE router in registers: MoE parity / fused-graph tests, Mixtral tg, decode trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r04rt}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "mul_mat_id or moe or mixtral or bit_identical or argsort or soft_max" > $OUT/pytest_moe.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $OUT/pytest_moe.log | head -20; tail -5 $OUT/pytest_moe.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_moe.log | tail -1
timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --no-cpu-baseline --no-split-series --roofline-steps 8 > $OUT/bench_mixtral.json 2> $OUT/bench_mixtral.err || { echo "bench rc=$?"; tail -20 $OUT/bench_mixtral.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_mixtral.json'));print('mixtral', d['value'], 'pp', d.get('pp_tok_s'), 'frac', d.get('model_bw_frac_of_8TBs'))"
OUT=${OUT#gpurun_out/} bash scripts/gpu_mixtral_trace.sh > /dev/null && head -8 $OUT/mixtral_kernel_stats_summary.txt
