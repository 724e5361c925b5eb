# MoE check: GPU tests (MUL_MAT_ID / MoE model / fused-vs-unfused), 8B tg, Mixtral tg + pp512
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/big
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "mul_mat_id or moe or fused_and_graph or tiny_q4km or argsort or graph_runs" > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --pp 0 --no-cpu-baseline --roofline-steps 8 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));print('8b tg', d['value'], d['step_split_ms'])"
timeout -k 10 900 python bench.py --config mixtral-8x7b-q5km --steps 32 --warmup 4 --no-cpu-baseline --roofline-steps 8 > gpurun_out/big/bench_mixtral.json 2> gpurun_out/big/bench_mixtral.err || { echo "mixtral rc=$?"; tail -20 gpurun_out/big/bench_mixtral.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/big/bench_mixtral.json'));print('mixtral tg', d['value'], 'pp', d['pp_tok_s'], 'gemv', d['roofline']['achieved'], d['step_split_ms'])"
