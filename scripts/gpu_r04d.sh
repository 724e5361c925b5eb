# round 4: model parity with the engine (norm + SwiGLU prologues), then tg A/B engine off/on
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
GGML_MI355X_GEMV_ENG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "greedy_tiny_q4km or greedy_tiny_q8_0 or greedy_llama3_8b_2layer_q4km or fused_and_graph or 70b_2layer_q4km or mixtral or graph_replay_survives" \
    > gpurun_out/pytest_r04d.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_r04d.log | tail -20; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_r04d.log | head -20; exit $rc; }
for v in 0 1 0 1; do
  GGML_MI355X_GEMV_ENG=$v timeout -k 10 300 python bench.py --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 8 > gpurun_out/bench_e$v.json 2> gpurun_out/bench_e$v.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_e$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/bench_e$v.json'));print('ENG=$v tg', d['value'], 'ms', d['ms_per_step'], 'split', d['step_split_ms'], 'gemv', d['roofline']['achieved'], d['roofline']['avg_launch_us'])"
done
