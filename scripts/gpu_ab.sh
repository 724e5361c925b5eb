# A/B of one plugin switch: model bit-identity with the switch on, then decode tg off/on/off/on
# and the in-graph kernel timeline off/on.   VAR=GGML_MI355X_ROUTER1 ON=1 OFF=0 bash scripts/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
VAR=${VAR:?switch name}
ON=${ON:-1}
OFF=${OFF:-0}
K=${TESTK:-greedy_tiny_q4km or greedy_llama3_8b_2layer_q4km or fused_and_graph or 70b_2layer_q4km or depth1536 or graph_replay_survives}
env $VAR=$ON timeout -k 10 700 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "$K" > gpurun_out/pytest_ab.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_ab.log | tail -20; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_ab.log | head -20; exit $rc; }
for v in $OFF $ON $OFF $ON; do
  env $VAR=$v timeout -k 10 300 python bench.py --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 8 > gpurun_out/bench_ab$v.json 2> gpurun_out/bench_ab$v.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_ab$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/bench_ab$v.json'));print('$VAR=$v tg', d['value'], 'ms', d['ms_per_step'], 'split', d['step_split_ms'])"
done
for v in $OFF $ON; do
  echo "== $VAR=$v"
  env $VAR=$v timeout -k 10 300 python -u scripts/ktrace.py --tokens 8 --csv gpurun_out/ktrace_ab$v.csv 2>&1 | tail -12 || exit 1
done
