# Round 6 lines on one MI355X: the default bench line (8B tg128 + pp512, roofline, cpu_baseline,
# the 70B split series at N = 1), the Mixtral line, and the metric's own driver (refhost
# llama-bench with the plugin) on the 8B and on Mixtral.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r06/bench}
M=${LLAMACOG_MODEL_DIR:-/tmp/llamacog_amd_models}
mkdir -p $OUT
(rocm-smi --showclocks --showpower --showperflevel > $OUT/devinfo.txt 2>&1 || true)
if [ -z "$SKIP8B" ]; then
  timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('8b tg', d['value'], 'pp', d.get('pp_tok_s'), 'split', d.get('step_split_ms'), 'roof', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
  rm -f $M/llama3-70b*.gguf
  GGML_BACKEND_PATH=$R/llamacog_amd/libggml-mi355x.so timeout -k 10 400 refhost/build/llama-bench -m $M/llama3-8b-q4km-s0.gguf -p 512 -n 128 -ngl 99 -fa 1 -r 3 -o json > $OUT/llama_bench_8b.json 2> $OUT/llama_bench_8b.err || { echo "llama-bench 8b rc=$?"; tail -20 $OUT/llama_bench_8b.err; exit 1; }
  python3 -c "import json;[print('llama-bench 8b', r['n_prompt'], r['n_gen'], round(r['avg_ts'],1), '+-', round(r['stddev_ts'],1)) for r in json.load(open('$OUT/llama_bench_8b.json'))]"
fi
timeout -k 10 900 python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --no-cpu-baseline --no-split-series --roofline-steps 8 > $OUT/bench_mixtral.json 2> $OUT/bench_mixtral.err || { echo "mixtral rc=$?"; tail -20 $OUT/bench_mixtral.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_mixtral.json'));print('mixtral tg', d['value'], 'pp', d.get('pp_tok_s'), 'frac', d.get('model_bw_frac_of_8TBs'), 'traffic', d['roofline'].get('traffic'))"
GGML_BACKEND_PATH=$R/llamacog_amd/libggml-mi355x.so timeout -k 10 600 refhost/build/llama-bench -m $M/mixtral-8x7b-q5km-s0.gguf -p 512 -n 128 -ngl 99 -fa 1 -r 3 -o json > $OUT/llama_bench_mixtral.json 2> $OUT/llama_bench_mixtral.err || { echo "llama-bench mixtral rc=$?"; tail -20 $OUT/llama_bench_mixtral.err; exit 1; }
python3 -c "import json;[print('llama-bench mixtral', r['n_prompt'], r['n_gen'], round(r['avg_ts'],1), '+-', round(r['stddev_ts'],1)) for r in json.load(open('$OUT/llama_bench_mixtral.json'))]"
