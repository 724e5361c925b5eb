# the reference's own drivers on one MI355X (BASELINE.json configs[0]):
#   * tests/test_refhost_drivers.py (llama-bench / llama-cli with the plugin via GGML_BACKEND_PATH);
#   * refhost llama-bench -p 512 -n 128 -ngl 99 -fa 1 on the Llama-3-8B Q4_K_M synthetic GGUF;
#   * config 1: stories15M Q8_0 on ggml-cpu through llama-bench (no plugin);
#   * tg at KV depth 4096 (bench.py --depth 4096).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r02}
mkdir -p $OUT
M=/tmp/llamacog_amd_models
timeout -k 10 300 python -u -m pytest tests/test_refhost_drivers.py -q -m gpu --timeout 200 --timeout-method thread > $OUT/refhost_tests.log 2>&1 || { tail -30 $OUT/refhost_tests.log; exit 1; }
tail -2 $OUT/refhost_tests.log
python3 -c "from llamacog_amd import gguf_synth as g; g.ensure('llama3-8b-q4km', '$M/llama3-8b-q4km-s0.gguf', seed=0); g.ensure('stories15m-q8_0', '$M/stories15m-q8_0-s0.gguf', seed=0)"
GGML_BACKEND_PATH=$R/llamacog_amd/libggml-mi355x.so timeout -k 10 400 refhost/build/llama-bench -m $M/llama3-8b-q4km-s0.gguf -p 512 -n 128 -ngl 99 -fa 1 -r 3 -o md > $OUT/llama_bench_plugin_8b.md 2> $OUT/llama_bench_plugin_8b.err || { tail -20 $OUT/llama_bench_plugin_8b.err; exit 1; }
cat $OUT/llama_bench_plugin_8b.md
timeout -k 10 300 refhost/build/llama-bench -m $M/stories15m-q8_0-s0.gguf -p 512 -n 128 -r 5 -t ${OMP_NUM_THREADS:-16} -o md > $OUT/llama_bench_stories15m_cpu.md 2> $OUT/llama_bench_stories15m_cpu.err || { tail -20 $OUT/llama_bench_stories15m_cpu.err; exit 1; }
cat $OUT/llama_bench_stories15m_cpu.md
timeout -k 10 600 python bench.py --depth 4096 --steps 32 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 8 > $OUT/bench_depth4096.json 2> $OUT/bench_depth4096.err || { tail -20 $OUT/bench_depth4096.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_depth4096.json')); print('depth4096 exact FA', d['value'], d['roofline']['fattn_avg_us'], d['step_split_ms'])"
