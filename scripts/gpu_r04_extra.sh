# round 4 evidence beside gpu_final.sh: decode at depth 4096 (f16 / q8_0 KV: timeline + bench
# lines), the default in-graph timeline, the pp512 per-kernel summary, tg128 with a q8_0 KV cache
# and the Mixtral line
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=${OUT:-r04}
OUT=$OUT bash scripts/gpu_depth.sh || exit 1
VARIANTS=base OUT=$OUT bash scripts/gpu_ktrace.sh || exit 1
OUT=$OUT bash scripts/gpu_pptrace.sh || exit 1
timeout -k 10 400 python -u scripts/probe_fal.py > gpurun_out/$OUT/probe_fal.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --kv q8_0 --steps 128 --warmup 8 --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 8 > gpurun_out/$OUT/bench_kv_q8_0.json 2> gpurun_out/$OUT/bench_kv_q8_0.err || { echo "kv q8_0 rc=$?"; tail -20 gpurun_out/$OUT/bench_kv_q8_0.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$OUT/bench_kv_q8_0.json'));print('tg128 kv q8_0', d['value'], 'fa us', d['roofline'].get('fattn_avg_us'))"
# the 70B GGUF (42 GB) from gpu_final.sh's split series leaves no room on the box's disk for Mixtral's 32 GB
rm -f ${LLAMACOG_MODEL_DIR:-/tmp/llamacog_amd_models}/llama3-70b*.gguf; df -h /tmp | tail -1
timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --no-cpu-baseline --no-split-series --roofline-steps 8 > gpurun_out/$OUT/bench_mixtral.json 2> gpurun_out/$OUT/bench_mixtral.err || { echo "mixtral rc=$?"; tail -20 gpurun_out/$OUT/bench_mixtral.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$OUT/bench_mixtral.json'));print('mixtral tg', d['value'], 'pp', d.get('pp_tok_s'), 'frac', d.get('model_bw_frac_of_8TBs'))"
