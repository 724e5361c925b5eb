# decode FA round: parity (kernel goldens, model greedy incl. depth 1536), the depth phase probe, tg at 4096
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-flash_attn or depth1536 or greedy_llama3_8b_2layer_q4km or greedy_tiny or fused_and_graph}" > $OUT/pytest_fa.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_fa.log | head -30; tail -30 $OUT/pytest_fa.log; exit 1; }
tail -1 $OUT/pytest_fa.log
timeout -k 10 200 python -u scripts/probe_fa_depth.py 256:136 4096:4096 > $OUT/probe_fa_depth.txt 2>&1; cat $OUT/probe_fa_depth.txt
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --pp 0 --depth 4096 --no-cpu-baseline --roofline-steps 4 --no-split-series > $OUT/bench_d4096.json 2> $OUT/bench_d4096.err && python3 -c "import json;d=json.load(open('$OUT/bench_d4096.json'));print('tg@4096', d['value'], 'fa us', d['roofline'].get('fattn_avg_us'))"
timeout -k 10 300 python bench.py --steps 64 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 4 --no-split-series > $OUT/bench_tg.json 2> $OUT/bench_tg.err && python3 -c "import json;d=json.load(open('$OUT/bench_tg.json'));print('tg', d['value'], 'fa us', d['roofline'].get('fattn_avg_us'))"
