# prefill round: parity of the prefill tiles (kernels, 512-token greedy, MoE), MMQ probe, FA prefill
# probe, the pp512 bench, and decode at depth 4096
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-prefill or prompt512 or moe or mul_mat_id or fused_and_graph}" > $OUT/pytest_pp.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_pp.log | head -30; tail -30 $OUT/pytest_pp.log; exit 1; }
tail -1 $OUT/pytest_pp.log
timeout -k 10 200 bash scripts/gpu_mmq_probe.sh 2>&1 | grep -v "mmq probe M=" | tee $OUT/mmq_probe.txt
timeout -k 10 120 python -u scripts/probe_fa_pf.py > $OUT/probe_fa_pf.txt 2>&1; cat $OUT/probe_fa_pf.txt
timeout -k 10 300 python bench.py --steps 32 --warmup 4 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/bench_pp.json 2> $OUT/bench_pp.err || { echo "bench rc=$?"; tail -20 $OUT/bench_pp.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_pp.json'));print('tg', d['value'], 'pp', d['pp_tok_s'])"
[ -n "$DEPTH" ] && { timeout -k 10 300 python bench.py --steps 16 --warmup 2 --pp 0 --depth 4096 --no-cpu-baseline --roofline-steps 4 --no-split-series > $OUT/bench_d4096.json 2> $OUT/bench_d4096.err && python3 -c "import json;d=json.load(open('$OUT/bench_d4096.json'));print('tg@4096', d['value'], 'fa us', d['roofline'].get('fattn_avg_us'))"; }
true
