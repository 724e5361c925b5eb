# prefill tile round: parity of the prefill mat-muls (kernel goldens, 512-token greedy, MoE), MMQ probe, pp512
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -k "prefill or prompt512 or moe or mul_mat_id" > $OUT/pytest_mmq.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" $OUT/pytest_mmq.log | head -30; tail -30 $OUT/pytest_mmq.log; exit 1; }
tail -1 $OUT/pytest_mmq.log
VARIANTS="base;base" timeout -k 10 300 bash scripts/gpu_mmq_probe.sh 2>&1 | grep -v "mmq probe M=" | tee $OUT/mmq_probe.txt
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --roofline-steps 0 --no-split-series > $OUT/bench_mmq.json 2> $OUT/bench_mmq.err || { echo "bench rc=$?"; tail -5 $OUT/bench_mmq.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_mmq.json'));print('pp', d['pp_tok_s'], 'tg', d['value'])"
done
