set -o pipefail
for v in 0 1; do
GGML_MI355X_NO_MMQ=$v timeout -k 10 300 python bench.py --steps 16 --warmup 4 --pp 512 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_pp$v.json 2> gpurun_out/bench_pp$v.err || { tail gpurun_out/bench_pp$v.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_pp$v.json'));print('NO_MMQ=$v pp512', d['pp_tok_s'], 'tg', d['value'])"
done
