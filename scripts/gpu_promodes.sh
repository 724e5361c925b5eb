set -o pipefail
mkdir -p gpurun_out
for m in 0 1 2 3; do
GGML_MI355X_NO_PROLOGUE=$m timeout -k 10 300 python bench.py --steps 64 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_p$m.json 2> gpurun_out/bench_p$m.err || { tail gpurun_out/bench_p$m.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_p$m.json'));print('NO_PROLOGUE=$m', d['value'], d['ms_per_step'])"
done
