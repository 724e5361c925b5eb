set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bin/ubench > gpurun_out/ubench.txt 2>&1; rc=$?; cat gpurun_out/ubench.txt; [ $rc -eq 0 ] || exit $rc
for g in 0 1; do
GGML_MI355X_NO_GRAPH=$g timeout -k 10 300 python bench.py --steps 64 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_g$g.json 2> gpurun_out/bench_g$g.err || { tail gpurun_out/bench_g$g.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_g$g.json'));print('NO_GRAPH=$g', d['value'], d['ms_per_step'])"
done
