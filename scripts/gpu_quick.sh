# quick GPU check: model-level GPU tests, then graph vs eager decode bench (no profiler)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -q -rA -x -k "not backend_ops" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E 'FAILED|ERROR|passed|failed|max rel' gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for g in 0 1; do
GGML_MI355X_NO_GRAPH=$g timeout -k 10 300 python bench.py --steps 64 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_g$g.json 2> gpurun_out/bench_g$g.err || { tail gpurun_out/bench_g$g.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_g$g.json'));print('NO_GRAPH=$g', d['value'], d['ms_per_step'])"
done
