# GPU check after a kernel change: kernel + model parity tests, op microbenchmarks, a short
# decode bench (no profiler)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -q -rA -x -k "not backend_ops" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E 'FAILED|ERROR|passed|failed|max rel' gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python scripts/op_bench.py > gpurun_out/op_bench.log 2>&1 || { tail gpurun_out/op_bench.log; exit 1; }
cat gpurun_out/op_bench.log
timeout -k 10 300 python bench.py --steps 128 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 32 > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail gpurun_out/bench_q.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_q.json'));print('tg', d['value'], d['ms_per_step'], 'gemv', d['roofline']['achieved'], d['roofline']['avg_launch_us'], 'fa us', d['roofline']['fattn_avg_us'])"
