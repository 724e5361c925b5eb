# GPU iteration: kernel + model tests (no test-backend-ops sweep), graph vs eager bench, profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -rA -x -k "not backend_ops" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E 'FAILED|ERROR|passed|failed|max rel' gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
GGML_MI355X_NO_GRAPH=1 timeout -k 10 300 python bench.py --steps 32 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_nograph.json 2> gpurun_out/bench_nograph.err || { echo "nograph bench failed"; tail -20 gpurun_out/bench_nograph.err; exit 1; }
echo "no-graph:"; cat gpurun_out/bench_nograph.json
bash scripts/gpu_prof.sh
