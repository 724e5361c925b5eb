set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "mul_mat or gemv" > gpurun_out/pytest_gemv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gemv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/gemv_bench.py > gpurun_out/gemv_run.txt 2>&1 || { cat gpurun_out/gemv_run.txt; exit 1; }
cat gpurun_out/gemv_run.txt
