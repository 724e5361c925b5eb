set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k mul_mat > gpurun_out/pytest_gemv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gemv.log; [ $rc -eq 0 ] || exit $rc
for cfg in "RING=0" "RING=1 WGS=512" "RING=1 WGS=768" "RING=1 WGS=1024" "RING=0 PIPE=0"; do
env $(echo $cfg | sed 's/\([A-Z]*=\)/GGML_MI355X_GEMV_\1/g') timeout -k 10 200 python scripts/gemv_bench.py > gpurun_out/gemv_run.txt 2>&1 || { cat gpurun_out/gemv_run.txt; exit 1; }
echo "== $cfg"; cat gpurun_out/gemv_run.txt
done
