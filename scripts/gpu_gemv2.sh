set -o pipefail
for cfg in "GGML_MI355X_GEMV_WGS=512" "GGML_MI355X_GEMV_WGS=512 GGML_MI355X_GEMV_FAKE=1" "GGML_MI355X_GEMV_WGS=1024 GGML_MI355X_GEMV_FAKE=1"; do
env $cfg timeout -k 10 200 python scripts/gemv_bench.py > gpurun_out/gemv_run.txt 2>&1 || { cat gpurun_out/gemv_run.txt; exit 1; }
echo "== $cfg"; cat gpurun_out/gemv_run.txt
done
