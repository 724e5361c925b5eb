set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bw_sweep.py > gpurun_out/bw.txt 2>&1 || { cat gpurun_out/bw.txt; exit 1; }
cat gpurun_out/bw.txt
for w in 512; do
GGML_MI355X_GEMV_WGS=$w timeout -k 10 200 python scripts/gemv_bench.py > gpurun_out/gemv_w$w.txt 2>&1 || { cat gpurun_out/gemv_w$w.txt; exit 1; }
echo "== WGS=$w"; cat gpurun_out/gemv_w$w.txt
done
