set -o pipefail
mkdir -p gpurun_out
for cfg in "PIPE=1" "PIPE=0" "PIPE=0 LDS=1"; do
env $(echo $cfg | sed 's/\([A-Z]*=\)/GGML_MI355X_GEMV_\1/g') timeout -k 10 200 python scripts/gemv_bench.py > gpurun_out/gemv_run.txt 2>&1 || { cat gpurun_out/gemv_run.txt; exit 1; }
echo "== $cfg"; cat gpurun_out/gemv_run.txt
done
