set -o pipefail
mkdir -p gpurun_out
for g in 0 1; do
GGML_MI355X_NO_GRAPH=$g timeout -k 10 300 python scripts/gpu_hostsplit.py > gpurun_out/split_g$g.txt 2>&1 || { tail gpurun_out/split_g$g.txt; exit 1; }
echo "NO_GRAPH=$g"; cat gpurun_out/split_g$g.txt
done
