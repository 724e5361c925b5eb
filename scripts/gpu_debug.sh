set -o pipefail
mkdir -p gpurun_out
export GGML_BACKEND_PATH=$PWD/llamacog_amd/libggml-mi355x.so
for op in FLASH_ATTN_EXT SOFT_MAX SILU MUL_MAT ROPE; do
  timeout -k 10 240 refhost/build/test-backend-ops -b MI355X0 -o $op > gpurun_out/tbo_$op.log 2>&1
  rc=$?; echo "$op rc=$rc $(grep -c 'OK' gpurun_out/tbo_$op.log) ok / $(grep -c 'FAIL' gpurun_out/tbo_$op.log) fail"
  [ $rc -gt 1 ] && exit 1
done
unset GGML_BACKEND_PATH
timeout -k 10 300 python scripts/diff_nodes.py tiny-q4km 8 1 > gpurun_out/diff_fa1.txt 2>&1; echo "rc=$?"
grep -E '<<<|logits|nodes' gpurun_out/diff_fa1.txt | head -30
timeout -k 10 300 python scripts/diff_nodes.py tiny-q4km 8 0 > gpurun_out/diff_fa0.txt 2>&1; echo "rc=$?"
grep -E '<<<|logits|nodes' gpurun_out/diff_fa0.txt | head -30
