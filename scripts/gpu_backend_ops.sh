set -o pipefail
export GGML_BACKEND_PATH=$PWD/llamacog_amd/libggml-mi355x.so
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -E 'Marketing|gfx' | head -4 > gpurun_out/devinfo.txt
lscpu | head -20 >> gpurun_out/devinfo.txt
for op in MUL_MAT RMS_NORM ADD MUL SCALE SOFT_MAX ROPE CPY GET_ROWS SILU FLASH_ATTN_EXT; do
  timeout -k 10 240 refhost/build/test-backend-ops -b MI355X0 -o $op > gpurun_out/tbo_$op.log 2>&1
  rc=$?
  echo "$op rc=$rc $(grep -c 'OK' gpurun_out/tbo_$op.log) ok / $(grep -c 'FAIL' gpurun_out/tbo_$op.log) fail" | tee -a gpurun_out/tbo_summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after rc=$rc"; break; fi
done
