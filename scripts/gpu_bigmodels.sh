# configs 5 and 4 on one MI355X: Mixtral-8x7B Q5_K_M (MUL_MAT_ID decode + batched routing) and
# Llama-3-70B Q4_K_M (fits one 288 GB GPU; the N>1 layer split runs in the driver's multi-GPU
# bench), synthetic GGUFs written on the box.  Lines go to gpurun_out/$OUT (default r02).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r02}
mkdir -p $OUT
df -h /tmp | tail -1
timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --no-cpu-baseline --roofline-steps 8 > $OUT/bench_mixtral.json 2> $OUT/bench_mixtral.err || { echo "mixtral rc=$?"; tail -20 $OUT/bench_mixtral.err; exit 1; }
cat $OUT/bench_mixtral.json
rm -f /tmp/llamacog_amd_models/mixtral-8x7b-q5km-s0.gguf
timeout -k 10 900 python bench.py --config llama3-70b-q4km --steps 64 --warmup 4 --no-cpu-baseline --roofline-steps 8 > $OUT/bench_70b.json 2> $OUT/bench_70b.err || { echo "70b rc=$?"; tail -20 $OUT/bench_70b.err; exit 1; }
cat $OUT/bench_70b.json
