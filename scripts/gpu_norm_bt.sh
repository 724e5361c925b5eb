# fused-norm threads per row: tests under BT=256, then tg for BT = 1024 / 512 / 256
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out/nbt
GGML_MI355X_NORM_BT=256 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "norm or model" > gpurun_out/nbt/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/nbt/pytest.log; exit 1; }
tail -1 gpurun_out/nbt/pytest.log
for v in "X=1" "GGML_MI355X_NORM_BT=512" "GGML_MI355X_NORM_BT=256" "X=1" "GGML_MI355X_NORM_BT=512" "GGML_MI355X_NORM_BT=256"; do
  env $v timeout -k 10 300 python bench.py --steps 64 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > gpurun_out/nbt/b.json 2> gpurun_out/nbt/b.err || { echo "bench rc=$?"; tail -20 gpurun_out/nbt/b.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/nbt/b.json'));print(sys.argv[1], 'tg', d['value'])" "$v"
done
