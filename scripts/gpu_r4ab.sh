# rows per wave of the four-wave (K = 14336) one-shot launches: A/B on Mixtral and Llama-3-8B tg
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r04r4}
mkdir -p $OUT
M="python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 8"
L="python bench.py --steps 128 --warmup 8 --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 8"
for i in 1 2; do
for v in 0 1 2; do
GGML_MI355X_OS_R4=$v timeout -k 10 400 $M > $OUT/mx_$v.json 2> $OUT/mx_$v.err || { echo "mx $v rc=$?"; tail -5 $OUT/mx_$v.err; exit 1; }
GGML_MI355X_OS_R4=$v timeout -k 10 400 $L > $OUT/l8_$v.json 2> $OUT/l8_$v.err || { echo "l8 $v rc=$?"; tail -5 $OUT/l8_$v.err; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/mx_$v.json'));b=json.load(open('$OUT/l8_$v.json'));print('pass $i R4=$v mixtral', a['value'], 'llama8b', b['value'])"
done
done
