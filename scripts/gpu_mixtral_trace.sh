# Mixtral-8x7B Q5_K_M (BASELINE configs[4]) decode: rocprofv3 --kernel-trace --stats of a
# decode-only bench run (eager: graph replay is off under the tracer), per decode token
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r04mx}
mkdir -p $OUT
# create the GGUF outside the traced run
timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --steps 4 --warmup 1 --pp 0 --no-cpu-baseline --no-split-series --roofline-steps 0 > $OUT/prep.json 2> $OUT/prep.err || { echo "prep rc=$?"; tail -20 $OUT/prep.err; exit 1; }
cd /tmp
W=2; K=16; RF=8
NTOK=$((W + K + 4 + K + 4 + RF))
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/bench.py --config mixtral-8x7b-q5km --steps $K --warmup $W --roofline-steps $RF --pp 0 --no-cpu-baseline --no-split-series > $R/$OUT/trace_bench.json 2> $R/$OUT/trace_bench.err || { echo "trace rc=$?"; tail -20 $R/$OUT/trace_bench.err; exit 1; }
cd $R
python3 scripts/kstats.py $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $NTOK > $OUT/mixtral_kernel_stats_summary.txt
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $OUT/mixtral_kernel_stats.csv
rm -rf $OUT/trace
head -30 $OUT/mixtral_kernel_stats_summary.txt
