# pp512 kernel-trace summary (scripts/pp_summary.py) of the default build
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/pptrace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --pp 512 --pp-reps 1 --no-cpu-baseline --roofline-steps 0 --no-split-series > $R/$OUT/pptrace_bench.json 2> $R/$OUT/pptrace_bench.err || { tail $R/$OUT/pptrace_bench.err; exit 1; }
cd $R
python3 scripts/pp_summary.py $(find $OUT/pptrace -name '*kernel_trace.csv' | head -1) > $OUT/pp512_kernels.txt
cp $(find $OUT/pptrace -name '*kernel_stats.csv' | head -1) $OUT/pp512_kernel_stats.csv
rm -rf $OUT/pptrace
cat $OUT/pp512_kernels.txt
