# Round artefacts on one MI355X: the default bench line, the rocprofv3 kernel-trace summary of
# the same command, and a separate PMC pass (FETCH_SIZE) for the decode GEMV HBM traffic.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo "trace rc=$?"; tail -20 $OUT/trace_bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc -o run -- python3 bench.py --steps 16 --warmup 2 --pp 0 --no-cpu-baseline --roofline-steps 0 > $OUT/pmc_bench.json 2> $OUT/pmc_bench.err || { echo "pmc rc=$?"; tail -20 $OUT/pmc_bench.err; exit 1; }
ls $OUT/trace $OUT/pmc
