# one box: GPU tests (subset $TESTK), then tg bench (+ pp when PP>0), optional kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/trace
[ -n "$NOTEST" ] || timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
[ -n "$NOTEST" ] || tail -2 gpurun_out/pytest_gpu.log
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
for v in "${VS[@]}"; do
  e=""; [ "$v" != "base" ] && e="$v"
  env $e timeout -k 10 300 python bench.py --pp ${PP:-0} --no-cpu-baseline --roofline-steps 8 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/bench.json'));print(sys.argv[1], 'tg', d['value'], 'ms', d['ms_per_step'], 'pp', d['pp_tok_s'], 'gemv', d['roofline']['achieved'], d['roofline']['avg_launch_us'], 'fa', d['roofline']['fattn_avg_us'])" "$v"
done
[ -n "$PROBE" ] && { timeout -k 10 120 python -u scripts/probe_fa.py 2>&1 | tee gpurun_out/probe_fa.txt || exit 1; }
if [ -n "$TRACE" ]; then
cd /tmp
env $TRACEENV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace/t -o run -- python3 $R/bench.py --steps 16 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/trace/bench.json 2> $R/gpurun_out/trace/bench.err || { tail $R/gpurun_out/trace/bench.err; exit 1; }
cd $R
python3 scripts/trace_summary.py $(find gpurun_out/trace/t -name '*kernel_trace.csv' | head -1) 4 > gpurun_out/trace/summary.txt
rm -rf gpurun_out/trace/t
head -24 gpurun_out/trace/summary.txt
fi
