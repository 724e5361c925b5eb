# validate HEAD on one MI355X: gpu tests, default bench line, kernel trace of a short decode run
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/trace
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace/t -o run -- python3 $R/bench.py --steps 32 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/trace/bench.json 2> $R/gpurun_out/trace/bench.err || { tail $R/gpurun_out/trace/bench.err; exit 1; }
cd $R
python3 scripts/trace_summary.py $(find gpurun_out/trace/t -name '*kernel_trace.csv' | head -1) 4 > gpurun_out/trace/summary.txt
cat gpurun_out/trace/summary.txt | head -40
