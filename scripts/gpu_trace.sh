# kernel trace of a short decode run (no graphs under the tracer), summarised per token
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace/t -o run -- python3 $R/bench.py --steps 32 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/trace/bench.json 2> $R/gpurun_out/trace/bench.err || { tail $R/gpurun_out/trace/bench.err; exit 1; }
cat $R/gpurun_out/trace/bench.json
