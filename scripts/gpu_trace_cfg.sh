# kernel trace of a short decode run of $CFG (default mixtral-8x7b-q5km), per-token kernel summary
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
CFG=${CFG:-mixtral-8x7b-q5km}
mkdir -p $R/gpurun_out/trace_cfg
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_cfg/t -o run -- python3 $R/bench.py --config $CFG --steps 16 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/trace_cfg/bench.json 2> $R/gpurun_out/trace_cfg/bench.err || { tail $R/gpurun_out/trace_cfg/bench.err; exit 1; }
cd $R
python3 scripts/trace_summary.py $(find gpurun_out/trace_cfg/t -name '*kernel_trace.csv' | head -1) 4 > gpurun_out/trace_cfg/summary.txt
rm -rf gpurun_out/trace_cfg/t
head -40 gpurun_out/trace_cfg/summary.txt
