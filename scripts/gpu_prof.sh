# rocprofv3 kernel trace + stats of a short decode bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 32 --warmup 8 --pp 0 --no-cpu-baseline --roofline-steps 4 "$@" > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { echo "rc=$?"; tail -20 gpurun_out/prof/bench.err; exit 1; }
find gpurun_out/prof -name '*kernel_stats*' | head
cat gpurun_out/prof/bench.json
