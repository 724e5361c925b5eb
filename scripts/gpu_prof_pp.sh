set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/profpp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profpp -o run -- python3 bench.py --steps 2 --warmup 1 --pp 512 --no-cpu-baseline --roofline-steps 0 > gpurun_out/profpp/bench.json 2> gpurun_out/profpp/bench.err || { echo "rc=$?"; tail -20 gpurun_out/profpp/bench.err; exit 1; }
cat gpurun_out/profpp/bench.json
