# kernel trace of a pp512 bench run split into runs (hbm calibration, pp64 warm, pp512, tg)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ppr/t -o run -- python3 $R/bench.py --steps 2 --warmup 1 --pp 512 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/ppr/bench.json 2> $R/gpurun_out/ppr/bench.err || { tail $R/gpurun_out/ppr/bench.err; exit 1; }
cd $R
python3 scripts/pp_breakdown.py $(find gpurun_out/ppr/t -name '*kernel_trace.csv' | head -1) > gpurun_out/ppr/runs.txt
rm -rf gpurun_out/ppr/t
cat gpurun_out/ppr/runs.txt
