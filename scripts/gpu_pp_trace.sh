# prefill (pp512) kernel breakdown: rocprofv3 kernel-trace --stats of a pp-only bench run
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp/t -o run -- python3 $R/bench.py --steps 1 --warmup 1 --pp 512 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/pp/bench.json 2> $R/gpurun_out/pp/bench.err || { tail $R/gpurun_out/pp/bench.err; exit 1; }
cd $R
python3 scripts/kstats.py $(find gpurun_out/pp/t -name '*kernel_stats.csv' | head -1) > gpurun_out/pp/summary.txt
rm -rf gpurun_out/pp/t
head -25 gpurun_out/pp/summary.txt
