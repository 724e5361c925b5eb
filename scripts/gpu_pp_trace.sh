# pp512 kernel breakdown: rocprofv3 kernel-trace stats of a prefill-heavy bench run (+ optional probe)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out/pp
[ -n "$PROBE" ] && { timeout -k 10 60 ./tools/bin/mfma_probe | tee gpurun_out/pp/mfma_probe.txt || exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp/t -o run -- python3 $R/bench.py --steps 2 --warmup 1 --pp 512 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/pp/bench.json 2> $R/gpurun_out/pp/bench.err || { tail $R/gpurun_out/pp/bench.err; exit 1; }
cd $R
f=$(find gpurun_out/pp/t -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(f\"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):7d} calls {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:110]}\")
" | tee gpurun_out/pp/stats.txt
rm -rf gpurun_out/pp/t
