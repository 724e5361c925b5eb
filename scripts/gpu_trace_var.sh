# kernel traces of short decode runs, one per variant of $VARIANTS (';'-separated env settings,
# "base" = none), config $CFG (default: bench.py's); per-token kernel summary of each
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/trace_var
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
k=0
for v in "${VS[@]}"; do
  e=""; [ "$v" != "base" ] && e="$v"
  cd /tmp
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_var/t$k -o run -- python3 $R/bench.py ${CFG:+--config $CFG} --steps 16 --warmup 4 --pp 0 --no-cpu-baseline --roofline-steps 0 > $R/gpurun_out/trace_var/bench$k.json 2> $R/gpurun_out/trace_var/bench$k.err || { tail $R/gpurun_out/trace_var/bench$k.err; exit 1; }
  cd $R
  python3 scripts/trace_summary.py $(find gpurun_out/trace_var/t$k -name '*kernel_trace.csv' | head -1) 4 > gpurun_out/trace_var/summary$k.txt
  rm -rf gpurun_out/trace_var/t$k
  echo "== $v"; head -${NL:-12} gpurun_out/trace_var/summary$k.txt
  k=$((k+1))
done
