# decode at depth: in-graph timeline (FA scores / chain split) and bench lines for f16 and
# quantized KV caches at depth 4096
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r04}
mkdir -p $OUT
for kv in ${KVS:-f16 q8_0}; do
  timeout -k 10 300 python -u scripts/ktrace.py --tokens 8 --depth 4096 --kv $kv --csv $OUT/ktrace_d4096_$kv.csv > $OUT/ktrace_d4096_$kv.txt 2>&1 || { echo "ktrace $kv rc=$?"; tail -20 $OUT/ktrace_d4096_$kv.txt; exit 1; }
  echo "== ktrace depth 4096 kv $kv"; cat $OUT/ktrace_d4096_$kv.txt
  timeout -k 10 300 python bench.py --steps 16 --warmup 2 --pp 0 --depth 4096 --kv $kv --no-cpu-baseline --roofline-steps 4 --no-split-series > $OUT/bench_d4096_$kv.json 2> $OUT/bench_d4096_$kv.err || { echo "bench rc=$?"; tail -20 $OUT/bench_d4096_$kv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_d4096_$kv.json'));print('tg@4096 kv=$kv', d['value'], 'ms', d['ms_per_step'], 'fa us', d['roofline'].get('fattn_avg_us'))"
done
