# Round 6 per-model evidence on one MI355X: for the 8B and for Mixtral, a
# rocprofv3 --pmc FETCH_SIZE pass over decode (profiles/r06/pmc/pmc_traffic_<config>.json, the file
# bench.py reads for its line's roofline.traffic) and rocprofv3 --kernel-trace --stats kernel splits
# of decode and of pp512.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r06/pmc}
mkdir -p $OUT
for C in ${CONFIGS:-llama3-8b-q4km mixtral-8x7b-q5km}; do
  python3 -c "from llamacog_amd import gguf_synth as g; g.ensure('$C')" > /dev/null || exit 1
  cd /tmp
  # decode-only traced run: W + K timed + (4 + K) split + (4 + R) roofline single-token decodes
  W=2; K=16; RF=4
  NTOK=$((W + K + 4 + K + 4 + RF))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/tr_$C -o run -- python3 $R/bench.py --config $C --steps $K --warmup $W --roofline-steps $RF --pp 0 --no-cpu-baseline --no-split-series > $R/$OUT/trace_$C.json 2> $R/$OUT/trace_$C.err || { echo "trace $C rc=$?"; tail -5 $R/$OUT/trace_$C.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/pp_$C -o run -- python3 $R/bench.py --config $C --steps 1 --warmup 0 --roofline-steps 0 --pp 512 --pp-reps 2 --no-cpu-baseline --no-split-series > $R/$OUT/pptrace_$C.json 2> $R/$OUT/pptrace_$C.err || { echo "pptrace $C rc=$?"; tail -5 $R/$OUT/pptrace_$C.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT/pmc_$C -o run -- python3 $R/bench.py --config $C --steps 8 --warmup 2 --pp 0 --no-cpu-baseline --roofline-steps 0 --no-split-series > $R/$OUT/pmc_$C.json 2> $R/$OUT/pmc_$C.err || { echo "pmc $C rc=$?"; tail -5 $R/$OUT/pmc_$C.err; exit 1; }
  cd $R
  python3 scripts/kstats.py $(find $OUT/tr_$C -name '*kernel_stats.csv' | head -1) $NTOK > $OUT/decode_kernels_$C.txt
  python3 scripts/kstats.py $(find $OUT/pp_$C -name '*kernel_stats.csv' | head -1) 1 > $OUT/pp512_kernels_$C.txt
  python3 scripts/pmc_traffic.py $(find $OUT/pmc_$C -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic_$C.json > /dev/null
  rm -rf $OUT/tr_$C $OUT/pp_$C $OUT/pmc_$C
  head -12 $OUT/decode_kernels_$C.txt
  python3 -c "import json;d=json.load(open('$OUT/pmc_traffic_$C.json'));print('$C gemv bytes/launch', d['gemv_bytes_per_launch'], 'launches', d['gemv_launches'])"
done
