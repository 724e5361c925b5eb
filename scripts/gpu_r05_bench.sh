# Round artefacts on one MI355X (the tests and smoke: gpu_r05_tests.sh): the default bench line, the rocprofv3
# kernel-trace --stats of the same command, and a separate PMC pass (FETCH_SIZE) for the GEMV traffic.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r02}
mkdir -p $OUT
# the box's clocks and power (boxes differ by up to ~30 % in decode tok/s)
(rocm-smi --showclocks --showpower --showmaxpower --showperflevel > $OUT/devinfo.txt 2>&1 || true)
(df -h /tmp >> $OUT/devinfo.txt 2>&1 || true)
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
# decode-only traced run: W + K timed + (4 + K) split + (4 + R) roofline single-token decodes
W=4; K=32; RF=8
NTOK=$((W + K + 4 + K + 4 + RF))
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/bench.py --steps $K --warmup $W --roofline-steps $RF --pp 0 --no-cpu-baseline --no-split-series > $R/$OUT/trace_bench.json 2> $R/$OUT/trace_bench.err || { echo "trace rc=$?"; tail -20 $R/$OUT/trace_bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT/pmc -o run -- python3 $R/bench.py --steps 16 --warmup 2 --pp 0 --no-cpu-baseline --roofline-steps 0 --no-split-series > $R/$OUT/pmc_bench.json 2> $R/$OUT/pmc_bench.err || { echo "pmc rc=$?"; tail -20 $R/$OUT/pmc_bench.err; exit 1; }
cd $R
python3 scripts/kstats.py $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $NTOK > $OUT/kernel_stats_summary.txt
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
python3 scripts/pmc_traffic.py $(find $OUT/pmc -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic.json > /dev/null
rm -rf $OUT/trace $OUT/pmc
head -20 $OUT/kernel_stats_summary.txt
# the Mixtral line (BASELINE configs[4]) on the same box
rm -f ${LLAMACOG_MODEL_DIR:-/tmp/llamacog_amd_models}/llama3-70b*.gguf
timeout -k 10 600 python bench.py --config mixtral-8x7b-q5km --steps 64 --warmup 4 --no-cpu-baseline --no-split-series --roofline-steps 8 > $OUT/bench_mixtral.json 2> $OUT/bench_mixtral.err || { echo "mixtral rc=$?"; tail -20 $OUT/bench_mixtral.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_mixtral.json'));print('mixtral tg', d['value'], 'pp', d.get('pp_tok_s'), 'frac', d.get('model_bw_frac_of_8TBs'))"
