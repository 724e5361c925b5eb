# interleaved tg A/B on one box: REPS rounds over VARIANTS (';'-separated env settings, "base" =
# none; MI355X_PLUGIN=<path> selects another build of the plugin)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/ab}
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    e=""; [ "$v" != "base" ] && e="$v"
    tag=$(echo "$v" | tr ' =/' '_-_' | cut -c1-60)
    env $e timeout -k 10 240 python bench.py --pp ${PP:-0} --no-cpu-baseline --roofline-steps ${RF:-0} --no-split-series ${BARGS:-} > $OUT/b_${tag}_$rep.json 2> $OUT/b_${tag}_$rep.err || { echo "bench $v rc=$?"; tail -5 $OUT/b_${tag}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[3], sys.argv[2], 'tg', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'pp', d.get('pp_tok_s'))" $OUT/b_${tag}_$rep.json "$v" $rep
  done
done
