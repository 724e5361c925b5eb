# Mixtral decode in-graph timeline (scripts/ktrace.py) with the router's phase stamps
# (GGML_MI355X_KTRACE_RAW=moe_router), for the tree's plugin and a baseline build
# (BASE=build_ab/<c>/libggml-mi355x.so), on one box
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/router}
mkdir -p $OUT
for v in new ${BASE:+base}; do
  e=""; [ "$v" = base ] && e="MI355X_PLUGIN=$BASE"
  env $e GGML_MI355X_KTRACE_RAW=moe_router timeout -k 10 600 python -u scripts/ktrace.py --config mixtral-8x7b-q5km --tokens ${TOK:-8} --csv $OUT/ktrace_$v.csv > $OUT/ktrace_$v.txt 2>&1 || { echo "ktrace $v rc=$?"; tail -20 $OUT/ktrace_$v.txt; exit 1; }
  echo "== $v"; grep -v ktraw $OUT/ktrace_$v.txt | tail -9
  python3 - $OUT/ktrace_$v.txt <<'PY'
import sys, numpy as np
rows = [list(map(float, l.split(":")[1].split())) for l in open(sys.argv[1]) if l.startswith("[ktraw] moe_router")]
a = np.array(rows)
print("router stamps (median over", len(a), "launches):", " ".join(f"{x:.2f}" for x in np.median(a, axis=0)))
PY
done
