# in-graph kernel timeline of 8B decode (scripts/ktrace.py) for the default build and variants
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r03}
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
for v in "${VS[@]}"; do
  e=""; [ "$v" != "base" ] && e="$v"
  tag=$(echo "$v" | tr ' =' '_-')
  env $e timeout -k 10 300 python -u scripts/ktrace.py --tokens ${TOK:-16} --depth ${DEPTH:-0} --csv $OUT/ktrace_$tag.csv > $OUT/ktrace_$tag.txt 2>&1 || { echo "ktrace $v rc=$?"; tail -20 $OUT/ktrace_$tag.txt; exit 1; }
  echo "== $v"; cat $OUT/ktrace_$tag.txt
done
