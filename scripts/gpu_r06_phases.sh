# in-kernel phase stamps of the one-shot GEMV launches (a MI_KT_PHASE=1 build in build_ab/phase) and
# the in-graph timeline of the product build, 8B decode
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r06/phases}
mkdir -p $OUT
timeout -k 10 200 python scripts/ktrace.py ${KARGS:-} > $OUT/ktrace.txt 2>&1 || exit 1
for L in ${LABELS:-"gemv+pro+epi" "gemv2+pro+epi" "gemv" "gemv+resid/w" "gemv/w"}; do
  t=$(echo "$L" | tr '+/' '__')
  MI355X_PLUGIN=${PLUG:-build_ab/phase}/libggml-mi355x.so GGML_MI355X_KTRACE_RAW="$L" timeout -k 10 200 python scripts/ktrace.py ${KARGS:-} > $OUT/ktrace_phase_$t.txt 2> $OUT/ktrace_phase_$t.err || exit 1
  python scripts/ktrace_phases.py $OUT/ktrace_phase_$t.err "$L" > $OUT/phases_$t.txt
done
cat $OUT/ktrace.txt $OUT/phases_*.txt
