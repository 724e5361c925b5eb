# round-end evidence on the final tree: the decode-FA parity subset first (stops on a failure),
# then the full GPU suite, smoke, the default bench line, rocprof stats + FETCH_SIZE pass, the
# in-graph timeline, the pp512 per-kernel summary, the depth-4096 line and the FA depth probe
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=${OUT:-r03g}
OUT=$OUT bash scripts/gpu_fa.sh && OUT=$OUT bash scripts/gpu_final.sh && VARIANTS=base OUT=$OUT bash scripts/gpu_ktrace.sh && OUT=$OUT bash scripts/gpu_pptrace.sh
