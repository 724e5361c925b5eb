# tg/pp sweep of launch-geometry knobs (no tests): VARIANTS="A=1;B=2 C=3"
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out/knobs
IFS=';' read -ra VS <<< "${VARIANTS:-X=1}"
for v in "${VS[@]}"; do
  env $v timeout -k 10 300 python bench.py --steps 64 --warmup 4 --pp ${PP:-0} --no-cpu-baseline --roofline-steps 0 > gpurun_out/knobs/b.json 2> gpurun_out/knobs/b.err || { echo "bench rc=$?"; tail -20 gpurun_out/knobs/b.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/knobs/b.json'));print(sys.argv[1], 'tg', d['value'], 'pp', d['pp_tok_s'])" "$v"
done
