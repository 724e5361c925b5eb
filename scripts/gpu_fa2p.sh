set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out/r03
for v in 0; do echo "== dbg $v"; GGML_MI355X_FA_DBG=$v timeout -k 10 120 python -u scripts/probe_fa_depth.py 256:16 256:136 1024:1024 4096:4096 2>&1 || exit 1; done > gpurun_out/r03/probe_fa2p.txt 2>&1; rc=$?; cat gpurun_out/r03/probe_fa2p.txt; exit $rc
