set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/probe_mall.py > gpurun_out/probe_mall.txt 2>&1; rc=$?
cat gpurun_out/probe_mall.txt
exit $rc
