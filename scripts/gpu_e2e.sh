# end-to-end on the GPU box: smoke (tiny model, GPU vs CPU greedy) then the 8B bench
set -o pipefail
mkdir -p gpurun_out
df -h /tmp | tail -1 > gpurun_out/e2e_env.txt
nproc >> gpurun_out/e2e_env.txt
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 1200 python bench.py --verbose "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -40 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
