# one GPU session: pytest -m gpu, smoke, bench (+ rocprofv3 kernel stats of a short bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
grep -E 'FAILED|passed|failed|max rel' gpurun_out/pytest_gpu.log | head -20
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
