# one GPU iteration: full GPU test suite, then a rocprofv3 kernel-stats profile of a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -x "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E 'FAILED|ERROR|passed|failed|max rel' gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
bash scripts/gpu_prof.sh
