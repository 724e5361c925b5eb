# FA change check: kernel tests (FA parity), FA phase profile, model tests, short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "fattn or flash or fa_" > gpurun_out/pytest_fa.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_fa.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/pytest_fa.log | head -30; exit $rc; }
timeout -k 10 200 python scripts/fa_prof.py > gpurun_out/fa_prof.log 2>&1 || { tail gpurun_out/fa_prof.log; exit 1; }
cat gpurun_out/fa_prof.log
bash scripts/gpu_check.sh
