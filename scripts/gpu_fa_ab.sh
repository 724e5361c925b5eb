set -o pipefail
O=/root/repo/llamacog_amd/libggml-mi355x-old.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "flash or FLASH or greedy or fused" > gpurun_out/pytest_fa.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" gpurun_out/pytest_fa.log | head -20; tail -20 gpurun_out/pytest_fa.log; exit 1; }
tail -1 gpurun_out/pytest_fa.log
timeout -k 10 200 python -u scripts/probe_fa_depth.py 136 4096 > gpurun_out/probe_new.txt 2>&1 && cat gpurun_out/probe_new.txt
MI355X_PLUGIN=$O timeout -k 10 200 python -u scripts/probe_fa_depth.py 136 4096 > gpurun_out/probe_old.txt 2>&1 && cat gpurun_out/probe_old.txt
NOTEST=1 VARIANTS="base;MI355X_PLUGIN=$O;base;MI355X_PLUGIN=$O" bash scripts/gpu_iter.sh
