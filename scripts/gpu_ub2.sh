set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ub2
timeout -k 10 120 ./tools/bin/ubench2 > gpurun_out/ub2/plain.txt 2>&1 && cat gpurun_out/ub2/plain.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ub2 -o ub -- ./tools/bin/ubench2 > gpurun_out/ub2/prof.txt 2>&1 && \
python3 scripts/kstats.py gpurun_out/ub2/ub_kernel_stats.csv
