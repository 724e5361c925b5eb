#!/bin/bash
# kernel durations of the GEMV probe and the lab under rocprofv3 (kernel trace only)
set -o pipefail
mkdir -p gpurun_out/r03/prof_probe gpurun_out/r03/prof_lab
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/prof_probe -o probe -- python3 -u scripts/probe_geom.py > gpurun_out/r03/prof_probe/out.txt 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/prof_lab -o lab -- tools/bin/gemv_lab_exact > gpurun_out/r03/prof_lab/out.txt 2>&1
rc=$?
find gpurun_out/r03/prof_probe gpurun_out/r03/prof_lab -name "*.csv" | head
exit $rc
