#!/bin/bash
# probe_geom.py once per environment variant (VARIANTS="a=1 b=2;c=3", "base" = defaults)
set -o pipefail
mkdir -p gpurun_out/r03
OUT=${OUT:-gpurun_out/r03/probe.txt}
: > $OUT
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
for v in "${VS[@]}"; do
  if [ "$v" = base ]; then env_args=(); else read -ra env_args <<< "$v"; fi
  timeout -k 10 120 env "${env_args[@]}" python3 -u scripts/probe_geom.py >> $OUT 2>&1 || { echo "FAILED: $v" >> $OUT; exit 1; }
done
cat $OUT
