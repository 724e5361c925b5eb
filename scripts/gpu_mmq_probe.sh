# prefill MUL_MAT kernel times on the 8B shapes under MMQ knob settings (VARIANTS ';'-separated)
set -o pipefail
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
for v in "${VS[@]}"; do
  e=""; [ "$v" != "base" ] && e="$v"
  env $e timeout -k 10 120 python3 scripts/probe_mmq.py || exit 1
done
