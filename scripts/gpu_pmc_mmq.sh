# SQ counters of the prefill MMQ kernels (one --pmc pass each, kernel-filtered)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R; mkdir -p gpurun_out/pmc
cd /tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
for P in "${PASSES[@]:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES}"; do :; done
i=0
IFS='|' read -ra PS <<< "${PMCS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS|SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM}"
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "${KRE:-k_mmq}" --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 1 --pp 512 --no-cpu-baseline --roofline-steps 0 --no-split-series > $R/gpurun_out/pmc/b$i.json 2> $R/gpurun_out/pmc/b$i.err || { echo "pass $i rc=$?"; tail -5 $R/gpurun_out/pmc/b$i.err; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for f in glob.glob('gpurun_out/pmc/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:60]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()): print(f"   {c:28s} {v:16.0f}")
PY
rm -rf gpurun_out/pmc/p*/
