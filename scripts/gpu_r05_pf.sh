# prefill flash attention: parity of k_fattn_pf and its phase split; the Mixtral op dump
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
OUT=gpurun_out/${OUT:-r05/pf}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k flash_attn > $OUT/pytest_fa.log 2>&1 || { echo "fa tests rc=$?"; tail -30 $OUT/pytest_fa.log; exit 1; }
tail -1 $OUT/pytest_fa.log
timeout -k 10 120 python scripts/probe_fa_pf.py > $OUT/probe_pf.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_pf.txt; exit 1; }
cat $OUT/probe_pf.txt
if [ -n "${OPS:-}" ]; then
  timeout -k 10 400 python scripts/dbg_ops.py $OPS > $OUT/ops.txt 2>&1 || { echo "ops rc=$?"; tail -5 $OUT/ops.txt; exit 1; }
  grep -c "\[ops\]" $OUT/ops.txt
fi
if [ -n "${BASE_PLUGIN:-}" ]; then
  MI355X_PLUGIN=$BASE_PLUGIN timeout -k 10 120 python scripts/probe_fa_pf.py > $OUT/probe_pf_base.txt 2>&1 || { echo "probe base rc=$?"; tail -5 $OUT/probe_pf_base.txt; exit 1; }
  cat $OUT/probe_pf_base.txt
fi
