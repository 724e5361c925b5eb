# round 6: the four-wave decode attention standalone (GGML_MI355X_FA_DSH4=1) and carried in the
# Q/K/V launch: parity tests, then which launches carry it (GGML_MI355X_DEBUG_FUSE)
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
OUT=gpurun_out/${OUT:-r06/fa4}
mkdir -p $OUT
GGML_MI355X_FA_DSH4=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread -k "flash_attn" > $OUT/dsh4.log 2>&1 || { echo "dsh4 rc=$?"; tail -3 $OUT/dsh4.log; exit 1; }; grep -E "passed|failed" $OUT/dsh4.log | tail -1
GGML_MI355X_DEBUG_FUSE=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -k "greedy_llama3_8b_2layer" > $OUT/fuse.log 2>&1 || { echo "fuse rc=$?"; grep -E "fa carry|MI355X" $OUT/fuse.log | tail -5; exit 1; }; grep -E "fa carry|carried" $OUT/fuse.log | sort | uniq -c | head -20
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "${K:-flash_attn or greedy or fused_and_graph or concurrent or virtual_devices_bit}" > $OUT/pytest.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" $OUT/pytest.log | head; exit 1; }; grep -E "passed|failed" $OUT/pytest.log | tail -1
