mkdir -p gpurun_out/fd
GGML_MI355X_DEBUG_FUSE=1 GGML_MI355X_NO_GRAPH=1 timeout -k 10 200 python scripts/fuse_diff.py llama3-8b-2l-q4km gpurun_out/fd/dbg.npy > gpurun_out/fusedbg.txt 2>&1; rc=$?
grep "mi355x\] \(gemv\|group\)" gpurun_out/fusedbg.txt | tail -24
exit $rc
