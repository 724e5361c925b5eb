set -o pipefail
mkdir -p gpurun_out/fd
C=llama3-8b-2l-q4km
TAG=unfused GGML_MI355X_NO_FUSE=1 GGML_MI355X_NO_GRAPH=1 timeout -k 10 200 python scripts/fuse_diff.py $C gpurun_out/fd/unfused.npy || exit 1
for m in 0; do
TAG=mode$m GGML_MI355X_NO_GRAPH=1 GGML_MI355X_NO_PROLOGUE=$m timeout -k 10 200 python scripts/fuse_diff.py $C gpurun_out/fd/m$m.npy || exit 1
done
python3 - <<'PY'
import numpy as np
d='gpurun_out/fd/'
u=np.load(d+'unfused.npy')
for m in (0,):
    a=np.load(d+f'm{m}.npy')
    diff=np.abs(a-u)
    print(m, 'max diff per step', [round(float(x),4) for x in diff.max(axis=1)], 'bitwise', bool((a.view(np.uint32)==u.view(np.uint32)).all()))
PY
