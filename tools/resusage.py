"""Per-kernel resource usage (VGPRs, scratch, occupancy) of one plugin source, from the
compiler's kernel-resource-usage remarks (device-only compile, nothing is linked).
Usage: python3 tools/resusage.py llamacog_amd/csrc/k_gemv.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics", "-ffp-contract=off", *(["-fno-slp-vectorize"] if "k_mmq_f16" in sys.argv[1] else []),
       "-DGGML_BACKEND_SHARED", "-DGGML_BACKEND_BUILD", "-DGGML_SHARED", "-DGGML_BACKEND_DL", "-DNDEBUG",
       "-I/root/reference/ggml/include", "-I/root/reference/ggml/src", "-Illamacog_amd/csrc", "--offload-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/_resusage.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?):\s*(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (name, r), d in zip(rows.items(), dem):
    if flt and flt not in d:
        continue
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  scratch {r.get('ScratchSize [bytes/lane]', '?'):>4}  occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {d[:110]}")
