"""Per-kernel HBM read traffic from a rocprofv3 --pmc FETCH_SIZE pass (counter_collection.csv).

FETCH_SIZE is reported in KiB per dispatch; on gfx950 it counts half the bytes of 16-B/lane
streaming reads (MI355X_MICROARCH.md, HBM section), so the per-dispatch bytes are
FETCH_SIZE x 1024 x 2.  Writes a JSON with the decode-GEMV average and a per-kernel table."""
import collections
import csv
import json
import sys

path, out = sys.argv[1], sys.argv[2]
per = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    if r.get("Counter_Name") != "FETCH_SIZE":
        continue
    name = r["Kernel_Name"].split("(")[0]
    per[name].append(float(r["Counter_Value"]) * 1024 * 2)
gemv = [v for k, vs in per.items() if "k_gemv" in k for v in vs]
res = {
    "gemv_bytes_per_launch": round(sum(gemv) / len(gemv)) if gemv else None,
    "gemv_launches": len(gemv),
    "method": "rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 bench.py --steps 16 --warmup 2 --pp 0 "
              "--no-cpu-baseline --roofline-steps 0; per dispatch FETCH_SIZE (KiB) x 1024 x 2 (gfx950 FETCH_SIZE "
              "counts half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM section); averaged over "
              "every k_gemv* dispatch",
    "per_kernel_MB_per_launch": {k: round(sum(v) / len(v) / 1e6, 3)
                                 for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:24]},
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
