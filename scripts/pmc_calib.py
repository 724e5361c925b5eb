"""FETCH_SIZE calibration against known bytes (verdict r02 item 4): the decode GEMV probe
(scripts/probe_geom.py: mi355x_bench_gemv2 launches of fixed shapes over rotating weight copies)
under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`; per shape (identified by kernel type and grid)
FETCH_SIZE x 1024 x 2 (the gfx950 correction for 16-B/lane streaming reads, MI355X_MICROARCH.md
HBM section) against the algorithmic weight bytes of one launch.  The one-shot GEMV streams every
weight type through 16-B/lane LDS-DMA, so the correction should hold for Q6_K as for Q4_K.

usage: python scripts/pmc_calib.py <counter_collection.csv> [out.json]"""
import collections
import csv
import json
import sys

# (type tag in the kernel name, grid workgroups) -> (shape, algorithmic weight bytes per launch)
BB = {"g_q4_K": 144, "g_q6_K": 210}
SHAPES = [("g_q4_K", 14336, 4096, 1), ("g_q6_K", 14336, 4096, 1), ("g_q4_K", 4096, 14336, 2),
          ("g_q4_K", 4096, 28672, 1), ("g_q4_K", 4096, 4096, 1), ("g_q4_K", 4096, 6144, 1), ("g_q6_K", 4096, 128256, 1)]


def main():
    path = sys.argv[1]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != "FETCH_SIZE":
            continue
        name = r["Kernel_Name"]
        tag = next((t for t in BB if t in name), None)
        if tag is None or "k_gemv" not in name:
            continue
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) // max(1, int(r.get("Workgroup_Size", 256) or 256))
        per[(tag, grid)].append(float(r["Counter_Value"]) * 1024 * 2)
    rows = []
    for tag, K, M, nm in SHAPES:
        alg = K // 256 * BB[tag] * M * nm
        cands = [(k, v) for k, v in per.items() if k[0] == tag]
        # the launches of this shape: the dispatch group whose mean is nearest the algorithmic bytes
        best = min(cands, key=lambda kv: abs(sum(kv[1]) / len(kv[1]) - alg), default=None)
        if best is None:
            continue
        m = sum(best[1]) / len(best[1])
        rows.append({"shape": f"{tag[2:]} {K}x{M}x{nm}", "grid": best[0][1], "launches": len(best[1]),
                     "algorithmic_MB": round(alg / 1e6, 3), "fetch_x2_MB": round(m / 1e6, 3), "ratio": round(m / alg, 3)})
    res = {"method": "rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 scripts/probe_geom.py; FETCH_SIZE KiB x 1024 x 2 "
                     "per dispatch, mean per shape; algorithmic = weight bytes of one launch", "shapes": rows}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
