"""Per-run kernel breakdown of a rocprofv3 kernel trace: runs are separated by host gaps > GAP us
(default 2000); prints each run's wall span and its kernels by total time.
Usage: python3 scripts/pp_breakdown.py run_kernel_trace.csv [GAP_US]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 2000.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
runs, cur, last = [], [], None
for s, e, n in ev:
    if last is not None and (s - last) / 1e3 > gap:
        runs.append(cur)
        cur = []
    cur.append((s, e, n))
    last = e
runs.append(cur)
for i, r in enumerate(runs):
    span = (r[-1][1] - r[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in r) / 1e3
    if len(r) < 50:
        continue
    print(f"run {i}: {len(r)} kernels, span {span:.0f} us, busy {busy:.0f} us")
    agg = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n in r:
        k = n.split("(")[0][:70]
        agg[k][0] += (e - s) / 1e3
        agg[k][1] += 1
    for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:14]:
        print(f"   {t:9.1f} us {c:5d}  {k}")
