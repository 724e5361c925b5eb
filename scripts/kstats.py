"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, average and share.
Usage: kstats.py kernel_stats.csv NTOK — NTOK = single-token decodes in the traced run (the
"/tok" columns divide by it; scripts/gpu_final.sh computes it from the bench flags)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ntok = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms over {ntok:.0f} decode tokens; per token {tot / 1e3 / ntok:.1f} us "
      f"(includes the model-load / HBM-calibration kernels, each a few calls)")
for r in rows[:30]:
    print(f"{r['Name'][:88]:88s} {int(r['Calls']) / ntok:7.1f}/tok {float(r['AverageNs']) / 1000:8.2f}us "
          f"{float(r['TotalDurationNs']) / 1e3 / ntok:8.1f}us/tok {float(r['Percentage']):6.2f}%")
