"""Per-token decode kernel breakdown from a rocprofv3 kernel trace (decode steps only)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# decode tokens: each llama_decode starts with one k_get_rows (token embedding)
starts = [i for i, r in enumerate(rows) if 'k_get_rows' in r['Kernel_Name']]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
toks = list(zip(starts[skip:-1], starts[skip + 1:]))
agg = collections.defaultdict(lambda: [0, 0.0])
busy = wall = 0.0
for a, b in toks:
    seg = rows[a:b]
    wall += (int(rows[b]['Start_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
    for r in seg:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        busy += d
        n = r['Kernel_Name'].split('(')[0][:64]
        agg[n][0] += 1
        agg[n][1] += d
nt = len(toks)
print(f"tokens {nt}: wall {wall / nt:.1f} us/token, kernel busy {busy / nt:.1f} us/token, "
      f"launches {sum(v[0] for v in agg.values()) / nt:.1f}/token")
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:64s} {c / nt:6.1f}/tok {t / c:7.2f} us  {t / nt:8.1f} us/tok")
