"""Per-token decode kernel breakdown from a rocprofv3 kernel trace (decode steps only)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# decode tokens: every decode graph launches the RoPE table kernel once (before its first
# Q/K projection); segment the trace there (fallback: the longest kernel, the output projection)
dur = lambda r: int(r['End_Timestamp']) - int(r['Start_Timestamp'])
starts = [i for i, r in enumerate(rows) if 'k_rope_table' in r['Kernel_Name']]
if len(starts) < 3:
    longest = max(rows, key=dur)['Kernel_Name']
    starts = [i for i, r in enumerate(rows) if r['Kernel_Name'] == longest and dur(r) > 0.5 * dur(max(rows, key=dur))]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
toks = list(zip(starts[skip:-1], starts[skip + 1:]))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
busy = wall = maxgap = 0.0
for a, b in toks:
    seg = rows[a:b + 1]
    wall += (int(rows[b]['Start_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
    gaps = [(int(seg[k + 1]['Start_Timestamp']) - int(seg[k]['End_Timestamp'])) / 1e3 for k in range(len(seg) - 1)]
    maxgap += max(gaps)
    for k, r in enumerate(seg[:-1]):
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        busy += d
        n = r['Kernel_Name'].split('(')[0].replace('void mi355x::', '')[:56] + f" g{int(r.get('Grid_Size_X', r.get('Grid_Size', 0))) // int(r.get('Workgroup_Size_X', r.get('Workgroup_Size', 1)) or 1)}"
        agg[n][0] += 1
        agg[n][1] += d
        agg[n][2] += gaps[k - 1] if k > 0 else 0.0   # idle time before this kernel
nt = max(len(toks), 1)
print(f"tokens {nt}: wall {wall / nt:.1f} us/token, kernel busy {busy / nt:.1f} us/token, "
      f"launches {sum(v[0] for v in agg.values()) / nt:.1f}/token, largest gap (host) {maxgap / nt:.1f} us/token")
for n, (c, t, gp) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:64s} {c / nt:6.1f}/tok {t / c:7.2f} us  {t / nt:8.1f} us/tok  gap-before {gp / c:5.2f} us")
