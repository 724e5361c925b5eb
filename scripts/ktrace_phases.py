"""Average the [ktraw] phase stamps (GGML_MI355X_KTRACE_RAW=<label>, a MI_KT_PHASE=1 build of
the plugin) that backend.cpp kt_collect printed for workgroup 0 of every launch of that label:
per slot, microseconds from the workgroup's entry (slots 1-4 the waves' exits, 5.. the phases).
usage: python scripts/ktrace_phases.py <stderr file> [label]"""
import collections
import sys

rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("[ktraw]"):
        continue
    name, vals = line[len("[ktraw] "):].split(":", 1)
    if len(sys.argv) > 2 and name.strip() != sys.argv[2]:
        continue
    rows[name.strip()].append([float(v) for v in vals.split()])
names = ["exit w0", "exit w1", "exit w2", "exit w3", "DMA issued", "x arrived", "mean", "act in LDS", "weights in",
         "records", "walk", "epilogue start"]
for name, rs in rows.items():
    n = len(rs)
    print(f"{name}: {n} launches (workgroup 0), us from entry")
    for k in range(len(rs[0])):
        v = [r[k] for r in rs if k < len(r) and r[k] >= 0]
        lab = names[k] if k < len(names) else f"slot {k + 1}"
        if v:
            print(f"  {lab:16s} {sum(v) / len(v):7.2f}  (n {len(v)})")
