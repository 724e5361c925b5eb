"""Summarise [ktdist] lines (GGML_MI355X_KTRACE_DIST=<label>): per launch, the start / end spread of
workgroups [0, split) and [split, n) in us from the launch's first start.
usage: python scripts/ktdist.py <stderr file> [split]"""
import sys

import numpy as np

split = int(sys.argv[2]) if len(sys.argv) > 2 else 16
S0, E0, S1, E1 = [], [], [], []
for line in open(sys.argv[1]):
    if not line.startswith("[ktdist]"):
        continue
    vals = np.array([[float(x) for x in p.split(",")] for p in line.split(":", 1)[1].split()])
    S0.append(vals[:split, 0]); E0.append(vals[:split, 1]); S1.append(vals[split:, 0]); E1.append(vals[split:, 1])
if not S0:
    sys.exit("no [ktdist] lines")
for nm, a in (("wg<split start", S0), ("wg<split end", E0), ("wg>=split start", S1), ("wg>=split end", E1)):
    a = np.concatenate(a)
    if a.size == 0:
        continue
    print(f"{nm:16s} n {len(a):6d}  p10 {np.percentile(a, 10):6.2f}  p50 {np.percentile(a, 50):6.2f}  p90 {np.percentile(a, 90):6.2f}  max {a.max():6.2f}")
# the latest-ending workgroups of the rest, by index (mean over launches)
e1 = np.mean(np.stack(E1), axis=0)
idx = np.argsort(e1)[-12:][::-1]
print("latest wg>=split (index: mean end):", ", ".join(f"{i + split}:{e1[i]:.1f}" for i in idx))
s1 = np.mean(np.stack(S1), axis=0)
idx = np.argsort(s1)[-12:][::-1]
print("latest-starting wg>=split (index: mean start):", ", ".join(f"{i + split}:{s1[i]:.1f}" for i in idx))
