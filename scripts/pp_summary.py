"""pp512 kernel summary from a rocprofv3 kernel trace of `bench.py --pp 512` (the last prefill run:
runs are split at host gaps > 200 us): per kernel its time, calls and share of the run, and for
the MFMA tiles the algorithmic TOPS against the dense peak of the MFMA dtype the tile issues
(k_mmq_q4Kh: v_mfma_f32_16x16x32_f16, 2.5 PFLOP/s; k_mmq_cls: v_mfma_i32_16x16x32_i8, 5 POPS).
Llama-3-8B Q4_K_M at T = 512 (src/llama-quant.cpp use_more_bits map): Q4_K weights 5.973 G
(Q, K, O, gate, up everywhere; V and down on 16 layers), Q6_K weights 1.007 G (V and down on
the other 16 layers); 2·T·params operations each.
Usage: python3 scripts/pp_summary.py run_kernel_trace.csv [T]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
GAP_US = 200.0   # a prefill graph launches back to back; decode tokens are separated by host work
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
runs, cur, last = [], [], None
for s, e, n in ev:
    if last is not None and (s - last) / 1e3 > GAP_US:
        runs.append(cur)
        cur = []
    cur.append((s, e, n))
    last = e
runs.append(cur)
pp = [r for r in runs if sum("k_mmq" in n for _, _, n in r) >= 32]
r = pp[-1]
span = (r[-1][1] - r[0][0]) / 1e3
busy = sum(e - s for s, e, _ in r) / 1e3
agg = collections.defaultdict(lambda: [0.0, 0])
for s, e, n in r:
    k = n.split("(")[0].replace("void ", "").replace("mi355x::", "")[:60]
    agg[k][0] += (e - s) / 1e3
    agg[k][1] += 1
ops = {"k_mmq_q4Kh": (2.0 * T * 5.973e9, 2500.0, "f16 MFMA"), "k_mmq_cls<mc_q6_K>": (2.0 * T * 1.007e9, 5000.0, "i8 MFMA")}
print(f"pp{T} prefill run: {len(r)} kernels, span {span:.0f} us ({T / span * 1e6:.0f} tok/s), busy {busy:.0f} us "
      f"({len(pp)} prefill runs in the trace, the last one shown)")
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:16]:
    extra = ""
    for key, (fl, peak, dt) in ops.items():
        if k.startswith(key):
            tops = fl / (t * 1e-6) / 1e12
            extra = f"  {tops:6.1f} TOPS = {tops / peak:.3f} of the {peak:.0f} {dt} dense peak"
    print(f"  {t:9.1f} us {100 * t / busy:5.1f}% {c:5d} calls  {k}{extra}")
