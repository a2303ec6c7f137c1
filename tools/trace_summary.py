"""Per-step kernel summary of a rocprofv3 --kernel-trace CSV (one encode step = the kernels between two launches of
the encode's last kernel: rvq_final, or the persistent rvq_chain on small grids): count, total us per kernel name,
busy vs wall.   python tools/trace_summary.py DIR"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "rvq_final" in r["Kernel_Name"] or "rvq_chain" in r["Kernel_Name"]]
a, b = ends[-3] + 1, ends[-2] + 1
seg = rows[a:b]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"kernels/step {len(seg)}  wall {(t1 - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f} us")
agg = collections.OrderedDict()
for r in seg:
    n = r["Kernel_Name"].replace("void ", "")[:70]
    agg.setdefault(n, [0, 0.0])
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in agg.items():
    print(f"{v[0]:3d} {v[1]:8.1f}  {k}")
# gaps between consecutive dispatches of the step (idle GPU between one kernel's end and the next one's start)
gaps = []
for p, q in zip(seg, seg[1:]):
    g = (int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
    gaps.append((g, p["Kernel_Name"].replace("void ", "")[:40], q["Kernel_Name"].replace("void ", "")[:40]))
gs = sorted(g for g, _, _ in gaps)
if gs:
    print(f"gaps: {len(gs)}  sum {sum(gs):.1f} us  median {gs[len(gs) // 2]:.2f}  max {gs[-1]:.2f}")
    for g, a_, b_ in sorted(gaps, reverse=True)[:8]:
        print(f"  {g:6.2f} us  {a_} -> {b_}")
