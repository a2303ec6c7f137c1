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
