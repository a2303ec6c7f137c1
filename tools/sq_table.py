"""SQ / GRBM counter table from tools/pmc_pass.sh passes (gpurun_out/<tag>/p*/run_counter_collection.csv).

    python tools/sq_table.py pmc_sq_r3 > profiles/r3_sq_counters.txt

Per kernel, means per dispatch after bench.py's spin marker: wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on
s_waitcnt / barrier), inst_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: MFMA / pipe / LDS queue),
active = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, lds_stall = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES; clock_GHz =
GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md "DVFS"); mfma_util = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x GRBM_GUI_ACTIVE / 8), the share of the kernel's SIMD-cycles its MFMA pipes were busy.
"""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc_sq"
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", tag)
per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> values
dur = collections.defaultdict(list)
for d in sorted(glob.glob(os.path.join(root, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    mk = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    rows = rows[mk[-1] + 1:] if mk else rows
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    tr = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tr) and not dur:
        for r in csv.DictReader(open(tr)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
mean = lambda v: sum(v) / len(v) if v else float("nan")  # noqa: E731
print(__doc__.strip().splitlines()[0])
print(f"{'kernel':78s} {'wait':>5s} {'stall':>5s} {'activ':>5s} {'ldsst':>5s} {'GHz':>5s} {'mfma%':>5s} {'ldsconf':>9s}")
for k, c in sorted(per.items(), key=lambda kv: -mean(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    wc = mean(c.get("SQ_WAVE_CYCLES", []))
    if not wc == wc or wc == 0:
        continue
    g = mean(c.get("GRBM_GUI_ACTIVE", []))
    t = mean(dur.get(k, []))
    clk = g / 8 / t / 1e9 if g == g and t == t and t > 0 else float("nan")
    mf = mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])) / (1024 * g / 8) if g == g and g > 0 else float("nan")
    print(f"{k[:78]:78s} {mean(c['SQ_WAIT_ANY'])/wc:5.2f} {mean(c['SQ_WAIT_INST_ANY'])/wc:5.2f} "
          f"{mean(c['SQ_ACTIVE_INST_ANY'])/wc:5.2f} {mean(c['SQ_WAIT_INST_LDS'])/wc:5.3f} {clk:5.2f} {100*mf:5.1f} "
          f"{mean(c['SQ_LDS_BANK_CONFLICT']):9.3g}")
