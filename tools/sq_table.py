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
# kernel -> pass -> (sum GRBM_GUI_ACTIVE, sum duration, sum MFMA busy) over the SAME dispatches (the
# clock used to be GRBM means after the spin marker over the first pass's mean duration of ALL dispatches, including
# the calibration launches before the marker, which gave clocks up to 13.8 GHz)
clk_parts = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0]))
for d in sorted(glob.glob(os.path.join(root, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    mk = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    rows = rows[mk[-1] + 1:] if mk else rows
    # this pass's own durations, per dispatch (its kernel trace; else the counter rows' own timestamps)
    dur = {}
    tr = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    by_disp = collections.defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        did = int(r["Dispatch_Id"])
        by_disp[did][r["Counter_Name"]] = float(r["Counter_Value"])
        by_disp[did]["_k"] = k
        if did not in dur and r.get("End_Timestamp"):
            dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for did, c in by_disp.items():
        if "GRBM_GUI_ACTIVE" in c and dur.get(did, 0) > 0:
            acc = clk_parts[c["_k"]][d]
            acc[0] += c["GRBM_GUI_ACTIVE"]
            acc[1] += dur[did]
            acc[2] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan"))
            acc[3] += 1
MIN_CLOCK_MS = 0.3  # shorter dispatches: the GRBM-based clock (and the mfma% built on it) is not meaningful
mean = lambda v: sum(v) / len(v) if v else float("nan")  # noqa: E731
print(__doc__.strip().splitlines()[0])
print("clock = sum GRBM_GUI_ACTIVE / 8 / sum duration over the same dispatches of one pass; mfma% = "
      "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) of the pass that collected it.  Both are printed "
      f"only for kernels whose mean dispatch is >= {MIN_CLOCK_MS} ms: below that GRBM_GUI_ACTIVE over the dispatch "
      "duration reads above the chip's 2.4 GHz (MI355X_MICROARCH.md 'DVFS'), so neither number is evidence there ('-')")
print(f"{'kernel':78s} {'wait':>5s} {'stall':>5s} {'activ':>5s} {'ldsst':>5s} {'GHz':>5s} {'mfma%':>5s} {'ldsconf':>9s} "
      f"{'ms':>7s}")
for k, c in sorted(per.items(), key=lambda kv: -mean(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    wc = mean(c.get("SQ_WAVE_CYCLES", []))
    if not wc == wc or wc == 0:
        continue
    parts = list(clk_parts.get(k, {}).values())
    g = sum(p[0] for p in parts)
    t = sum(p[1] for p in parts)
    n = sum(p[3] for p in parts)
    clk = g / 8 / t / 1e9 if t > 0 else float("nan")
    mparts = [p for p in parts if p[2] == p[2]]
    mf = (sum(p[2] for p in mparts) / (1024 * sum(p[0] for p in mparts) / 8)
          if mparts and sum(p[0] for p in mparts) > 0 else float("nan"))
    ms = 1e3 * t / n if n else float("nan")
    ok = ms >= MIN_CLOCK_MS
    ghz = f"{clk:5.2f}" if ok else f"{'-':>5s}"
    mfp = f"{100 * mf:5.1f}" if ok else f"{'-':>5s}"
    print(f"{k[:78]:78s} {mean(c['SQ_WAIT_ANY'])/wc:5.2f} {mean(c['SQ_WAIT_INST_ANY'])/wc:5.2f} "
          f"{mean(c['SQ_ACTIVE_INST_ANY'])/wc:5.2f} {mean(c['SQ_WAIT_INST_LDS'])/wc:5.3f} {ghz} {mfp} "
          f"{mean(c['SQ_LDS_BANK_CONFLICT']):9.3g} {ms:7.3f}")
