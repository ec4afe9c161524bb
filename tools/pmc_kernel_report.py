#!/usr/bin/env python3
"""Per-kernel counter summary of rocprofv3 --pmc passes over any program:
mean per launch of each counter for kernels whose name contains FILTER, plus the
derived clock / MFMA-busy / LDS-busy / wait fractions.
usage: pmc_kernel_report.py <dir with pass*/run_counter_collection.csv> FILTER"""
import collections
import csv
import glob
import sys

d, filt = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
    per, name, dur = collections.defaultdict(dict), {}, {}
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        name[k] = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, cs in per.items():
        for c, v in cs.items():
            acc[name[k]][c].append(v)
        acc[name[k]]["ns"].append(dur[k])
for n, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    ns = m["ns"]
    line = f"{n}: {ns / 1e3:.1f} us"
    if "GRBM_GUI_ACTIVE" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        line += f", clock {cyc / ns:.2f} GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            line += f", MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}"
        if "SQ_LDS_IDX_ACTIVE" in m:
            line += f", LDS busy {m['SQ_LDS_IDX_ACTIVE'] / (cyc * 256):.3f}"
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in m:
                line += f", {c[3:]} {m[c] / m['SQ_WAVE_CYCLES']:.3f}"
    print(line)
    print("   ", {c: round(v, 1) for c, v in sorted(m.items())})
