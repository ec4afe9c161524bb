#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of tools/conv_bench.py per layer.
usage: pmc_report.py <dir-with-passN> <iters>   (conv_bench runs 3 warm-up + iters launches/layer)"""
import collections
import csv
import glob
import sys

d, iters = sys.argv[1], int(sys.argv[2])
sys.path.insert(0, ".")
from tools.conv_bench import LAYERS  # noqa: E402
layers = list(LAYERS)
per_layer = 3 + iters
res = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
    p = f.split("/")[-2]
    per, dur = collections.defaultdict(dict), {}
    for r in csv.DictReader(open(f)):
        if "conv" not in r["Kernel_Name"] or "pack_weights" in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for i, k in enumerate(sorted(per)):
        if i // per_layer >= len(layers) or i % per_layer < 3:
            continue
        L = layers[i // per_layer]
        for c, v in per[k].items():
            res[L][c] += v / iters
        res[L][p + ":ns"] += dur[k] / iters
print(f"{'layer':26s} {'us':>7s} {'GHz':>5s} {'MFMA%':>6s} {'VALU/MFMA':>9s} {'LDS/MFMA':>8s} "
      f"{'bank/LDS':>8s} {'wait%':>6s} {'waitLDS%':>8s} {'occ w/SIMD':>10s}")
for L in layers:
    r = res[L]
    if not r:
        continue
    ns = r["pass1:ns"]
    cyc = r["GRBM_GUI_ACTIVE"] / 2 / 8  # the counter is in two passes (1 and 4)
    mf = r["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
    nm = max(r["SQ_INSTS_MFMA"], 1)
    valu = (r["SQ_INSTS_VALU"] - nm) / nm
    lds = r["SQ_INSTS_LDS"] / 2 / nm  # SQ_INSTS_LDS collected in passes 2 and 4
    bank = r["SQ_LDS_BANK_CONFLICT"] / max(r["SQ_LDS_IDX_ACTIVE"], 1)
    wc = r["SQ_WAVE_CYCLES"]
    occ = wc / (cyc * 1024) if cyc else 0
    print(f"{L:26s} {ns / 1e3:7.1f} {cyc / ns:5.2f} {100 * mf:6.1f} {valu:9.2f} {lds:8.2f} "
          f"{bank:8.3f} {100 * r['SQ_WAIT_ANY'] / wc:6.1f} {100 * r['SQ_WAIT_INST_LDS'] / wc:8.1f} {occ:10.2f}")
