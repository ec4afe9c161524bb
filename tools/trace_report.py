#!/usr/bin/env python3
"""Per-kernel time of ONE forward from a rocprofv3 kernel trace of bench.py
(the interval between the last two disparity kernels).
usage: trace_report.py <prof dir>"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
disp = [i for i, r in enumerate(rows) if "disparity" in r["Kernel_Name"] and "_f32" in r["Kernel_Name"]]
seg = rows[disp[-2] + 1: disp[-1] + 1]
t0, t1 = int(rows[disp[-2]]["End_Timestamp"]), int(rows[disp[-1]]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"forward wall {(t1 - t0) / 1e6:.3f} ms, kernels {len(seg)}, busy {busy / 1e6:.3f} ms")
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    n = r["Kernel_Name"].replace("void ", "").replace("lea::", "")[:64]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{t:9.1f} us {c:4d}  {n}")
