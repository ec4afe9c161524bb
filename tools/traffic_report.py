#!/usr/bin/env python3
"""Per-launch HBM traffic of the bench's conv kernels from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are in KB (x1024).  Per MI355X_MICROARCH.md (HBM section),
on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane) coalesced read;
the LDS-DMA input pieces here are 4 B/lane and the weight pieces 16 B/lane, so both
the raw and the x2-corrected read bytes are recorded; WRITE_SIZE is exact for
16-B stores and uncalibrated for the 4-B stores of the conv epilogue.
usage: traffic_report.py <fetch_pass_dir> <write_pass_dir> <out.json>
"""
import collections
import csv
import json
import re
import sys


def load(d, counter):
    per = collections.defaultdict(float)
    names = {}
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            per[k] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"]
    return per, names


# kernels the library names without their (code-variant) template arguments
PLAIN = {"conv3d_wino44_kernel", "conv3d_wino2p_kernel"}


def short(n):
    """Our kernel name (lea_*_kernel_name) of a rocprof name: 'fn<args>' or plain 'fn'."""
    m = re.search(r"lea::(?:\w+::)*(\w+)<([^>]*)>", n)
    if m:
        # a bool-only template (conv3d_wino2p_kernel<true>, conv3d_wino44_kernel<false>: code
        # variants of one kernel the library names without arguments)
        if m.group(1) in PLAIN or m.group(2) in ("true", "false"):
            return m.group(1)
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"lea::(?:\w+::)*(\w+)\(", n)
    return m.group(1) if m else None


fetch, names = load(sys.argv[1], "FETCH_SIZE")
write, wnames = load(sys.argv[2], "WRITE_SIZE")
agg = collections.defaultdict(lambda: {"launches": 0, "fetch_kb": 0.0})
for k, v in fetch.items():
    s = short(names[k])
    if s:
        agg[s]["launches"] += 1
        agg[s]["fetch_kb"] += v
wagg = collections.defaultdict(lambda: {"launches": 0, "write_kb": 0.0})
for k, v in write.items():
    s = short(wnames[k])
    if s:
        wagg[s]["launches"] += 1
        wagg[s]["write_kb"] += v
out = {}
for s, a in agg.items():
    w = wagg.get(s, {"launches": 1, "write_kb": 0.0})
    fr = a["fetch_kb"] * 1024 / a["launches"]
    wr = w["write_kb"] * 1024 / max(w["launches"], 1)
    out[s] = {"launches_profiled": a["launches"], "fetch_bytes_raw": fr, "write_bytes": wr,
              "bytes_per_launch": 2 * fr + wr,
              "note": "FETCH_SIZE*1024*2 (gfx950 wide-read correction) + WRITE_SIZE*1024, mean over "
                      "all launches of this instantiation in a `bench.py --steps 3` run"}
json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
for s, v in sorted(out.items(), key=lambda kv: -kv[1]["bytes_per_launch"]):
    print(f"{s:40s} {v['launches_profiled']:4d}  fetch(raw) {v['fetch_bytes_raw'] / 1e6:9.1f} MB  "
          f"write {v['write_bytes'] / 1e6:9.1f} MB  corrected total {v['bytes_per_launch'] / 1e6:9.1f} MB")
