#!/usr/bin/env python3
"""Merge a traffic_report.py JSON from a `bench.py --config TAG` run into
profiles/hbm_traffic.json under keys "<kernel>@TAG" (per-launch bytes depend on the
config's shapes); bf16 names drop the kernel-depth argument the bench does not print
(conv_bf16_kernel<3, 1, 4, 8, 2, 2, false, 3> -> conv_bf16_kernel<3, 1, 4, 8, 2, 2, false>).
usage: traffic_merge.py TAG report.json [profiles/hbm_traffic.json]"""
import json
import re
import sys

tag, src = sys.argv[1], sys.argv[2]
dst = sys.argv[3] if len(sys.argv) > 3 else "profiles/hbm_traffic.json"
merged = json.load(open(dst))
for name, v in json.load(open(src)).items():
    m = re.match(r"(conv_bf16_kernel<(\d+), .*), (\d+)>$", name)
    if m and m.group(2) == m.group(3):
        name = m.group(1) + ">"
    merged[f"{name}@{tag}"] = v
json.dump(merged, open(dst, "w"), indent=1, sort_keys=True)
print(f"merged {tag}: {len(merged)} entries")
