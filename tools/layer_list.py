#!/usr/bin/env python3
"""Every probed launch of one forward, in launch order: kernel, (B, cin, cout, D, H, W, k),
HIP-event microseconds (median over --reps forwards), direct-conv TFLOP/s and algorithmic
GB/s (the probe's bytes: inputs + output + weights [+ residual]).

    python tools/layer_list.py [--config c2|c3|c4|c5] [--reps 5]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from leastereo_amd import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    model = bench.build_model(cfg["maxdisp"], dev, cfg["precision"])
    g = torch.Generator(device=dev).manual_seed(1234)
    shape = (cfg["batch"], 3, cfg["height"], cfg["width"])
    left = torch.randn(*shape, device=dev, generator=g)
    right = torch.randn(*shape, device=dev, generator=g)
    runs = []
    with torch.no_grad():
        for _ in range(3):
            model(left, right)
        for _ in range(a.reps):
            with kernels.KernelProbe() as probe:
                model(left, right)
            torch.cuda.synchronize()
            runs.append([(n, f, s, e0.elapsed_time(e1), nb) for n, f, nb, e0, e1, _, s in probe.records])
    total = 0.0
    for i, rec in enumerate(runs[0]):
        us = statistics.median(r[i][3] for r in runs) * 1e3
        total += us
        name, flops, shp = rec[0], rec[1], rec[2]
        tf = flops / us / 1e6 if us > 0 else 0.0
        gbs = rec[4] / us / 1e3 if us > 0 else 0.0
        print(f"{i:3d} {us:8.1f} us {tf:7.1f} TF/s {gbs:7.1f} GB/s  {str(shp):34s} {name}")
    print(f"conv launches {len(runs[0])}, {total / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
