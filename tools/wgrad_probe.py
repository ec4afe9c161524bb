#!/usr/bin/env python3
"""lea_conv3d_wgrad at the C2 training shapes (B = 1): HIP-event time per call (the MFMA
kernel plus the two fixed-order partial sums), direct-conv TFLOP/s (2 cout cin k^3 per
voxel) and the largest |dw - torch float64| / max|dw| on a small shape.

  python tools/wgrad_probe.py [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import training  # noqa: E402

SHAPES = [("conv1 128->64", 128, 64, (32, 96, 160)), ("L1 16->16", 16, 16, (32, 96, 160)),
          ("L0 8->8", 8, 8, (64, 192, 320)), ("L2 32->32", 32, 32, (16, 48, 80))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    # correctness on a small ragged shape
    x = torch.randn(2, 12, 5, 9, 70, device=dev, generator=g)
    dz = torch.randn(2, 20, 5, 9, 70, device=dev, generator=g)
    dw = training.conv3d_wgrad(x, dz, 3)
    ref = torch.nn.grad.conv3d_weight(x.double(), (20, 12, 3, 3, 3), dz.double(), padding=1)
    print(f"small 12->20: max|dw - f64|/max {float((dw.double() - ref).abs().max() / ref.abs().max()):.2e}", flush=True)
    for name, cin, cout, (d, h, w) in SHAPES:
        x = torch.randn(1, cin, d, h, w, device=dev, generator=g)
        dz = torch.randn(1, cout, d, h, w, device=dev, generator=g)
        training.conv3d_wgrad(x, dz, 3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            training.conv3d_wgrad(x, dz, 3)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        flops = 2.0 * cout * cin * 27 * d * h * w
        print(f"{name:14s} {us:9.1f} us  {flops / us / 1e6:7.1f} TF/s ({flops / us / 1e6 / 157.3:.3f} of 157.3)", flush=True)


if __name__ == "__main__":
    main()
