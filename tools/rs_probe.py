#!/usr/bin/env python3
"""Per-call time and algorithmic GB/s of lea_conv1x1_resampled_bf16 (the down-sampling
gather-GEMM) and of the streamed 1x1 (conv1x1_c8_kernel) at the C4 shapes; run it under two
libraries (LEASTEREO_HIP_LIB, tools/ab_libs.sh) to compare builds.

    python tools/rs_probe.py [--one]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import kernels  # noqa: E402

# (B, cin, cout, src DHW, dst DHW): tools/layer_list.py --config c4 (r05)
SHAPES = [(8, 32, 16, (64, 192, 320), (32, 96, 160)), (8, 32, 32, (64, 192, 320), (32, 96, 160)),
          (8, 64, 32, (32, 96, 160), (16, 48, 80)), (8, 64, 64, (32, 96, 160), (16, 48, 80))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for b, cin, cout, src, dst in SHAPES:
        x = kernels.to_c8(torch.randn((b, cin) + src, device=dev))
        w = torch.randn(cout, cin, 1, 1, 1, device=dev) / cin ** 0.5
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        packed = kernels.pack_conv_weight_bf16(w)
        nbytes = x.numel() * 2 + b * cout * dst[0] * dst[1] * dst[2] * 2
        out = kernels.conv1x1_resampled_bf16(x, dst, packed, cout, scale, shift, relu=True)
        for _ in range(3):
            kernels.conv1x1_resampled_bf16(x, dst, packed, cout, scale, shift, relu=True, out=out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(a.reps):
            kernels.conv1x1_resampled_bf16(x, dst, packed, cout, scale, shift, relu=True, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / a.reps
        print(f"rs  b {b} cin {cin:3d} cout {cout:2d} {src}->{dst} {us:8.1f} us "
              f"{nbytes / us / 1e3:7.1f} GB/s", flush=True)


ONE = [(8, 64, 16, (32, 96, 160)), (8, 64, 8, (32, 96, 160)), (8, 32, 32, (32, 96, 160)),
       (8, 64, 32, (32, 96, 160)), (8, 128, 32, (16, 48, 80)), (8, 128, 16, (16, 48, 80)),
       (16, 32, 8, (1, 192, 320))]


def one_by_one(reps):
    """The streamed 1x1 (conv1x1_c8_kernel) at the C4 shapes."""
    dev = torch.device("cuda", 0)
    for b, cin, cout, dhw in ONE:
        x = kernels.to_c8(torch.randn((b, cin) + dhw, device=dev))
        w = torch.randn(cout, cin, 1, 1, 1, device=dev) / cin ** 0.5
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        packed = kernels.pack_conv_weight_bf16(w)
        nbytes = x.numel() * 2 + b * cout * dhw[0] * dhw[1] * dhw[2] * 2
        out = kernels.conv3d_bnrelu_bf16(x, packed, cout, 1, scale, shift, relu=True)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(reps):
            kernels.conv3d_bnrelu_bf16(x, packed, cout, 1, scale, shift, relu=True, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
        print(f"1x1 b {b} cin {cin:3d} cout {cout:2d} {dhw} {us:8.1f} us "
              f"{nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
    one_by_one(20)
