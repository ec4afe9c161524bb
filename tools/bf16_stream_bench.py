#!/usr/bin/env python3
"""bf16 single-chunk 3x3x3 layers at config-4 batch (B=8, 576x960 D192): the D-streaming
kernel (variant 0) vs the tile kernel (variant 1), HIP-event timed, bit-identity checked.

  python tools/bf16_stream_bench.py [--iters 10] [--batch 8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402

L0, L1, L2 = (64, 192, 320), (32, 96, 160), (16, 48, 80)
LAYERS = {  # name: cin, cout, volume, accumulate
    "cell_8to8_L0": (8, 8, L0, True),
    "cell_8to24_L0_s1grp": (8, 24, L0, False),
    "cell_16to16_L1": (16, 16, L1, True),
    "cell_16to48_L1_s1grp": (16, 48, L1, False),
    "stem1_32to32_L0": (32, 32, L0, False),
    "cell_32to32_L2": (32, 32, L2, True),
    "cell_32to96_L2_s1grp": (32, 96, L2, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    B = a.batch
    for name, (cin, cout, (d, h, w), acc) in LAYERS.items():
        x = kernels.to_c8(torch.randn(B, cin, d, h, w, device=dev))
        packed = kernels.pack_conv_weight_bf16(torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05)
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        y0 = kernels.to_c8(torch.randn(B, cout, d, h, w, device=dev))
        res = {}
        for v in (1, 0):
            lib.lea_conv3d_bf16_set_variant(v)
            y = y0.clone()
            kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, y, acc)
            res[v] = y
            yy = y0.clone()
            for _ in range(2):
                kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, yy, acc)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, yy, acc)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            nbytes = 2.0 * B * d * h * w * (cin + cout * (2 if acc else 1))
            print(f"{name:22s} v{v} {kernels.conv_kernel_name_bf16(B, cout, cin, d, h, w, 3):40s} "
                  f"{ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.1f} GB/s", flush=True)
        lib.lea_conv3d_bf16_set_variant(0)
        print(f"  bit-identical: {torch.equal(res[0], res[1])}", flush=True)


if __name__ == "__main__":
    main()
