#!/usr/bin/env python3
"""Per-layer microbenchmark of the HIP ConvBR3d kernel at the matching-net
shapes of the 576x960 D192 workload (B=1).  Times each layer with HIP events
over --iters back-to-back launches and prints TFLOP/s and GB/s (algorithmic).

  python tools/conv_bench.py [--iters 20] [--only name,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import kernels  # noqa: E402

L0, L1, L2 = (64, 192, 320), (32, 96, 160), (16, 48, 80)
# name: (cin, cout, k, level, count per forward[, accumulate: the cell's second op
# of a step adds into the slot the first one wrote, LEA_RESIDUAL])
LAYERS = {
    "stem0_64to32_k3_L0": (64, 32, 3, L0, 1),
    "stem1_32to32_k3_L0": (32, 32, 3, L0, 1),
    "conv12_128to64_k3_L1": (128, 64, 3, L1, 2),
    "cell_16to48_k3_L1_s1grp": (16, 48, 3, L1, 6),
    "cell_16to32_k3_L1_s1grp2": (16, 32, 3, L1, 0),  # (a candidate split of the 16->48 group)
    "cell_16to16_k3_L1": (16, 16, 3, L1, 18, True),
    "cell_32to96_k3_L2_s1grp": (32, 96, 3, L2, 5),
    "cell_32to32_k3_L2": (32, 32, 3, L2, 15, True),
    "cell_8to24_k3_L0_s1grp": (8, 24, 3, L0, 1),
    "cell_8to16_k3_L0_s1grp2": (8, 16, 3, L0, 0),  # (a candidate split of the 8->24 group)
    "cell_8to8_k3_L0": (8, 8, 3, L0, 3, True),
    "last3_32to1_k3_L0": (32, 1, 3, L0, 1),
    "pre_64to8_k1_L1": (64, 8, 1, L1, 2),
    "pre_32to16_k1_L1": (32, 16, 1, L1, 6),
    "pre_128to32_k1_L2": (128, 32, 1, L2, 8),
}


# name: (cin, cout, input volume, output volume, count per forward)
RESAMPLED = {
    "down_32to16_k1_L0toL1": (32, 16, L0, L1, 4),
    "down_64to32_k1_L1toL2": (64, 32, L1, L2, 5),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--only", default="")
    a = p.parse_args()
    dev = "cuda"
    only = set(a.only.split(",")) if a.only else None
    res = {}
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        acc = bool(acc and acc[0])
        if only and name not in only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(1, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, k, k, k, device=dev, generator=g) * 0.05
        packed = kernels.pack_conv_weight(wt)
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        out = torch.zeros(1, cout, d, h, w, device=dev)
        for _ in range(3):
            kernels.conv3d_bnrelu(x, packed, cout, k, scale, shift, True, out, acc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            kernels.conv3d_bnrelu(x, packed, cout, k, scale, shift, True, out, acc)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        vox = d * h * w
        flops = 2.0 * vox * cin * cout * k ** 3
        nbytes = 4.0 * vox * (cin + cout * (2 if acc else 1))
        res[name] = {"ms": ms, "tflops": flops / ms / 1e9, "gbs": nbytes / ms / 1e6,
                     "per_forward_ms": ms * count,
                     "kernel": kernels.conv_kernel_name(1, cout, d, h, w, k)}
        print(f"{name:24s} {ms * 1e3:9.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s  "
              f"{nbytes / ms / 1e6:8.1f} GB/s  x{count:2d} = {ms * count:6.3f} ms/fwd  "
              f"{res[name]['kernel']}", flush=True)
    # resampled 1x1 preprocess (trilinear align_corners down by 2 fused into the conv)
    for name, (cin, cout, src, dst, count) in RESAMPLED.items():
        if only and name not in only:
            continue
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn((1, cin) + src, device=dev, generator=g)
        wt = torch.randn(cout, cin, 1, 1, 1, device=dev, generator=g) * 0.1
        packed = kernels.pack_conv_weight(wt)
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        for _ in range(3):
            y = kernels.conv3d_bnrelu_resampled(x, dst, packed, cout, 1, scale, shift, True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            y = kernels.conv3d_bnrelu_resampled(x, dst, packed, cout, 1, scale, shift, True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        nbytes = 4.0 * (cin * src[0] * src[1] * src[2] + cout * dst[0] * dst[1] * dst[2])
        res[name] = {"ms": ms, "tflops": 0.0, "gbs": nbytes / ms / 1e6, "per_forward_ms": ms * count,
                     "kernel": kernels.conv_kernel_name(1, cout, *dst, 1, True)}
        print(f"{name:24s} {ms * 1e3:9.1f} us  {'':15s}  {nbytes / ms / 1e6:8.1f} GB/s  "
              f"x{count:2d} = {ms * count:6.3f} ms/fwd  {res[name]['kernel']}", flush=True)
    print("total ms/forward", sum(v["per_forward_ms"] for v in res.values()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
