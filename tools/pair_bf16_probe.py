#!/usr/bin/env python3
"""bf16 cell-step launches at C4 (B = 8): one LEA_PAIR_SUM launch (two ConvBRs summed, the
D-streaming kernel) against the two-launch form it replaces (conv a, then conv b accumulating
into a's output), HIP-event timed, with the bytes each moves (algorithmic: inputs once, output
once; the two-launch form also reads the accumulated output back) and the largest |pair -
two launches| in the output's bf16 units.

  python tools/pair_bf16_probe.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import kernels  # noqa: E402

B = 8
CASES = [("L1 16+16->16", 16, (32, 96, 160)), ("L0 8+8->8", 8, (64, 192, 320))]


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, c, (d, h, w) in CASES:
        xa = kernels.to_c8(torch.randn(B, c, d, h, w, device=dev, generator=g))
        xb = kernels.to_c8(torch.randn(B, c, d, h, w, device=dev, generator=g))
        wa = torch.randn(c, c, 3, 3, 3, device=dev, generator=g) / (c * 27) ** 0.5
        wb = torch.randn(c, c, 3, 3, 3, device=dev, generator=g) / (c * 27) ** 0.5
        sc = torch.rand(2 * c, device=dev, generator=g) + 0.5
        sh = torch.randn(2 * c, device=dev, generator=g) * 0.1
        pa, pb = kernels.pack_conv_weight_bf16(wa), kernels.pack_conv_weight_bf16(wb)
        pp = torch.cat([pa, pb])
        y1 = torch.empty(B, c // 8, d, h, w, 8, device=dev, dtype=torch.bfloat16)
        y2 = torch.empty_like(y1)

        def pair():
            kernels.conv3d_bnrelu_bf16(xa, pp, c, 3, sc, sh, True, y1, x2=xb, pair_sum=True)

        def two():
            kernels.conv3d_bnrelu_bf16(xa, pa, c, 3, sc[:c], sh[:c], True, y2)
            kernels.conv3d_bnrelu_bf16(xb, pb, c, 3, sc[c:], sh[c:], True, y2, accumulate=True)
        from leastereo_amd import _lib
        lib = _lib.load()
        lib.lea_conv3d_bf16_set_pair_split(0)
        t_pair0 = timed(pair, a.iters)
        lib.lea_conv3d_bf16_set_pair_split(1)
        t_pair1 = timed(pair, a.iters)
        y1b = y1.clone()
        lib.lea_conv3d_bf16_set_pair_split(2)
        t_pair, t_two = timed(pair, a.iters), timed(two, a.iters)
        lib.lea_conv3d_bf16_set_pair_split(3)  # the default again
        print(f"{name:14s} pair (both convs per wave) {t_pair0:8.1f} us ({3 * (B * d * h * w * c * 2) / t_pair0 / 1e6:5.2f} TB/s)")
        print(f"{name:14s} pair (split, no PP)        {t_pair1:8.1f} us ({3 * (B * d * h * w * c * 2) / t_pair1 / 1e6:5.2f} TB/s)"
              f"   max|PP - no PP|/max {float((y1.float() - y1b.float()).abs().max() / y1b.float().abs().max()):.2e}")
        vol = B * d * h * w * c * 2
        diff = float((y1.float() - y2.float()).abs().max() / y2.float().abs().max())
        print(f"{name:14s} pair {t_pair:8.1f} us ({3 * vol / t_pair / 1e6:5.2f} TB/s)   two launches "
              f"{t_two:8.1f} us ({5 * vol / t_two / 1e6:5.2f} TB/s)   max|diff|/max {diff:.2e}", flush=True)


if __name__ == "__main__":
    main()
