#!/usr/bin/env python3
"""The tap-sum head (lea_tapsum_upsample) at the bench shapes, every pass-2 form
(lea_tapsum_set_rows 2 = fused, 1 = two passes row-staged, 0 = two passes gather), f32 (C2)
and bf16 c8 (C4): HIP-event microseconds per call and whether the outputs agree bit for bit.

  python tools/tapsum_probe.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402

# (name, B, low-res volume (D, H, W), output volume, c8)
SHAPES = [("C2 f32", 1, (32, 96, 160), (64, 192, 320), False), ("C4 bf16", 8, (32, 96, 160), (64, 192, 320), True),
          ("C5 f32", 1, (44, 168, 252), (88, 336, 504), False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, b, src, dst, c8 in SHAPES:
        q = torch.randn((b, 27) + src, device="cuda", generator=g)
        if c8:
            q = kernels.to_c8(torch.cat([q, torch.zeros((b, 5) + src, device="cuda")], 1))
        call = (lambda: kernels.tapsum_upsample_bf16(q, 1, dst)) if c8 else (lambda: kernels.tapsum_upsample(q, 1, dst))
        outs = {}
        for mode in (2, 1, 0):
            _lib.check(lib.lea_tapsum_set_rows(mode), "rows")
            outs[mode] = call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                call()
            e1.record()
            torch.cuda.synchronize()
            print(f"{name:8s} mode={mode} {e0.elapsed_time(e1) / a.iters * 1e3:8.1f} us  "
                  f"same bits as mode 2: {bool(torch.equal(outs[mode], outs[2]))}", flush=True)
    _lib.check(lib.lea_tapsum_set_rows(2), "rows")


if __name__ == "__main__":
    main()
