#!/usr/bin/env python3
"""lea_feature_stem_bnrelu (the fused feature stems 0 + 1) at the bench workloads: HIP-event
microseconds per launch and a digest of the output bytes (compare builds bit for bit with
tools/ab_libs.sh).

  python tools/stem_probe.py [--iters 20]
"""
import argparse
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import kernels  # noqa: E402

SHAPES = [("C2 f32", 2, 576, 960, False), ("C4 bf16", 16, 576, 960, True), ("C3 bf16", 16, 384, 1248, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    w0 = torch.randn(16, 3, 3, 3, device=dev, generator=g) / 27 ** 0.5
    w1 = torch.randn(32, 16, 3, 3, device=dev, generator=g) / 144 ** 0.5
    s0, t0 = torch.rand(16, device=dev, generator=g) + 0.5, torch.randn(16, device=dev, generator=g) * 0.1
    s1, t1 = torch.rand(32, device=dev, generator=g) + 0.5, torch.randn(32, device=dev, generator=g) * 0.1
    for name, b, h, w, c8 in SHAPES:
        x = torch.randn(b, 3, h, w, device=dev, generator=g)
        y = kernels.feature_stem(x, w0, s0, t0, w1, s1, t1, c8)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            kernels.feature_stem(x, w0, s0, t0, w1, s1, t1, c8)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        digest = hashlib.sha1(y.cpu().contiguous().view(torch.uint8).numpy().tobytes()).hexdigest()[:12]
        print(f"{name:8s} {us:8.1f} us  digest {digest}", flush=True)


if __name__ == "__main__":
    main()
