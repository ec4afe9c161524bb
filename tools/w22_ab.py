#!/usr/bin/env python3
"""Same-process A/B of the 16-cout tiles on the C2 layer shapes: the per-lane F(4,3) x F(2,3)
tile (lea_conv3d_wino_set_w22(0)) against the F(2,3) x F(2,3) tile (1), HIP-event timed over
--iters launches, interleaved --rounds times (the first layer of a process runs at a lower
clock), with the largest |difference| between the two outputs.

  python tools/w22_ab.py [--iters 50] [--rounds 3] [--walks 0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402

# (name, cin, cout, (D, H, W), accumulate)
SHAPES = [("L1 16->16 acc", 16, 16, (32, 96, 160), True),
          ("L1 16->16", 16, 16, (32, 96, 160), False),
          ("C5 L1 16->16 acc", 16, 16, (44, 168, 252), True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--walks", default="0", help="depth pairs per workgroup for the w22 tile (0 = planner)")
    ap.add_argument("--only", default="", help="substring of the shape names to run (_ for a space)")
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    for name, cin, cout, (d, h, w), acc in SHAPES:
        if w % 4 or (a.only and a.only.replace("_", " ") not in name):
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(1, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, 3, 3, 3, device=dev, generator=g) / (cin * 27) ** 0.5
        sc = torch.rand(cout, device=dev, generator=g) + 0.5
        sh = torch.randn(cout, device=dev, generator=g) * 0.1
        r = torch.randn(1, cout, d, h, w, device=dev, generator=g)
        pw = kernels.pack_conv_weight_wino(wt)
        flops = 2.0 * d * h * w * cin * cout * 27
        outs = {}
        for rnd in range(a.rounds):
            for on, walk in [(0, 0)] + [(1, int(s)) for s in a.walks.split(",")]:
                _lib.check(lib.lea_conv3d_wino_set_w22(on), "w22")
                _lib.check(lib.lea_conv3d_wino2_set_walk(walk), "walk")
                y = r.clone()
                kernels.conv3d_bnrelu_wino(x, pw, cout, sc, sh, True, y, acc)
                outs[(on, walk)] = y
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    kernels.conv3d_bnrelu_wino(x, pw, cout, sc, sh, True, y, acc)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / a.iters * 1e3
                kname = kernels.wino_kernel_name(1, cout, d, h, w, cin=cin)
                print(f"{name:18s} r{rnd} w22={on} spw={walk} {kname:48s} {t:8.1f} us "
                      f"{flops / t / 1e6:7.1f} TF/s direct-equivalent", flush=True)
        diff = max(float((outs[k] - outs[(0, 0)]).abs().max()) for k in outs if k != (0, 0))
        print(f"{name:18s} max |w22 - per-lane| after {a.iters + 1} accumulations: {diff:.3e}", flush=True)
    _lib.check(lib.lea_conv3d_wino_set_w22(0), "w22")
    _lib.check(lib.lea_conv3d_wino2_set_walk(0), "walk")


if __name__ == "__main__":
    main()
