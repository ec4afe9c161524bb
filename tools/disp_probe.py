#!/usr/bin/env python3
"""The disparity regression at the bench shapes, every form (lea_disparity_set_register_form
3 / 2 / 1 / 0), f32 and fast exp: HIP-event microseconds and the largest difference from form 1.

  python tools/disp_probe.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402

SHAPES = [("C2", 1, 64, 192, 320, 192), ("C4", 8, 64, 192, 320, 192), ("C3", 8, 64, 128, 416, 192),
          ("C5", 1, 88, 336, 504, 264)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, b, d3, h3, w3, md in SHAPES:
        x = torch.randn(b, 1, d3, h3, w3, device="cuda", generator=g) * 3
        for fast in (False, True):
            out = {}
            for form in (1, 2, 3, 4, 0):
                _lib.check(lib.lea_disparity_set_register_form(form), "form")
                out[form] = kernels.disparity_regression(x, md, fast)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    kernels.disparity_regression(x, md, fast)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.iters * 1e3
                print(f"{name} fast={int(fast)} form={form} {us:8.1f} us  max|d - form1| "
                      f"{float((out[form] - out.get(1, out[form])).abs().max()):.2e}"
                      + (f"  form 3 == form 2: {bool(torch.equal(out[3], out[2]))}" if form == 3 else ""),
                      flush=True)
    _lib.check(lib.lea_disparity_set_register_form(4), "form")


if __name__ == "__main__":
    main()
