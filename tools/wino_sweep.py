#!/usr/bin/env python3
"""Tile sweep of the Winograd engine (np, td) vs the direct engine's default plan on
every f32 3x3x3 matching-net layer shape at config 2 (B=1), HIP-event timed.

  python tools/wino_sweep.py [--iters 10] [--batch 1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402


def timed(fn, iters):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    out = {}
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        if k != 3 or not kernels.wino_eligible(cout, cin, k) or (a.only and name not in a.only.split(",")):
            continue
        acc = bool(acc and acc[0])
        x = torch.randn(a.batch, cin, d, h, w, device=dev)
        wt = torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        y = torch.zeros(a.batch, cout, d, h, w, device=dev)
        flops = 2.0 * a.batch * d * h * w * cin * cout * 27
        pd, pw = kernels.pack_conv_weight(wt), kernels.pack_conv_weight_wino(wt)
        res = {"direct": timed(lambda: kernels.conv3d_bnrelu(x, pd, cout, 3, scale, shift, True, y, acc),
                               a.iters)}
        for f, np_, td in [(f, n, t) for f in (2, 4, 8) for n in (1, 2) for t in (1, 2)]:
            if True:
                lib.lea_conv3d_wino_set_tile_override(np_, td, f)
                try:
                    res[f"wino f={f} np={np_} td={td}"] = timed(
                        lambda: kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, acc), a.iters)
                except _lib.HipKernelError:
                    pass  # tile not instantiated for this block size
        lib.lea_conv3d_wino_set_tile_override(0, 0, 0)
        res["wino default"] = timed(lambda: kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, acc),
                                    a.iters)
        default = kernels.wino_kernel_name(a.batch, cout, d, h, w, cin=cin)
        for kk, ms in res.items():
            print(f"{name:26s} {kk:18s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF/s  x{count}", flush=True)
        print(f"  -> default {default}", flush=True)
        out[name] = {"count": count, "ms": res, "default": default}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
