#!/usr/bin/env python3
"""Winograd engine variants (lea_conv3d_wino_set_variant: 1 = F(4,3) along W, 2..4 =
F(4,3) along W x F(2,3) along D tiles) on every f32 3x3x3 matching-net layer shape at
config 2, HIP-event timed, each checked against the 1-D engine's output.

  python tools/wino2_sweep.py [--iters 10] [--batch 1] [--only name,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402
from tools.wino_sweep import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="1,2,3,4")
    ap.add_argument("--walks", default="0", help="W x D engine depth pairs per workgroup (0 = planner)")
    ap.add_argument("--small", default="0", help="couts <= 8: 1 = 16-row blocks (W x D), 0 = depth-paired")
    ap.add_argument("--block48", default="1", help="48k couts: 1 = 48-row 1-D blocks, 0 = padded W x D")
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    out = {}
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        if k != 3 or not kernels.wino_eligible(cout, cin, k) or (a.only and name not in a.only.split(",")):
            continue
        acc = bool(acc and acc[0])
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(a.batch, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, 3, 3, 3, device=dev, generator=g) / (cin * 27) ** 0.5
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        r = torch.randn(a.batch, cout, d, h, w, device=dev, generator=g)
        flops = 2.0 * a.batch * d * h * w * cin * cout * 27
        pw = kernels.pack_conv_weight_wino(wt)
        res, ref = {}, None
        for v, walk, sm, b48 in [(int(s), int(t), int(u), int(x)) for s in a.variants.split(",")
                                 for t in a.walks.split(",") for u in a.small.split(",")
                                 for x in a.block48.split(",")]:
            assert lib.lea_conv3d_wino_set_small_cout(sm) == 0
            assert lib.lea_conv3d_wino_set_block48(b48) == 0
            pw = kernels.pack_conv_weight_wino(wt)
            assert lib.lea_conv3d_wino_set_variant(v) == 0
            assert lib.lea_conv3d_wino2_set_walk(walk) == 0
            kname = kernels.wino_kernel_name(a.batch, cout, d, h, w, cin=cin) + (f" spw{walk}" if walk else "") + \
                ("" if cout > 8 else f" small{sm}") + ("" if cout % 48 or cout % 32 == 0 else f" b48={b48}")
            y = r.clone()
            kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, acc)
            torch.cuda.synchronize()
            if ref is None:
                ref = y
            err = float((y - ref).abs().max() / (ref.abs().max() + 1e-30))
            yy = torch.zeros_like(r)
            ms = timed(lambda: kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, yy, acc), a.iters)
            res[f"{v}/{walk}/{sm}/{b48}"] = {"kernel": kname, "ms": ms, "tflops": flops / ms / 1e9, "max_rel_diff_vs_v1": err}
            print(f"{name:26s} v{v} {kname:44s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF/s  "
                  f"x{count}  diff {err:.2e}", flush=True)
        lib.lea_conv3d_wino_set_variant(0)
        lib.lea_conv3d_wino2_set_walk(0)
        lib.lea_conv3d_wino_set_small_cout(0)
        lib.lea_conv3d_wino_set_block48(1)
        out[name] = {"count": count, "variants": res}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
