#!/usr/bin/env python3
"""Tile sweep of the k=3 DMA conv engine: every instantiated (NT, TW, TD) tile on
every matching-net layer shape (tools/conv_bench.py LAYERS, B=1 at C2), timed
with HIP events.  Prints one line per (layer, tile) and the best tile per layer;
the planner's heuristics in csrc/conv3d.hip are fitted to this table.

  python tools/conv_sweep.py [--iters 10] [--only name,...] [--batch B] [--scale s]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402

TILES = [(nt, tw, td) for td in (1, 2) for nt in (1, 2, 4, 8) for tw in (16, 32, 64)
         if not (tw == 16 and nt > 2)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--only", default="")
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--bf16", action="store_true", help="sweep the bf16 engine (th, td, mt) tiles")
    a = p.parse_args()
    if a.bf16:
        return sweep_bf16(a)
    lib = _lib.load()
    dev = "cuda"
    only = set(a.only.split(",")) if a.only else None
    out = {}
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        if k != 3 or cout <= 2 or (only and name not in only):
            continue
        acc = bool(acc and acc[0])
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(a.batch, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, k, k, k, device=dev, generator=g) * 0.05
        packed = kernels.pack_conv_weight(wt)
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        y = torch.zeros(a.batch, cout, d, h, w, device=dev)
        flops = 2.0 * a.batch * d * h * w * cin * cout * 27
        lib.lea_conv3d_set_tile_override(0, 0, 0)
        default = kernels.conv_kernel_name(a.batch, cout, d, h, w, 3)
        res = {}
        for nt, tw, td in TILES:
            lib.lea_conv3d_set_tile_override(nt, tw, td)
            try:
                for _ in range(2):
                    kernels.conv3d_bnrelu(x, packed, cout, 3, scale, shift, True, y, acc)
            except _lib.HipKernelError:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                kernels.conv3d_bnrelu(x, packed, cout, 3, scale, shift, True, y, acc)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            res[f"{nt},{tw},{td}"] = ms
            print(f"{name:26s} nt={nt} tw={tw:2d} td={td}  {ms * 1e3:8.1f} us  "
                  f"{flops / ms / 1e9:6.1f} TF/s", flush=True)
        lib.lea_conv3d_set_tile_override(0, 0, 0)
        best = min(res, key=res.get)
        print(f"BEST {name}: {best} {res[best] * 1e3:.1f} us (default {default})", flush=True)
        out[name] = {"default": default, "best": best, "times_ms": res}
    print(json.dumps(out))


def sweep_bf16(a):
    lib = _lib.load()
    dev = "cuda"
    only = set(a.only.split(",")) if a.only else None
    tiles = [(th, td, mt) for th in (4, 8, 16) for td in (1, 2, 4) for mt in (1, 2)]
    out = {}
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        if k != 3 or cout <= 2 or (only and name not in only):
            continue
        acc = bool(acc and acc[0])
        cout8 = -(-cout // 8) * 8
        x = kernels.to_c8(torch.randn(a.batch, cin, d, h, w, device=dev))
        packed = kernels.pack_conv_weight_bf16(torch.randn(cout8, cin, 3, 3, 3, device=dev) * 0.05)
        scale = torch.rand(cout8, device=dev) + 0.5
        shift = torch.randn(cout8, device=dev) * 0.1
        y = torch.zeros(a.batch, cout8 // 8, d, h, w, 8, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * a.batch * d * h * w * cin * cout8 * 27
        lib.lea_conv3d_bf16_set_tile_override(0, 0, 0)
        default = kernels.conv_kernel_name_bf16(a.batch, cout8, cin, d, h, w, 3)
        res = {}
        for th, td, mt in tiles:
            lib.lea_conv3d_bf16_set_tile_override(th, td, mt)
            try:
                for _ in range(2):
                    kernels.conv3d_bnrelu_bf16(x, packed, cout8, 3, scale, shift, True, y, acc)
            except _lib.HipKernelError:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                kernels.conv3d_bnrelu_bf16(x, packed, cout8, 3, scale, shift, True, y, acc)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            res[f"{th},{td},{mt}"] = ms
            print(f"{name:26s} th={th:2d} td={td} mt={mt}  {ms * 1e3:8.1f} us  "
                  f"{flops / ms / 1e9:7.1f} TF/s", flush=True)
        lib.lea_conv3d_bf16_set_tile_override(0, 0, 0)
        best = min(res, key=res.get)
        print(f"BEST {name}: {best} {res[best] * 1e3:.1f} us (default {default})", flush=True)
        out[name] = {"default": default, "best": best, "times_ms": res}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
