#!/usr/bin/env python3
"""c8 trilinear resample at the C4 level changes (B = 8): HIP-event time and output
bandwidth for 1, 2 and 4 output words per thread (lea_resample_bf16_set_batch), and k = 0:
the planner's choice (up-samplings: the column-walking kernel, r05)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from leastereo_amd import _lib, kernels  # noqa: E402

CASES = [("up 8ch L1->L0", 8, (32, 96, 160), (64, 192, 320)),
         ("up 16ch L2->L1", 16, (16, 48, 80), (32, 96, 160)),
         ("down 32ch L0->L1", 32, (64, 192, 320), (32, 96, 160)),
         ("down 64ch L1->L2", 64, (32, 96, 160), (16, 48, 80))]


def main():
    lib = _lib.load()
    only = sys.argv[1] if len(sys.argv) > 1 else None  # substring of a case name
    ks = tuple(int(k) for k in sys.argv[2].split(",")) if len(sys.argv) > 2 else (0, 4, 1)
    for name, c, src, dst in CASES:
        if only and only not in name:
            continue
        x = torch.randn((8, c // 8) + src + (8,), device="cuda").to(torch.bfloat16)
        sc = torch.rand(c, device="cuda") + 0.5
        sh = torch.rand(c, device="cuda")
        ref = None
        for k in ks:  # k = -2: the column walker with R = 16
            _lib.check(lib.lea_resample_bf16_set_cols(2 if k == -2 else 1), "set_cols")
            _lib.check(lib.lea_resample_bf16_set_batch(max(k, 0)), "set_batch")
            go = lambda: kernels.resample_trilinear_bf16(x, dst, True, None, sc, sh, True)  # noqa: E731
            y = go()
            if ref is None:
                ref = y
            assert torch.equal(y, ref), f"resample k={k} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                go()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 20
            nb = y.numel() * 2 + x.numel() * 2
            print(f"{name:18s} k={k}  {t * 1e3:7.1f} us  {nb / t / 1e9:5.2f} TB/s (in + out)")
        _lib.check(lib.lea_resample_bf16_set_batch(0), "set_batch")
        _lib.check(lib.lea_resample_bf16_set_cols(1), "set_cols")


if __name__ == "__main__":
    main()
