#!/usr/bin/env python3
"""HBM bandwidth probe on the box: write-only (fill_), read-only (sum) and copy
of a 2 GiB fp32 buffer, HIP-event timed (the ceilings the HBM-bound kernels are
compared against)."""
import torch

n = 1 << 29  # 2 GiB of fp32
x = torch.empty(n, device="cuda")
y = torch.empty(n, device="cuda")
x.fill_(1.0)


def timed(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


for name, fn, nbytes in [("write (fill_)", lambda: y.fill_(2.0), 4 * n),
                         ("read (sum)", lambda: x.sum(), 4 * n),
                         ("copy", lambda: y.copy_(x), 8 * n)]:
    t = timed(fn)
    print(f"{name:14s} {nbytes / t / 1e12:6.2f} TB/s ({t * 1e3:.3f} ms)")
