#!/usr/bin/env python3
"""lea_cv_stem_combine timing at the c2 (f32, B1) and c4 (bf16 c8, B8) stem0 shapes:
the full kernel vs its store-only probe variant (flag 0x100), HIP events, 20 reps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from leastereo_amd import _lib  # noqa: E402


def run(b, cout, d3, h, w, bf16, flags):
    lib = _lib.load()
    if bf16:
        lm = torch.randn(b, 9 * cout // 8, 1, h, w, 8, device="cuda").to(torch.bfloat16)
        rm = torch.randn(b, 6 * cout // 8, 1, h, w, 8, device="cuda").to(torch.bfloat16)
        y = torch.empty(b, cout // 8, d3, h, w, 8, device="cuda", dtype=torch.bfloat16)
    else:
        lm = torch.randn(b, 9 * cout, 1, h, w, device="cuda")
        rm = torch.randn(b, 6 * cout, 1, h, w, device="cuda")
        y = torch.empty(b, cout, d3, h, w, device="cuda")
    sc = torch.rand(cout, device="cuda")
    sh = torch.rand(cout, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def go():
        _lib.check(lib.lea_cv_stem_combine(lm.data_ptr(), lm.stride(0), rm.data_ptr(), rm.stride(0),
                                           sc.data_ptr(), sh.data_ptr(), y.data_ptr(), y.stride(0), b,
                                           cout, d3, h, w, flags, _lib.LEA_BF16 if bf16 else _lib.LEA_F32,
                                           st), "combine")
    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        go()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20
    nb = y.numel() * y.element_size()
    return t, nb / t / 1e9


for name, args in [("c2 f32", (1, 32, 64, 192, 320, False)), ("c4 c8", (8, 32, 64, 192, 320, True))]:
    for fl, lab in [(1, "full"), (0x100, "stores only")]:
        t, bw = run(*args, fl)
        print(f"{name:6s} {lab:12s} {t * 1e3:8.1f} us  {bw:6.2f} TB/s of output")
