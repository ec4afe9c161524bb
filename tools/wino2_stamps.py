#!/usr/bin/env python3
"""Where the W x D Winograd kernel's waves spend their cycles: runs each f32 3x3x3
layer shape of config 2 that the planner puts on conv3d_wino2_kernel through the
diagnostic build (tools/build_variants.sh conv3d_wino2 stamps:"-DLEA_EXP_STAMPS
-fno-slp-vectorize" -> leastereo_amd/var_stamps.so) and prints the share of each
loop phase in the per-wave cycle sums (s_memtime stamps; shares only -- the stamps'
fences change the kernel's overlap, so the diagnostic build's run time means nothing).

  LEASTEREO_HIP_LIB=leastereo_amd/var_stamps.so python tools/wino2_stamps.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402

PHASES = ("dma wait", "barrier 1", "dma issue", "V pass", "barrier 2", "kh steps", "epilogue")


def main():
    lib = _lib.load()
    fn = lib.lea_exp_wino2_stamps
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    dev = "cuda"
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    for name, (cin, cout, k, (d, h, w), count, *acc) in LAYERS.items():
        if k != 3 or not kernels.wino_eligible(cout, cin, k) or (only and name not in only):
            continue
        kname = kernels.wino_kernel_name(1, cout, d, h, w, cin=cin)
        if not kname.startswith("conv3d_wino2_kernel<"):  # (the pipelined tile has no stamps)
            continue
        acc = bool(acc and acc[0])
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(1, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, 3, 3, 3, device=dev, generator=g) / (cin * 27) ** 0.5
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        y = torch.randn(1, cout, d, h, w, device=dev, generator=g)
        pw = kernels.pack_conv_weight_wino(wt)
        nw = int(kname.split("<")[1].split(",")[3])
        buf = torch.zeros(4 << 20, dtype=torch.int32, device=dev)  # 16 MiB: >= nblk * nw * 8 words
        for rep in range(3):  # the last of three runs (warm clocks and caches)
            buf.zero_()
            fn(buf.data_ptr())
            kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, acc)
            torch.cuda.synchronize()
            fn(None)
        v = buf.view(-1, 8).to(torch.int64).cpu()
        v = v[v[:, 7] > 0]
        tot = float(v[:, 7].sum())
        shares = [float(v[:, i].sum()) / tot for i in range(7)]
        print(f"{name:26s} {kname:48s} waves {v.shape[0]:6d}  cycles/wave {tot / v.shape[0]:9.0f}  " +
              "  ".join(f"{p} {s * 100:5.1f}%" for p, s in zip(PHASES, shares)), flush=True)


if __name__ == "__main__":
    main()
