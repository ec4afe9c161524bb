#!/usr/bin/env python3
"""HIP-event timing of the bf16 layer set of tools/bf16_layer_pmc.py (B=8, default
plans) with whatever library LEASTEREO_HIP_LIB selects; one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import kernels  # noqa: E402
from tools.bf16_layer_pmc import B, LAYERS  # noqa: E402


def main():
    dev = "cuda"
    out = {"lib": os.path.basename(os.environ.get("LEASTEREO_HIP_LIB", "libleastereo_hip.so"))}
    for name, (cin, cout, (d, h, w), acc) in LAYERS.items():
        x = kernels.to_c8(torch.randn(B, cin, d, h, w, device=dev))
        packed = kernels.pack_conv_weight_bf16(torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05)
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        y = torch.zeros(B, cout // 8, d, h, w, 8, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, y, acc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, y, acc)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        out[name] = round(2.0 * B * d * h * w * cin * cout * 27 / ms / 1e9, 1)  # TF/s
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
