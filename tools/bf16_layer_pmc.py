#!/usr/bin/env python3
"""bf16 conv layers at config-4 batch (B=8 per GPU, 576x960 D192), default plans,
for counter passes: `run` launches each layer WARM + ITERS times; `report <dir>`
summarises rocprofv3 --pmc passes (tools/gpu_pmc.sh layout) per layer.

  python tools/bf16_layer_pmc.py run
  python tools/bf16_layer_pmc.py report gpurun_out/pmc_bf16
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B, WARM, ITERS = 8, 2, 3
L0, L1, L2 = (64, 192, 320), (32, 96, 160), (16, 48, 80)
LAYERS = {  # name: cin, cout, volume, accumulate
    "conv12_128to64_L1": (128, 64, L1, False),
    "stem1_32to32_L0": (32, 32, L0, False),
    "cell_16to16_L1": (16, 16, L1, True),
    "cell_8to8_L0": (8, 8, L0, True),
    "cell_32to32_L2": (32, 32, L2, True),
}


def run():
    import torch
    from leastereo_amd import kernels
    dev = "cuda"
    for name, (cin, cout, (d, h, w), acc) in LAYERS.items():
        x = kernels.to_c8(torch.randn(B, cin, d, h, w, device=dev))
        packed = kernels.pack_conv_weight_bf16(torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05)
        scale = torch.rand(cout, device=dev) + 0.5
        shift = torch.randn(cout, device=dev) * 0.1
        y = torch.zeros(B, cout // 8, d, h, w, 8, device=dev, dtype=torch.bfloat16)
        torch.cuda.synchronize()
        for _ in range(WARM + ITERS):
            kernels.conv3d_bnrelu_bf16(x, packed, cout, 3, scale, shift, True, y, acc)
        torch.cuda.synchronize()
        print(name, kernels.conv_kernel_name_bf16(B, cout, cin, d, h, w, 3), flush=True)


def report(d):
    names = list(LAYERS)
    res = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
        p = f.split("/")[-2]
        per, dur = collections.defaultdict(dict), {}
        for r in csv.DictReader(open(f)):
            if "conv_bf16_kernel" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
            dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for i, k in enumerate(sorted(per)):
            L, j = divmod(i, WARM + ITERS)
            if L >= len(names) or j < WARM:
                continue
            for c, v in per[k].items():
                res[names[L]][c] += v / ITERS
            res[names[L]][p + ":ns"] += dur[k] / ITERS
    for L in names:
        r = res[L]
        if not r:
            continue
        print(L, {k: round(v, 1) for k, v in sorted(r.items())})


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])
