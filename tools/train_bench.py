"""Times one training step of the matching path on the GPU:
cost volume -> newMatching in train mode -> Disp -> smooth_l1 -> backward, on the HIP
ops (leastereo_amd.training), and the same step with every op swapped for torch's
own (F.conv3d / F.batch_norm / F.interpolate on MIOpen: the reference's aten path on
this GPU) -- a measurement tool, not part of the product.  Also times ConvBR3d
forward + backward alone at the hot layer shapes.  One JSON line per measurement.

    python tools/train_bench.py [--height 288 --width 576 --maxdisp 96] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from leastereo_amd import training  # noqa: E402
from leastereo_amd.config import LEAStereoArgs, default_arch_args  # noqa: E402
from leastereo_amd.model import LEAStereo  # noqa: E402


def _torch_convbr(m, x, train):
    y = F.conv3d(x, m.conv.weight, padding=m.conv.weight.shape[-1] // 2)
    if m.use_bn:
        y = F.batch_norm(y, m.bn.running_mean, m.bn.running_var, m.bn.weight, m.bn.bias, train, m.bn.momentum,
                         m.bn.eps)
    return F.relu(y) if m.relu else y


def _torch_interp(x, size, align_corners=True):
    return F.interpolate(x, list(size), mode="trilinear", align_corners=align_corners)


def _torch_cost(fl, fr, maxdisp):
    d3, c = int(maxdisp / 3), fl.shape[1]
    cost = fl.new_zeros(fl.shape[0], 2 * c, d3, fl.shape[2], fl.shape[3])
    for i in range(d3):
        cost[:, :c, i, :, i:] = fl[:, :, :, i:]
        cost[:, c:, i, :, i:] = fr[:, :, :, :-i] if i > 0 else fr
    return cost


def _torch_disp(cost, maxdisp):
    u = F.interpolate(cost, [maxdisp, cost.shape[3] * 3, cost.shape[4] * 3], mode="trilinear", align_corners=False)
    p = F.softmax(-torch.squeeze(u, 1), dim=1)
    return torch.sum(p * torch.arange(maxdisp, device=cost.device, dtype=p.dtype).view(1, maxdisp, 1, 1), 1)


def step_fn(model, fl, fr, target, impl):
    if impl == "torch":
        saved = training._convbr, training.interpolate3d
        training._convbr, training.interpolate3d = _torch_convbr, _torch_interp
        try:
            disp = _torch_disp(training.matching_forward(model.matching, _torch_cost(fl, fr, model.maxdisp)),
                               model.maxdisp)
        finally:
            training._convbr, training.interpolate3d = saved
    else:
        disp = training.cost_to_disparity_train(model, fl, fr)
    loss = F.smooth_l1_loss(disp, target)
    loss.backward()
    return loss


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=288)
    ap.add_argument("--width", type=int, default=576)
    ap.add_argument("--maxdisp", type=int, default=96)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--impl", default="hip,torch")
    ap.add_argument("--whole", type=int, default=0, help="1: time only the whole-model train step")
    ap.add_argument("--torch-modes", default="default,benchmark",
                    help="MIOpen modes for the torch leg: default (immediate mode) and/or benchmark "
                         "(torch.backends.cudnn.benchmark=True: MIOpen's find per shape, more warm-up)")
    args = ap.parse_args()
    torch.backends.cudnn.allow_tf32 = False
    dev = "cuda"
    if args.whole:
        return whole_model(args, dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    # ConvBR3d forward + backward at the hot shapes (C2's L0 8->8 cell, L1 16->16, conv1)
    for name, (cin, cout, d, h, w) in {"L0_8to8": (8, 8, 64, 192, 320), "L1_16to16": (16, 16, 32, 96, 160),
                                       "conv1_128to64": (128, 64, 32, 96, 160)}.items():
        m = training.ConvBR3d(cin, cout, 3, 1, 1).to(dev).train()
        x = torch.randn(1, cin, d, h, w, device=dev, generator=gen).requires_grad_(True)
        dy = torch.randn(1, cout, d, h, w, device=dev, generator=gen)
        ms = timed(lambda: m(x).backward(dy), args.steps, args.warmup)
        fl = 2.0 * cin * cout * 27 * d * h * w  # one direct conv: 2 FLOPs per MAC
        # forward + data gradient + weight gradient = three convs' work
        print(json.dumps({"what": "convbr3d_fwd_bwd", "layer": name, "ms": round(ms, 3),
                          "direct_tflops": round(3 * fl / ms / 1e9, 1)}), flush=True)
    model = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=args.maxdisp)), dev).to(dev).train()
    h3, w3 = (args.height - 1) // 3 + 1, (args.width - 1) // 3 + 1
    fl = torch.randn(1, 32, h3, w3, device=dev, generator=gen).requires_grad_(True)
    fr = torch.randn(1, 32, h3, w3, device=dev, generator=gen).requires_grad_(True)
    target = torch.rand(1, 3 * h3, 3 * w3, device=dev, generator=gen) * args.maxdisp
    for impl in args.impl.split(","):
        for mode in (args.torch_modes.split(",") if impl == "torch" else ["-"]):
            torch.backends.cudnn.benchmark = mode == "benchmark"
            warm = args.warmup + (3 if mode == "benchmark" else 0)
            t0 = time.perf_counter()
            ms = timed(lambda: step_fn(model, fl, fr, target, impl), args.steps, warm)
            print(json.dumps({"what": "matching_train_step", "impl": impl, "miopen_mode": mode,
                              "height": args.height, "width": args.width, "maxdisp": args.maxdisp,
                              "ms": round(ms, 2), "warmup_steps": warm,
                              "wall_s": round(time.perf_counter() - t0, 1),
                              "peak_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}), flush=True)


def whole_model(args, dev):
    """train.py:150-158 on the drop-in: model.train(), model(left, right) with inputs that
    require grad, smooth_l1, backward, SGD step -- the whole model (feature net twice,
    cost volume, matching net, Disp) on the HIP library."""
    model = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=args.maxdisp)), dev).to(dev).train()
    opt = torch.optim.SGD(model.parameters(), lr=1e-4, momentum=0.9)
    gen = torch.Generator(device=dev).manual_seed(1)
    left = torch.randn(1, 3, args.height, args.width, device=dev, generator=gen).requires_grad_(True)
    right = torch.randn(1, 3, args.height, args.width, device=dev, generator=gen).requires_grad_(True)
    target = torch.rand(1, args.height, args.width, device=dev, generator=gen) * (args.maxdisp - 1)

    def step():
        opt.zero_grad()
        disp = model(left, right)
        mask = (target < args.maxdisp) & (target > 0.001)
        F.smooth_l1_loss(disp[mask], target[mask], reduction="mean").backward()
        opt.step()
    torch.cuda.reset_peak_memory_stats()
    ms = timed(step, args.steps, args.warmup)
    print(json.dumps({"what": "whole_model_train_step", "impl": "hip", "height": args.height, "width": args.width,
                      "maxdisp": args.maxdisp, "ms": round(ms, 2),
                      "peak_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}), flush=True)


if __name__ == "__main__":
    main()
