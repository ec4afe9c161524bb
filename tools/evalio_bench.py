#!/usr/bin/env python3
"""HIP-event timing of the host-step kernels either side of forward (SURVEY.md
§8f rank 3) against the HBM roofline, next to the numpy reference code on the host.

  standardize: lea_standardize_crop_u8, B pairs of 540x960 RGBA (SceneFlow PNGs)
               -> 576x960 float32 (config 2's crop, top-left pad).  Algorithmic
               bytes: uint8 images read once + float32 crops written once.
  metrics:     lea_disparity_metrics, B frames of 576x960; pred + gt read once.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from leastereo_amd import kernels  # noqa: E402
from oracle import metrics_ref as MR  # noqa: E402
from oracle import predict_ref as PR  # noqa: E402

HBM_GBS = 8000.0


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    B = int(os.environ.get("B", "8"))
    dev = "cuda:0"
    rng = np.random.default_rng(0)
    h, w, ps, ch, cw = 540, 960, 4, 576, 960
    lu = rng.integers(0, 256, (B, h, w, ps), dtype=np.uint8)
    ru = rng.integers(0, 256, (B, h, w, ps), dtype=np.uint8)
    lt, rt = torch.from_numpy(lu).to(dev), torch.from_numpy(ru).to(dev)
    ms = timed(lambda: kernels.standardize_crop_u8(lt, rt, ch, cw))
    nbytes = 2 * B * h * w * ps + 2 * B * 3 * ch * cw * 4
    t0 = time.perf_counter()
    for i in range(B):
        PR.test_transform(PR.standardize(lu[i], ru[i]), ch, cw)
    cpu = (time.perf_counter() - t0) / B
    out = [{"kernel": "lea_standardize_crop_u8", "case": f"B={B} {h}x{w}x{ps} u8 -> {ch}x{cw} f32",
            "ms": ms, "bytes": nbytes, "GB/s": nbytes / ms / 1e6, "hbm_frac": nbytes / ms / 1e6 / HBM_GBS,
            "pairs_per_s": B / ms * 1e3, "cpu_numpy_s_per_pair": cpu, "cpu_cores": 1}]

    gt = rng.uniform(-2, 200, (B, ch, cw)).astype(np.float32)
    pred = (gt + rng.normal(0, 3, gt.shape)).astype(np.float32)
    gtt, prt = torch.from_numpy(gt).to(dev), torch.from_numpy(pred).to(dev)
    ms = timed(lambda: kernels.disparity_metrics(prt, gtt, 192))
    nbytes = 2 * B * ch * cw * 4
    t0 = time.perf_counter()
    for i in range(B):
        MR.evaluation_epe(pred[i], gt[i], 192)
        MR.calculate_3px_error(pred[i], gt[i], 192)
        for t in (1, 2, 3):
            MR.calculate_bad_pixel_frac(pred[i], gt[i], 192, t)
    cpu = (time.perf_counter() - t0) / B
    out.append({"kernel": "lea_disparity_metrics", "case": f"B={B} {ch}x{cw} (EPE, 3px, bad1/2/3)",
                "ms": ms, "bytes": nbytes, "GB/s": nbytes / ms / 1e6,
                "hbm_frac": nbytes / ms / 1e6 / HBM_GBS, "frames_per_s": B / ms * 1e3,
                "cpu_numpy_s_per_frame": cpu, "cpu_cores": 1})
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
