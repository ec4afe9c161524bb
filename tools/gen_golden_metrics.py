#!/usr/bin/env python3
"""Golden vectors for the disparity metrics.

Imports the reference's utils/metrics.py (plain numpy, read-only tree,
PYTHONDONTWRITEBYTECODE=1) and evaluates it on seeded disparity maps that carry
the edge cases its code has: invalid ground truth (0, negative, >= maxdisp),
NaN ground truth, ground truth so large that gt * 0.05 > 10000, NaN and inf
predictions, differences on the integer truncation boundaries.  The EPE line of
evaluation.py:287-288 (and the :169 rounding) is evaluated with the same numpy
expressions (evaluation.py cannot be imported: argv parsing at import).

Writes tests/golden/metrics.npz (inputs + reference outputs).  Container only.
Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_metrics.py
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")


def cases():
    rng = np.random.default_rng(20261016)
    out = {}
    # a: typical frame with every edge case sprinkled in
    h, w = 48, 80
    gt = rng.uniform(-5, 230, (h, w)).astype(np.float32)
    gt[rng.random((h, w)) < 0.05] = 0.0
    gt[rng.random((h, w)) < 0.01] = np.nan
    gt[rng.random((h, w)) < 0.01] = 3.0e5
    gt[0, :4] = [0.001, 192.0, 191.999, 0.0011]
    pred = (gt + rng.normal(0, 2.5, (h, w))).astype(np.float32)
    pred[rng.random((h, w)) < 0.01] = np.nan
    pred[rng.random((h, w)) < 0.005] = np.inf
    pred[1, :6] = gt[1, :6] + np.array([1.0, 2.0, 3.0, 0.999, 1.999, 2.999], np.float32)
    out["a"] = (pred, gt, 192)
    # b: near-perfect prediction, maxdisp 48, a ragged odd shape
    gt = rng.uniform(0, 60, (33, 17)).astype(np.float32)
    out["b"] = ((gt + rng.normal(0, 0.4, gt.shape)).astype(np.float32), gt, 48)
    # c: one valid pixel
    gt = np.zeros((3, 5), np.float32)
    gt[1, 2] = 10.0
    out["c"] = (np.full((3, 5), 12.5, np.float32), gt, 192)
    return out


def main():
    sys.path.insert(0, "/root/reference")
    from utils import metrics as M  # utils/metrics.py:6-46

    arrays = {}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for name, (pred, gt, md) in cases().items():
            arrays[f"{name}/pred"] = pred
            arrays[f"{name}/gt"] = gt
            arrays[f"{name}/maxdisp"] = np.array(md)
            e3, correct = M.calculate_3px_error_and_correct_mask(pred, gt, md)
            arrays[f"{name}/three_px"] = np.array(M.calculate_3px_error(pred, gt, md))
            assert e3 == arrays[f"{name}/three_px"]
            arrays[f"{name}/correct"] = correct
            for t in (1, 2, 3):
                arrays[f"{name}/bad{t}"] = np.array(M.calculate_bad_pixel_frac(pred, gt, md, t))
            for rnd in (0, 1):
                p = pred.round() + 2 if rnd else pred  # evaluation.py:169 with z_shift 2
                mask = np.logical_and(gt >= 0.001, gt <= md)  # evaluation.py:287
                arrays[f"{name}/epe_r{rnd}"] = np.array(np.mean(np.abs(p[mask] - gt[mask])))
                arrays[f"{name}/three_px_r{rnd}"] = np.array(M.calculate_3px_error(p, gt, md))
    np.savez_compressed(os.path.join(GOLD, "metrics.npz"), **arrays)
    print({k: float(v) for k, v in arrays.items() if v.ndim == 0})


if __name__ == "__main__":
    main()
