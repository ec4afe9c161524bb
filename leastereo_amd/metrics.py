"""utils/metrics.py and evaluation.py's per-frame metrics on the device.

Same names, arguments and results as the reference (utils/metrics.py:6-46), but
one HIP pass per call (``lea_disparity_metrics``) instead of numpy on the host;
``evaluate`` returns evaluation.py:287-307's per-frame numbers for a whole batch.
Inputs are float32 torch tensors on the ROCm device, or numpy arrays (moved
there).  The reference's quirks are kept, because they are its results:
  * ``abs_diff`` is the int64 array of ``np.full(shape, 10000)``: the float
    difference is truncated toward zero, so ``calculate_bad_pixel_frac(.., 1)``
    counts |d| < 2 as correct, and an invalid pixel whose gt * 0.05 exceeds
    10000 counts as correct in the 3-px error;
  * the EPE mask (evaluation.py:287: 0.001 <= gt <= maxdisp) and the metrics'
    validity mask (metrics.py:6-8: 0.001 < gt < maxdisp) differ at the bounds;
  * no valid pixel -> ZeroDivisionError, as the reference's float division.
"""
from __future__ import annotations

import numpy as np
import torch

from . import kernels


def _device_tensor(x):
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    if not x.is_cuda:
        if not torch.cuda.is_available():
            raise RuntimeError("leastereo_amd metrics run on a ROCm device only")
        x = x.cuda()
    return x.float()


def _counts(predicted_disparity, true_disparity, max_disp, thresholds=(1, 2, 3), mask=False,
            round_pred=False, z_shift=0):
    pred = _device_tensor(predicted_disparity)
    gt = _device_tensor(true_disparity).to(pred.device)
    out, m = kernels.disparity_metrics(pred, gt, max_disp, round_pred, z_shift, thresholds, mask)
    return out.cpu().numpy(), m


def calculate_validity_mask(target, max_disp: int):
    """utils/metrics.py:6-8 (elementwise; device tensor in, bool tensor out)."""
    t = _device_tensor(target)
    return (t < max_disp) & (t > 0.001)


def calculate_3px_error(predicted_disparity, true_disparity, max_disp: int) -> float:
    """utils/metrics.py:11-22."""
    c, _ = _counts(predicted_disparity, true_disparity, max_disp)
    return 1 - float(c[0, 3]) / float(c[0, 2])


def calculate_3px_error_and_correct_mask(predicted_disparity, true_disparity, max_disp: int):
    """utils/metrics.py:25-36: (3-px error, bool correct mask [H, W] on the device)."""
    c, m = _counts(predicted_disparity, true_disparity, max_disp, mask=True)
    return 1 - float(c[0, 3]) / float(c[0, 2]), m[0].bool()


def calculate_bad_pixel_frac(predicted_disparity, true_disparity, max_disp: int, threshold: int) -> float:
    """utils/metrics.py:39-46."""
    c, _ = _counts(predicted_disparity, true_disparity, max_disp, thresholds=(threshold,) * 3)
    return 1 - float(c[0, 4]) / float(c[0, 2])


def evaluate(prediction, disp, maxdisp: int, round_pred: bool = False, z_shift: int = 0):
    """evaluation.py:287-307 for a batch [B, H, W] (or one [H, W] frame): per-frame
    EPE, 3-px error, bad 2.0, bad 1.0, bad 3.0.  ``round_pred`` applies
    evaluation.py:169 (``prediction.round() + z_shift``) on the device first."""
    c, _ = _counts(prediction, disp, maxdisp, (1, 2, 3), round_pred=round_pred, z_shift=z_shift)
    rows = []
    for r in c:
        rows.append({
            "epe": float(r[1] / r[0]) if r[0] > 0 else float("nan"),  # np.mean of empty -> nan
            "three_px_error": 1 - float(r[3]) / float(r[2]),
            "bad_2": 1 - float(r[5]) / float(r[2]),
            "bad_1": 1 - float(r[4]) / float(r[2]),
            "bad_3": 1 - float(r[6]) / float(r[2]),
        })
    return rows
