"""ORACLE (test infrastructure only; never imported by the product): numpy
restatement of the reference's disparity metrics, the checker for
``lea_disparity_metrics`` (leastereo_amd/csrc/evalio.hip).

  * utils/metrics.py:6-8    calculate_validity_mask
  * utils/metrics.py:11-22  calculate_3px_error
  * utils/metrics.py:25-36  calculate_3px_error_and_correct_mask
  * utils/metrics.py:39-46  calculate_bad_pixel_frac
  * evaluation.py:169, 287-288  prediction.round() + z_shift; EPE over 0.001 <= gt <= maxdisp

Pinned by tests/golden/metrics.npz: the imported reference module
(utils/metrics.py is plain numpy) evaluated on seeded disparity maps with the
edge cases it has (invalid, NaN and huge ground truth; NaN / inf predictions),
written by tools/gen_golden_metrics.py.
"""
from __future__ import annotations

import numpy as np

INF_DISP = 10000


def calculate_validity_mask(target, max_disp):
    return (target < max_disp) & (target > 0.001)


def _abs_diff(pred, true, max_disp):
    mask = calculate_validity_mask(true, max_disp)
    abs_diff = np.full(true.shape, INF_DISP)  # int64: the float difference is truncated
    with np.errstate(invalid="ignore"):
        abs_diff[mask] = np.abs(true[mask] - pred[mask])
    return abs_diff, mask


def calculate_3px_error_and_correct_mask(pred, true, max_disp):
    abs_diff, mask = _abs_diff(pred, true, max_disp)
    with np.errstate(invalid="ignore"):
        correct = (abs_diff < 3) | (abs_diff < true * 0.05)
    return 1 - (float(np.sum(correct)) / float(len(np.argwhere(mask)))), correct


def calculate_3px_error(pred, true, max_disp):
    return calculate_3px_error_and_correct_mask(pred, true, max_disp)[0]


def calculate_bad_pixel_frac(pred, true, max_disp, threshold):
    abs_diff, mask = _abs_diff(pred, true, max_disp)
    correct = abs_diff <= threshold
    return 1 - (float(np.sum(correct)) / float(len(np.argwhere(mask))))


def evaluation_epe(prediction, disp, maxdisp, round_pred=False, z_shift=0):
    """evaluation.py:169 (optional) and :287-288."""
    if round_pred:
        prediction = prediction.round() + z_shift
    mask = np.logical_and(disp >= 0.001, disp <= maxdisp)
    return np.mean(np.abs(prediction[mask] - disp[mask])), prediction
