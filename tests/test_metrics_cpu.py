"""Disparity-metric oracle (oracle/metrics_ref.py) against the reference's own
utils/metrics.py outputs (tests/golden/metrics.npz, tools/gen_golden_metrics.py)."""
import numpy as np
import pytest

from oracle import metrics_ref as MR
from tests.golden_util import golden

CASES = ("a", "b", "c")


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_metrics(name):
    g = golden("metrics")
    pred, gt, md = g[f"{name}/pred"], g[f"{name}/gt"], int(g[f"{name}/maxdisp"])
    e3, correct = MR.calculate_3px_error_and_correct_mask(pred, gt, md)
    assert e3 == float(g[f"{name}/three_px"])
    np.testing.assert_array_equal(correct, g[f"{name}/correct"])
    for t in (1, 2, 3):
        assert MR.calculate_bad_pixel_frac(pred, gt, md, t) == float(g[f"{name}/bad{t}"])
    for rnd in (0, 1):
        epe, p = MR.evaluation_epe(pred, gt, md, round_pred=bool(rnd), z_shift=2)
        np.testing.assert_array_equal(epe, g[f"{name}/epe_r{rnd}"])
        assert MR.calculate_3px_error(p, gt, md) == float(g[f"{name}/three_px_r{rnd}"])


def test_reference_quirks_are_in_the_vectors():
    """The cases exercise what the device kernel must reproduce: int64 truncation
    (|d| = 1.999 is within bad-1), invalid pixels with gt * 0.05 > 10000 counted
    correct, NaN predictions counted correct (INT64_MIN)."""
    g = golden("metrics")
    gt, pred, correct = g["a/gt"], g["a/pred"], g["a/correct"]
    huge = gt == 3.0e5
    assert huge.any() and correct[huge].all()
    mask = MR.calculate_validity_mask(gt, 192)
    nanp = np.isnan(pred) & mask
    assert nanp.any() and correct[nanp].all()
    assert MR.calculate_bad_pixel_frac(np.float32([[2.999]]), np.float32([[1.0]]), 192, 1) == 0.0
    assert MR.calculate_bad_pixel_frac(np.float32([[3.0]]), np.float32([[1.0]]), 192, 1) == 1.0
