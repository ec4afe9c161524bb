"""Device preprocessing and metrics (lea_standardize_crop_u8, lea_disparity_metrics)
against the numpy oracles (oracle/predict_ref.py, oracle/metrics_ref.py) and the
reference's own metric outputs (tests/golden/metrics.npz)."""
import numpy as np
import pytest
import torch

from leastereo_amd import kernels, metrics
from oracle import metrics_ref as MR
from oracle import predict_ref as PR
from tests.golden_util import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _images(seed, h, w, ps, b=1):
    rng = np.random.default_rng(seed)
    return (rng.integers(0, 256, (b, h, w, ps), dtype=np.uint8),
            rng.integers(0, 256, (b, h, w, ps), dtype=np.uint8))


def _ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    return np.abs(ai - bi).max()


@pytest.mark.parametrize("h,w,ps,ch,cw", [
    (540, 960, 4, 288, 576),    # config 1: SceneFlow RGBA, centre crop
    (375, 1242, 3, 384, 1248),  # KITTI RGB into a larger crop: top-left zero pad
    (41, 67, 3, 41, 67),        # exact fit
    (50, 60, 4, 32, 60),        # crop on one axis only
    (1, 1, 3, 4, 4),            # one pixel (std 0 -> NaN, as numpy)
])
def test_standardize_crop_matches_numpy(h, w, ps, ch, cw):
    """load_data + test_transform (predict.py:144-184): float32 output within one
    ulp of the numpy float64 expression (exact integer statistics on the device;
    numpy's pairwise float64 variance can differ in its last bits)."""
    lu, ru = _images(h * w + ps, h, w, ps)
    want_l, want_r, _, _ = PR.test_transform(PR.standardize(lu[0], ru[0]), ch, cw)
    with np.errstate(all="ignore"):
        got_l, got_r = kernels.standardize_crop_u8(torch.from_numpy(lu).to(DEV),
                                                   torch.from_numpy(ru).to(DEV), ch, cw)
    for got, want in ((got_l, want_l), (got_r, want_r)):
        g, wnt = got.cpu().numpy(), want.numpy()
        assert g.shape == wnt.shape
        fin = np.isfinite(wnt)
        np.testing.assert_array_equal(np.isnan(g), np.isnan(wnt))
        if fin.any():
            assert _ulp_diff(g[fin], wnt[fin]) <= 1
            assert np.mean(g[fin] == wnt[fin]) > 0.9999


def test_standardize_constant_channel_and_batch():
    """A constant channel gives NaN (0 / 0) like np.std == 0; batched pairs are
    standardised with their own statistics."""
    lu, ru = _images(7, 30, 40, 3, b=3)
    lu[1, :, :, 2] = 17
    got_l, got_r = kernels.standardize_crop_u8(torch.from_numpy(lu).to(DEV),
                                               torch.from_numpy(ru).to(DEV), 30, 40)
    for i in range(3):
        with np.errstate(all="ignore"):
            want_l, want_r, _, _ = PR.test_transform(PR.standardize(lu[i], ru[i]), 30, 40)
        np.testing.assert_array_equal(np.isnan(got_l[i].cpu().numpy()), np.isnan(want_l[0].numpy()))
        fin = np.isfinite(want_l[0].numpy())
        assert _ulp_diff(got_l[i].cpu().numpy()[fin], want_l[0].numpy()[fin]) <= 1
        assert _ulp_diff(got_r[i].cpu().numpy(), want_r[0].numpy()) <= 1
    assert torch.isnan(got_l[1, 2]).all()


def test_standardize_rejects_what_the_reference_cannot_copy():
    lu, ru = _images(3, 20, 100, 3)
    with pytest.raises(ValueError, match="test_transform"):
        kernels.standardize_crop_u8(torch.from_numpy(lu).to(DEV), torch.from_numpy(ru).to(DEV), 32, 64)


def test_standardize_on_the_c1_fixture_crop():
    """The config-1 SceneFlow crop (reference sample pair): device standardisation
    of the 288x576 crop == numpy's on the same pixels."""
    g = golden("c1_sceneflow")
    lu, ru = g["left_u8"], g["right_u8"]
    want_l, want_r, _, _ = PR.test_transform(PR.standardize(lu, ru), 288, 576)
    got_l, got_r = kernels.standardize_crop_u8(torch.from_numpy(lu).to(DEV),
                                               torch.from_numpy(ru).to(DEV), 288, 576)
    assert _ulp_diff(got_l.cpu().numpy(), want_l.numpy()) <= 1
    assert _ulp_diff(got_r.cpu().numpy(), want_r.numpy()) <= 1


@pytest.mark.parametrize("name", ["a", "b", "c"])
def test_metrics_match_reference_vectors(name):
    """utils/metrics.py outputs of the reference itself, including its int64
    truncation, NaN/inf and huge-gt quirks; EPE of evaluation.py:287-288 within
    float32 summation noise (the reference sums in float32)."""
    g = golden("metrics")
    pred, gt, md = g[f"{name}/pred"], g[f"{name}/gt"], int(g[f"{name}/maxdisp"])
    e3, mask = metrics.calculate_3px_error_and_correct_mask(pred, gt, md)
    assert e3 == float(g[f"{name}/three_px"])
    np.testing.assert_array_equal(mask.cpu().numpy(), g[f"{name}/correct"])
    assert metrics.calculate_3px_error(pred, gt, md) == float(g[f"{name}/three_px"])
    for t in (1, 2, 3):
        assert metrics.calculate_bad_pixel_frac(pred, gt, md, t) == float(g[f"{name}/bad{t}"])
    for rnd in (0, 1):
        row = metrics.evaluate(pred, gt, md, round_pred=bool(rnd), z_shift=2)[0]
        want = float(g[f"{name}/epe_r{rnd}"])
        if np.isnan(want):
            assert np.isnan(row["epe"])
        else:
            assert abs(row["epe"] - want) <= 1e-5 * max(1.0, abs(want))
        assert row["three_px_error"] == float(g[f"{name}/three_px_r{rnd}"])


def test_metrics_batch_at_full_size_vs_oracle():
    """A batch of 4 frames at 576x960: per-frame metrics == the oracle's, counts
    exact, EPE to float32 summation noise; every frame also equals its B=1 call."""
    rng = np.random.default_rng(5)
    gt = rng.uniform(-2, 200, (4, 576, 960)).astype(np.float32)
    pred = (gt + rng.normal(0, 3, gt.shape)).astype(np.float32)
    rows = metrics.evaluate(torch.from_numpy(pred).to(DEV), torch.from_numpy(gt).to(DEV), 192)
    for i, r in enumerate(rows):
        epe, _ = MR.evaluation_epe(pred[i], gt[i], 192)
        assert abs(r["epe"] - float(epe)) <= 1e-5 * float(epe)
        assert r["three_px_error"] == MR.calculate_3px_error(pred[i], gt[i], 192)
        for t in (1, 2, 3):
            assert r[f"bad_{t}"] == MR.calculate_bad_pixel_frac(pred[i], gt[i], 192, t)
        assert metrics.evaluate(pred[i], gt[i], 192)[0] == r


def test_metrics_no_valid_pixel_raises_like_the_reference():
    gt = np.zeros((4, 4), np.float32)
    with pytest.raises(ZeroDivisionError):
        metrics.calculate_3px_error(gt, gt, 192)
