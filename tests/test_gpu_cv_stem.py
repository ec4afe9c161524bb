"""GPU parity of the factored stem0 (csrc/cv_stem.hip): 2D maps of the feature maps
(lea_conv2d_bnrelu[_bf16]) + lea_cv_stem_combine against float64 torch of stem0's
ConvBR3d over the materialised cost volume (retrain/LEAStereo.py:34-48,
skip_model_3d.py:141).

Tolerances: f32 |d| <= 1e-4 + 1e-4*|ref| (the ConvBR3d bar: same products, summed in
another order); bf16 |d| <= 1e-2 * max|ref| (the bf16 path's bar; bf16-rounded inputs
and weights, the maps rounded to bf16 before the f32 sum)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from leastereo_amd import kernels
from oracle import torch_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(b, c, cout, maxdisp, hw, seed):
    g = torch.Generator().manual_seed(seed)
    fl = torch.randn((b, c) + hw, generator=g)
    fr = torch.randn((b, c) + hw, generator=g)
    w = torch.randn(cout, 2 * c, 3, 3, 3, generator=g) / np.sqrt(2 * c * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    return fl, fr, w, scale, shift


def _want(fl, fr, w, scale, shift, maxdisp):
    y = F.conv3d(ref.build_cost_volume(fl.double(), fr.double(), maxdisp), w.double(), None, 1, 1)
    return torch.relu(y * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))


@pytest.mark.parametrize("b,c,cout,maxdisp,hw", [
    (2, 32, 32, 48, (12, 40)), (1, 4, 16, 27, (5, 8)), (1, 32, 32, 192, (10, 100)),
    (1, 8, 48, 9, (9, 20)), (1, 8, 16, 6, (3, 4)), (1, 32, 32, 264, (4, 132)), (1, 16, 24, 96, (7, 320)),
    (1, 4, 8, 1700, (2, 8))])  # D3 = 566: the planes split over two workgroups
def test_cv_stem_f32_vs_float64(b, c, cout, maxdisp, hw):
    fl, fr, w, scale, shift = _case(b, c, cout, maxdisp, hw, c + cout + maxdisp)
    d3 = int(maxdisp / 3)
    assert kernels.cv_stem_supported(cout, d3, hw[1], False)
    wl, wr = kernels.cv_stem_split_weights(w.to(DEV))
    lm = kernels.conv2d_bnrelu(fl.to(DEV).unsqueeze(2), kernels.pack_conv2d_weight(wl), 9 * cout, None,
                               None, relu=False)
    rm = kernels.conv2d_bnrelu(fr.to(DEV).unsqueeze(2), kernels.pack_conv2d_weight(wr), 6 * cout, None,
                               None, relu=False)
    got = kernels.cv_stem_combine(lm, rm, cout, d3, scale.to(DEV), shift.to(DEV), relu=True)
    want = _want(fl, fr, w, scale, shift, maxdisp)
    np.testing.assert_allclose(got.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


def test_cv_stem_split_weights_layout():
    g = torch.Generator().manual_seed(1)
    w = torch.randn(5, 6, 3, 3, 3, generator=g)
    wl, wr = kernels.cv_stem_split_weights(w.to(DEV))
    wl, wr = wl.cpu(), wr.cpu()
    for kd in range(3):
        for t in range(3):
            blk = w[:, :3, kd].clone()
            blk[..., :t] = 0
            assert torch.equal(wl[(3 * kd + t) * 5:(3 * kd + t + 1) * 5], blk)
        assert torch.equal(wr[kd * 5:(kd + 1) * 5], w[:, 3:, kd])
        k2 = torch.zeros(5, 3, 3, 3)
        k2[..., 1] = w[:, 3:, kd, :, 2]
        assert torch.equal(wr[(3 + kd) * 5:(4 + kd) * 5], k2)


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("b,c,cout,maxdisp,hw", [(2, 32, 32, 48, (12, 40)), (1, 16, 16, 27, (5, 19)),
                                                  (1, 32, 32, 192, (6, 70)), (1, 16, 40, 12, (3, 5)),
                                                  (1, 16, 16, 700, (2, 24))])  # D3 = 233: split
def test_cv_stem_bf16_vs_float64(b, c, cout, maxdisp, hw):
    fl, fr, w, scale, shift = _case(b, c, cout, maxdisp, hw, 7 * c + cout + maxdisp)
    fl, fr, w = _bf(fl), _bf(fr), _bf(w)
    d3 = int(maxdisp / 3)
    assert kernels.cv_stem_supported(cout, d3, hw[1], True)
    wl, wr = kernels.cv_stem_split_weights(w.to(DEV))
    lm = kernels.conv2d_bnrelu_bf16(kernels.to_c8(fl.to(DEV)), kernels.pack_conv2d_weight_bf16(wl),
                                    9 * cout, None, None, relu=False)
    rm = kernels.conv2d_bnrelu_bf16(kernels.to_c8(fr.to(DEV)), kernels.pack_conv2d_weight_bf16(wr),
                                    6 * cout, None, None, relu=False)
    got = kernels.from_c8(kernels.cv_stem_combine(lm, rm, cout, d3, scale.to(DEV), shift.to(DEV)))
    want = _want(fl, fr, w, scale, shift, maxdisp)
    err = float((got.cpu().double() - want).abs().max())
    assert err <= 1e-2 * float(want.abs().max()), err


def test_cv_stem_rejects_unsupported_shapes():
    lm = torch.zeros(1, 9 * 16, 1, 4, 6, device=DEV)
    rm = torch.zeros(1, 6 * 16, 1, 4, 6, device=DEV)
    with pytest.raises(kernels._lib.HipKernelError):  # f32 rows must be float4-aligned
        kernels.cv_stem_combine(lm, rm, 16, 4, None, None)
    lm = torch.zeros(1, 9 * 16, 1, 4, 8, device=DEV)
    rm = torch.zeros(1, 6 * 16, 1, 4, 8, device=DEV)
    with pytest.raises(kernels._lib.HipKernelError):  # one plane: d = 0 is also the last
        kernels.cv_stem_combine(lm, rm, 16, 1, None, None)
