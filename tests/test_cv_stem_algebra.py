"""CPU check of the algebra behind csrc/cv_stem.hip: stem0's 3x3x3 conv over the cost
volume (retrain/LEAStereo.py:34-48, skip_model_3d.py:141) equals the per-plane sum of
2D maps the factored kernel combines (include/leastereo_hip.h, lea_cv_stem_combine).
Float64 torch on CPU: the identity is exact up to summation order."""
import pytest
import torch
import torch.nn.functional as F

from oracle import torch_ref as ref


def split_weights(w):
    """lea_cv_stem_split_weights restated: [cout, 2C, 3, 3, 3] -> wl [9 cout, C, 3, 3],
    wr [6 cout, C, 3, 3]."""
    cout, c2 = w.shape[:2]
    c = c2 // 2
    wl = torch.zeros(9 * cout, c, 3, 3, dtype=w.dtype)
    wr = torch.zeros(6 * cout, c, 3, 3, dtype=w.dtype)
    for kd in range(3):
        for t in range(3):
            blk = w[:, :c, kd].clone()
            blk[..., :t] = 0
            wl[(3 * kd + t) * cout:(3 * kd + t + 1) * cout] = blk
        wr[kd * cout:(kd + 1) * cout] = w[:, c:, kd]
        wr[(3 + kd) * cout:(4 + kd) * cout, :, :, 1] = w[:, c:, kd, :, 2]
    return wl, wr


def combine(lm, rm, cout, d3):
    """lea_cv_stem_combine's sum (pre-BN), restated with explicit loops over planes."""
    b, _, h, wd = lm.shape
    lk = lm.view(b, 3, 3, cout, h, wd)
    bk = rm[:, :3 * cout].view(b, 3, cout, h, wd)
    k2 = rm[:, 3 * cout:].view(b, 3, cout, h, wd)
    out = torch.zeros(b, cout, d3, h, wd, dtype=lm.dtype)
    cols = torch.arange(wd)
    for d in range(d3):
        u = cols - d
        for kd in range(3):
            if not 0 <= d + kd - 1 < d3:
                continue
            t = (kd - u).clamp(min=0)
            left = torch.zeros(b, cout, h, wd, dtype=lm.dtype)
            for tv in range(3):
                sel = t == tv
                left[..., sel] = lk[:, kd, tv][..., sel]
            z = u - kd + 1
            right = torch.zeros_like(left)
            ok = (z >= 0) & (z < wd)
            right[..., ok] = bk[:, kd][..., z[ok]]
            right[..., z == -1] = k2[:, kd][..., 0:1].expand_as(right[..., z == -1])
            x = u[-1] - kd + 2  # last column: taps past the volume's right edge
            if 0 <= x < wd:
                right[..., -1] -= k2[:, kd][..., x]
            out[:, :, d] += left + right
    return out


@pytest.mark.parametrize("b,c,cout,maxdisp,hw", [(1, 4, 8, 27, (5, 8)), (2, 3, 4, 48, (4, 21)),
                                                  (1, 2, 3, 6, (3, 4)), (1, 4, 4, 9, (6, 3)),
                                                  (1, 3, 5, 24, (2, 30))])
def test_factored_stem_equals_the_cost_volume_conv(b, c, cout, maxdisp, hw):
    g = torch.Generator().manual_seed(b * 100 + c * 10 + cout)
    fl = torch.randn((b, c) + hw, generator=g, dtype=torch.float64)
    fr = torch.randn((b, c) + hw, generator=g, dtype=torch.float64)
    w = torch.randn(cout, 2 * c, 3, 3, 3, generator=g, dtype=torch.float64)
    d3 = int(maxdisp / 3)
    want = F.conv3d(ref.build_cost_volume(fl, fr, maxdisp), w, None, 1, 1)
    wl, wr = split_weights(w)
    lm = F.conv2d(fl, wl, None, 1, 1)
    rm = F.conv2d(fr, wr, None, 1, 1)
    got = combine(lm, rm, cout, d3)
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)
