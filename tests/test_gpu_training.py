"""Training backward of ConvBR3d (leastereo_amd/training.py,
csrc/conv3d_grad.hip) against torch autograd of the reference's ConvBR
(models/operations_3d.py:31-47: Conv3d bias-free -> BatchNorm3d -> ReLU) in float64 on
the CPU, on the same seeded inputs.  The reference's train.py:130-178 runs the layer in
train mode (batch statistics, running-stat update); eval mode is covered too.

Tolerance (fp32 kernels vs the float64 reference): every output / gradient within
2e-4 * max|reference| + 1e-6 elementwise; running statistics within 1e-5 relative."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref(x, w, g, bt, rm, rv, training, momentum, eps, use_bn, relu, dy):
    x = x.detach().cpu().double().requires_grad_(True)
    w = w.detach().cpu().double().requires_grad_(True)
    g = g.detach().cpu().double().requires_grad_(True)
    bt = bt.detach().cpu().double().requires_grad_(True)
    rm, rv = rm.detach().cpu().double().clone(), rv.detach().cpu().double().clone()
    z = F.conv3d(x, w, padding=w.shape[-1] // 2)
    if use_bn:
        z = F.batch_norm(z, rm, rv, g, bt, training, momentum, eps)
    if relu:
        z = F.relu(z)
    z.backward(dy.detach().cpu().double())
    return z.detach(), x.grad, w.grad, g.grad, bt.grad, rm, rv


def _close(a, r, what):
    a = a.detach().double().cpu()
    tol = 2e-4 * float(r.abs().max()) + 1e-6
    err = float((a - r).abs().max())
    assert err <= tol, f"{what}: max|d| {err:.3e} > {tol:.3e}"


CASES = [
    # B, cin, cout, D, H, W, k, training, bn, relu
    (2, 8, 8, 6, 10, 70, 3, True, True, True),     # L0 cell shape, ragged W segments
    (1, 16, 16, 4, 8, 16, 3, True, True, True),    # L1 cell
    (2, 64, 32, 3, 5, 9, 3, False, True, True),    # eval mode (frozen statistics)
    (1, 32, 1, 4, 6, 20, 3, False, False, False),  # last_3: no BN, no ReLU
    (2, 24, 48, 3, 4, 33, 1, True, True, True),    # 1x1 preprocess
    (1, 128, 64, 2, 4, 12, 3, True, True, True),   # conv1 / conv2
    (1, 4, 80, 2, 3, 7, 3, True, True, False),     # two cout blocks, BN without ReLU
    (2, 3, 5, 1, 1, 1, 3, True, True, True),       # one voxel per sample (padding only)
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:7])) + f"-t{int(c[7])}b{int(c[8])}r{int(c[9])}")
def test_convbr3d_forward_backward_vs_fp64(case):
    from leastereo_amd.training import _ConvBR3dFn
    b, cin, cout, d, h, w, k, training, use_bn, relu = case
    gen = torch.Generator().manual_seed(7 + cin * 31 + cout)
    x = torch.randn(b, cin, d, h, w, generator=gen)
    wt = torch.randn(cout, cin, k, k, k, generator=gen) * (2.0 / (cin * k ** 3)) ** 0.5
    g = 1 + 0.2 * torch.randn(cout, generator=gen)
    bt = 0.1 * torch.randn(cout, generator=gen)
    rm = 0.1 * torch.randn(cout, generator=gen)
    rv = 1 + torch.rand(cout, generator=gen)
    dy = torch.randn(b, cout, d, h, w, generator=gen)
    momentum, eps = 0.1, 1e-5
    ref = _ref(x, wt, g, bt, rm, rv, training, momentum, eps, use_bn, relu, dy)

    xd = x.to(DEV).requires_grad_(True)
    wd = wt.to(DEV).requires_grad_(True)
    gd = g.to(DEV).requires_grad_(True)
    bd = bt.to(DEV).requires_grad_(True)
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    y = _ConvBR3dFn.apply(xd, wd, gd if use_bn else None, bd if use_bn else None, rmd if use_bn else None,
                          rvd if use_bn else None, training, momentum, eps, use_bn, relu)
    y.backward(dy.to(DEV))
    torch.cuda.synchronize()
    _close(y, ref[0], "y")
    _close(xd.grad, ref[1], "dx")
    _close(wd.grad, ref[2], "dw")
    if use_bn:
        _close(gd.grad, ref[3], "dgamma")
        _close(bd.grad, ref[4], "dbeta")
        assert torch.allclose(rmd.cpu().double(), ref[5], rtol=1e-5, atol=1e-6)
        assert torch.allclose(rvd.cpu().double(), ref[6], rtol=1e-5, atol=1e-6)


def test_single_value_per_channel_in_train_mode_raises():
    """torch's batch_norm refuses one value per channel in train mode; so does ConvBR3d."""
    from leastereo_amd.training import ConvBR3d
    m = ConvBR3d(3, 5, 3, 1, 1).to(DEV).train()
    with pytest.raises(ValueError):
        m(torch.randn(1, 3, 1, 1, 1, device=DEV))


def test_wgrad_deterministic_and_vs_torch_at_l1_size():
    """The weight gradient at a full-size L1 cell (C2: 16 -> 16 on 32 x 96 x 160) against
    torch's own GPU fp32 convolution backward (size-independent bar: 1e-4 of the
    gradient's scale), and bit-identical across two calls (fixed-order partial sums)."""
    from leastereo_amd.training import conv3d_wgrad
    gen = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(1, 16, 32, 96, 160, device=DEV, generator=gen)
    dz = torch.randn(1, 16, 32, 96, 160, device=DEV, generator=gen)
    a = conv3d_wgrad(x, dz, 3)
    b = conv3d_wgrad(x, dz, 3)
    assert torch.equal(a, b)
    with torch.backends.cudnn.flags(enabled=True, deterministic=True, allow_tf32=False):
        r = torch.nn.grad.conv3d_weight(x.double().cpu(), (16, 16, 3, 3, 3), dz.double().cpu(), padding=1)
    err = float((a.double().cpu() - r).abs().max())
    assert err <= 1e-4 * float(r.abs().max()), err


def test_train_steps_match_torch():
    """train.py:150-158's step (train mode, smooth_l1, SGD) through two stacked ConvBR3d
    layers: parameters and running statistics after three steps match the same steps
    taken by torch's own modules in float64."""
    from leastereo_amd.training import ConvBR3d
    torch.manual_seed(0)
    ours = torch.nn.Sequential(ConvBR3d(8, 16, 3, 1, 1), ConvBR3d(16, 1, 3, 1, 1, bn=False, relu=False)).to(DEV)
    ref = torch.nn.Sequential(
        torch.nn.Conv3d(8, 16, 3, padding=1, bias=False), torch.nn.BatchNorm3d(16), torch.nn.ReLU(),
        torch.nn.Conv3d(16, 1, 3, padding=1, bias=False)).double()
    with torch.no_grad():
        ref[0].weight.copy_(ours[0].conv.weight.double().cpu())
        ref[3].weight.copy_(ours[1].conv.weight.double().cpu())
    opt = torch.optim.SGD(ours.parameters(), lr=0.05, momentum=0.9)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    ours.train()
    ref.train()
    gen = torch.Generator().manual_seed(11)
    for _ in range(3):
        x = torch.randn(2, 8, 4, 6, 40, generator=gen)
        t = torch.randn(2, 1, 4, 6, 40, generator=gen)
        opt.zero_grad()
        loss = F.smooth_l1_loss(ours(x.to(DEV)), t.to(DEV))
        loss.backward()
        opt.step()
        ropt.zero_grad()
        rloss = F.smooth_l1_loss(ref(x.double()), t.double())
        rloss.backward()
        ropt.step()
        assert abs(loss.item() - rloss.item()) <= 1e-5 * abs(rloss.item()) + 1e-7
    pairs = [(ours[0].conv.weight, ref[0].weight), (ours[0].bn.weight, ref[1].weight),
             (ours[0].bn.bias, ref[1].bias), (ours[0].bn.running_mean, ref[1].running_mean),
             (ours[0].bn.running_var, ref[1].running_var), (ours[1].conv.weight, ref[3].weight)]
    for a, r in pairs:
        assert torch.allclose(a.detach().double().cpu(), r.detach(), rtol=1e-4, atol=1e-5)
    assert int(ours[0].bn.num_batches_tracked) == int(ref[1].num_batches_tracked) == 3


@pytest.mark.parametrize("src,dst,ac", [
    ((16, 48, 80), (32, 96, 160), True),   # L2 -> L1 up-sampling (skip_model_3d.py:48)
    ((32, 96, 160), (16, 48, 80), True),   # L1 -> L2 down-sampling
    ((9, 7, 13), (5, 4, 7), True),         # odd sizes (scale_dimension's (n + 1) / 2)
    ((5, 4, 7), (9, 7, 13), True),
    ((4, 6, 10), (12, 18, 30), False),     # Disp's x3 (build_model_2d.py:53, align_corners=False)
    ((3, 1, 5), (3, 1, 5), True),          # identity axis, a single-plane axis
    ((1, 2, 3), (4, 1, 6), True),          # an axis of output size 1
])
def test_interpolate3d_backward_vs_fp64(src, dst, ac):
    from leastereo_amd.training import interpolate3d
    gen = torch.Generator().manual_seed(sum(src) + sum(dst))
    x = torch.randn((2, 3) + src, generator=gen)
    dy = torch.randn((2, 3) + dst, generator=gen)
    xr = x.double().requires_grad_(True)
    yr = F.interpolate(xr, size=dst, mode="trilinear", align_corners=ac)
    yr.backward(dy.double())
    xd = x.to(DEV).requires_grad_(True)
    y = interpolate3d(xd, dst, ac)
    y.backward(dy.to(DEV))
    torch.cuda.synchronize()
    _close(y, yr.detach(), "y")
    _close(xd.grad, xr.grad, "dx")


@pytest.mark.parametrize("b,d3,h3,w3,maxdisp", [(2, 8, 5, 7, 24), (1, 16, 4, 6, 48), (1, 6, 3, 4, 17)])
def test_disparity_regression_backward_vs_fp64(b, d3, h3, w3, maxdisp):
    """build_model_2d.py:52-57 then :33-42 (upsample, softmax(-x), sum d * p)."""
    from leastereo_amd.training import disparity_regression
    gen = torch.Generator().manual_seed(d3 * 7 + maxdisp)
    cost = 2 * torch.randn(b, 1, d3, h3, w3, generator=gen)
    dout = torch.randn(b, 3 * h3, 3 * w3, generator=gen)
    cr = cost.double().requires_grad_(True)
    u = F.interpolate(cr, [maxdisp, 3 * h3, 3 * w3], mode="trilinear", align_corners=False)
    p = F.softmax(-torch.squeeze(u, 1), dim=1)
    ref = torch.sum(p * torch.arange(maxdisp, dtype=torch.float64).view(1, maxdisp, 1, 1), 1)
    ref.backward(dout.double())
    cd = cost.to(DEV).requires_grad_(True)
    disp = disparity_regression(cd, maxdisp)
    disp.backward(dout.to(DEV))
    torch.cuda.synchronize()
    _close(disp, ref.detach(), "disp")
    _close(cd.grad, cr.grad, "dcost")


@pytest.mark.parametrize("b,c,h,w,maxdisp", [(2, 4, 3, 16, 24), (1, 32, 2, 12, 48), (1, 3, 2, 5, 30)])
def test_cost_volume_backward_vs_fp64(b, c, h, w, maxdisp):
    """retrain/LEAStereo.py:34-48 (D3 may exceed W: the last case)."""
    from leastereo_amd.training import build_cost_volume
    gen = torch.Generator().manual_seed(c * 5 + w)
    fl, fr = torch.randn(b, c, h, w, generator=gen), torch.randn(b, c, h, w, generator=gen)
    d3 = int(maxdisp / 3)
    dcost = torch.randn(b, 2 * c, d3, h, w, generator=gen)
    lr, rr = fl.double().requires_grad_(True), fr.double().requires_grad_(True)
    cost = lr.new_zeros(b, 2 * c, d3, h, w)
    for i in range(d3):
        if i > 0:
            cost[:, :c, i, :, i:] = lr[:, :, :, i:]
            cost[:, c:, i, :, i:] = rr[:, :, :, :-i]
        else:
            cost[:, :c, i, :, :] = lr
            cost[:, c:, i, :, :] = rr
    cost.backward(dcost.double())
    ld, rd = fl.to(DEV).requires_grad_(True), fr.to(DEV).requires_grad_(True)
    out = build_cost_volume(ld, rd, maxdisp)
    out.backward(dcost.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().double(), cost.detach())
    _close(ld.grad, lr.grad, "dleft")
    _close(rd.grad, rr.grad, "dright")


def test_matching_train_step_vs_reference_golden():
    """One train.py:150-156 step of the matching path -- cost volume (LEAStereo.py:34-48),
    newMatching in train mode (skip_model_3d.py:140-174), Disp (build_model_2d.py:52-57),
    smooth_l1 over the validity mask -- against the reference itself run in float64
    (tests/golden/train_step.npz, tools/gen_golden_train.py) at 96 x 192 D48.
    Bars: the reference's OWN fp32 step differs from its float64 step (train-mode BN over
    a batch of one, a sharp softmin: disparity 1.1e-2 px, gradients 0.3-9 % of their
    scale; ``noise/*`` in the fixture, measured by the generator); every quantity here
    must be within 3x that figure (plus 1e-4 of its scale, 1e-6 for the statistics)."""
    import numpy as np
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from leastereo_amd.training import cost_to_disparity_train
    from leastereo_amd.weights import seeded_normal
    from tests.golden_util import golden, state_dict
    g = golden("train_step")
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV)
    m.load_state_dict(state_dict(), strict=True)
    m = m.to(DEV)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm3d):
            mod.momentum = 1.0
    m.train()
    fl = torch.from_numpy(seeded_normal(301, (1, 32, 32, 64))).to(DEV).requires_grad_(True)
    fr = torch.from_numpy(seeded_normal(302, (1, 32, 32, 64))).to(DEV).requires_grad_(True)
    target = torch.from_numpy(seeded_normal(303, (1, 96, 192))).to(DEV) * 4 + 20
    disp = cost_to_disparity_train(m, fl, fr)
    mask = (target < 48) & (target > 0.001)
    loss = F.smooth_l1_loss(disp[mask], target[mask], reduction="mean")
    loss.backward()
    torch.cuda.synchronize()
    noise = {k[6:]: float(v) for k, v in g.items() if k.startswith("noise/")}
    derr = float((disp.detach().cpu().double() - torch.from_numpy(g["disp"]).double()).abs().max())
    assert derr <= 3 * noise["disp"] + 1e-4, (derr, noise["disp"])
    lrel = abs(loss.item() - float(g["loss"])) / abs(float(g["loss"]))
    assert lrel <= 3 * noise["loss"] + 1e-6, (lrel, noise["loss"])
    got = {"d_fea_l": fl.grad, "d_fea_r": fr.grad}
    params = dict(m.named_parameters())
    bufs = dict(m.named_buffers())
    for k in g:
        if k.startswith("grad/"):
            name = k[5:]
            t = params[name].grad
            got[k] = t[:8] if name in ("matching.conv1.conv.weight", "matching.conv2.conv.weight") else t
        elif k.startswith("mean/") or k.startswith("var/"):
            got[k] = bufs[k.split("/", 1)[1] + (".running_mean" if k.startswith("mean/") else ".running_var")]
    worst = {}
    for k, t in got.items():
        r = torch.from_numpy(np.asarray(g[k], dtype=np.float64))
        a = t.detach().double().cpu()
        assert a.shape == r.shape, k
        rel = float((a - r).abs().max()) / max(float(r.abs().max()), 1e-12)
        bar = 3 * noise[k] + (1e-6 if k.startswith(("mean/", "var/")) else 1e-4)
        worst[k] = (rel, noise[k])
        assert rel <= bar, f"{k}: {rel:.3e} > {bar:.3e} (reference fp32 noise {noise[k]:.3e})"
    print(f"disp max |d| {derr:.2e} px (reference fp32: {noise['disp']:.2e}); relative error / reference "
          "fp32 noise per tensor:", {k: f"{v[0]:.1e}/{v[1]:.1e}" for k, v in sorted(worst.items())})


# ---- the feature net's 2D ops (retrain/new_model_2d.py:93-95, models/operations_2d.py:31-47)
CASES_2D = [
    # B, cin, cout, H, W, kind, training, bn, relu
    (2, 16, 16, 12, 70, "2d", True, True, True),    # cell 3x3 op, ragged W segments
    (1, 3, 16, 20, 33, "2d", True, True, True),     # stem0 on the image (cin 3), dx wanted
    (1, 32, 32, 9, 17, "2d", False, True, True),    # stem2 shape, eval mode
    (1, 8, 8, 5, 130, "2d", True, True, False),     # 8-channel cell op, BN without ReLU
    (2, 16, 32, 29, 50, "s3", True, True, True),    # stem1, H/W not multiples of 3
    (1, 16, 32, 30, 48, "s3", True, True, True),
    (1, 5, 40, 7, 8, "s3", False, True, True),      # partial channel chunk, three cout blocks
]


@pytest.mark.parametrize("case", CASES_2D, ids=lambda c: "x".join(map(str, c[:5])) + f"-{c[5]}-t{int(c[6])}r{int(c[8])}")
def test_convbr2d_forward_backward_vs_fp64(case):
    """Conv2d 3x3 (stride 1 or 3, pad 1) -> BatchNorm2d -> ReLU on [B, C, 1, H, W] views,
    forward and every gradient against torch autograd in float64."""
    from leastereo_amd.training import _ConvBRFn
    b, cin, cout, h, w, kind, training, use_bn, relu = case
    stride = 3 if kind == "s3" else 1
    gen = torch.Generator().manual_seed(11 + cin * 7 + cout + h)
    x = torch.randn(b, cin, h, w, generator=gen)
    wt = torch.randn(cout, cin, 3, 3, generator=gen) * (2.0 / (cin * 9)) ** 0.5
    g = 1 + 0.2 * torch.randn(cout, generator=gen)
    bt = 0.1 * torch.randn(cout, generator=gen)
    rm = 0.1 * torch.randn(cout, generator=gen)
    rv = 1 + torch.rand(cout, generator=gen)
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    dy = torch.randn(b, cout, ho, wo, generator=gen)
    momentum, eps = 0.1, 1e-5
    xr = x.double().requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), bt.double().requires_grad_(True)
    rmr, rvr = rm.double().clone(), rv.double().clone()
    z = F.conv2d(xr, wr, stride=stride, padding=1)
    z = F.batch_norm(z, rmr, rvr, gr, br, training, momentum, eps)
    z = F.relu(z) if relu else z
    z.backward(dy.double())

    xd = x.to(DEV).unsqueeze(2).requires_grad_(True)
    wd = wt.to(DEV).requires_grad_(True)
    gd, bd = g.to(DEV).requires_grad_(True), bt.to(DEV).requires_grad_(True)
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    y = _ConvBRFn.apply(xd, wd, gd, bd, rmd, rvd, training, momentum, eps, use_bn, relu, kind)
    y.backward(dy.to(DEV).unsqueeze(2))
    torch.cuda.synchronize()
    _close(y.squeeze(2), z.detach(), "y")
    _close(xd.grad.squeeze(2), xr.grad, "dx")
    _close(wd.grad, wr.grad, "dw")
    _close(gd.grad, gr.grad, "dgamma")
    _close(bd.grad, br.grad, "dbeta")
    assert torch.allclose(rmd.cpu().double(), rmr, rtol=1e-5, atol=1e-6)
    assert torch.allclose(rvd.cpu().double(), rvr, rtol=1e-5, atol=1e-6)


def test_conv2d_wgrads_deterministic_at_c2_feature_size():
    """The feature net's weight gradients at C2's map size (stem2: 32 -> 32 on 192 x 320;
    stem1: 16 -> 32 stride 3 from 576 x 960) against float64 torch (1e-4 of the scale),
    bit-identical across two calls."""
    from leastereo_amd.training import conv2d_s3_backward, conv2d_wgrad
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(1, 32, 1, 192, 320, device=DEV, generator=gen)
    dz = torch.randn(1, 32, 1, 192, 320, device=DEV, generator=gen)
    a, b = conv2d_wgrad(x, dz), conv2d_wgrad(x, dz)
    assert torch.equal(a, b)
    r = torch.nn.grad.conv2d_weight(x[:, :, 0].double().cpu(), (32, 32, 3, 3), dz[:, :, 0].double().cpu(), padding=1)
    assert float((a.double().cpu() - r).abs().max()) <= 1e-4 * float(r.abs().max())
    xs = torch.randn(1, 16, 1, 576, 960, device=DEV, generator=gen)
    dzs = torch.randn(1, 32, 1, 192, 320, device=DEV, generator=gen)
    w = torch.randn(32, 16, 3, 3, device=DEV, generator=gen)
    (dx1, dw1), (dx2, dw2) = conv2d_s3_backward(xs, dzs, w, True, True), conv2d_s3_backward(xs, dzs, w, True, True)
    assert torch.equal(dw1, dw2) and torch.equal(dx1, dx2)
    r = torch.nn.grad.conv2d_weight(xs[:, :, 0].double().cpu(), (32, 16, 3, 3), dzs[:, :, 0].double().cpu(),
                                    stride=3, padding=1)
    assert float((dw1.double().cpu() - r).abs().max()) <= 1e-4 * float(r.abs().max())


def test_whole_model_train_step_vs_reference_golden():
    """train.py:150-158 through the drop-in's public API: ``model.train()``,
    ``disp = model(input1, input2)`` with inputs that require grad (train.py:136),
    smooth_l1 over the validity mask, ``loss.backward()`` -- the feature net twice (its own
    train-mode BN statistics per image), the cost volume, newMatching, Disp, every op on
    the HIP library -- against the reference model itself run in float64
    (tests/golden/train_step_full.npz, tools/gen_golden_train_full.py) at 96 x 192 D48.
    Bars: 3x the reference's own fp32-vs-fp64 difference per quantity (``noise/*``:
    disparity 4.6e-2 px, gradients 1.3-3.9 % of their scale) plus 1e-4 of the scale."""
    import numpy as np
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from leastereo_amd.weights import seeded_normal
    from tests.golden_util import golden, state_dict
    g = golden("train_step_full")
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV)
    m.load_state_dict(state_dict(), strict=True)
    m = m.to(DEV)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
            mod.momentum = 1.0
    m.train()
    left = torch.from_numpy(seeded_normal(311, (1, 3, 96, 192))).to(DEV).requires_grad_(True)
    right = torch.from_numpy(seeded_normal(312, (1, 3, 96, 192))).to(DEV).requires_grad_(True)
    target = torch.from_numpy(seeded_normal(313, (1, 96, 192))).to(DEV) * 4 + 20
    disp = m(left, right)
    mask = (target < 48) & (target > 0.001)
    loss = F.smooth_l1_loss(disp[mask], target[mask], reduction="mean")
    loss.backward()
    torch.cuda.synchronize()
    noise = {k[6:]: float(v) for k, v in g.items() if k.startswith("noise/")}
    derr = float((disp.detach().cpu().double() - torch.from_numpy(g["disp"]).double()).abs().max())
    assert derr <= 3 * noise["disp"] + 1e-4, (derr, noise["disp"])
    lrel = abs(loss.item() - float(g["loss"])) / abs(float(g["loss"]))
    assert lrel <= 3 * noise["loss"] + 1e-6, (lrel, noise["loss"])
    got = {"d_left_rows32": left.grad[:, :, :32]}
    params, bufs = dict(m.named_parameters()), dict(m.named_buffers())
    for k in g:
        if k.startswith("grad/"):
            name = k[5:]
            t = params[name].grad
            got[k] = t[:8] if name in ("matching.stem0.conv.weight", "matching.conv1.conv.weight") else t
        elif k.startswith("mean/") or k.startswith("var/"):
            got[k] = bufs[k.split("/", 1)[1] + (".running_mean" if k.startswith("mean/") else ".running_var")]
    worst = {}
    for k, t in got.items():
        r = torch.from_numpy(np.asarray(g[k], dtype=np.float64))
        a = t.detach().double().cpu()
        assert a.shape == r.shape, k
        rel = float((a - r).abs().max()) / max(float(r.abs().max()), 1e-12)
        bar = 3 * noise[k] + (1e-6 if k.startswith(("mean/", "var/")) else 1e-4)
        worst[k] = (rel, noise[k])
        assert rel <= bar, f"{k}: {rel:.3e} > {bar:.3e} (reference fp32 noise {noise[k]:.3e})"
    print(f"disp max |d| {derr:.2e} px (reference fp32: {noise['disp']:.2e}); relative error / reference "
          "fp32 noise per tensor:", {k: f"{v[0]:.1e}/{v[1]:.1e}" for k, v in sorted(worst.items())})


def test_whole_model_eval_mode_gradients_vs_oracle_fp64():
    """Gradients through the drop-in in eval mode (running-statistics BN, inputs that
    require grad: the differentiable path) against torch autograd of the oracle
    (oracle/torch_ref.py, the reference's aten op sequence) in float64 on the CPU, same
    weights and inputs, at 96 x 192 D48: disparity within 1e-3 px, the input and every
    parameter gradient within 2e-3 of its scale (eval mode has no batch-statistics
    amplification: the forward's fp32 noise is 5e-6 px)."""
    import numpy as np
    from oracle import torch_ref as ref
    from leastereo_amd.config import ARCH_DIR, LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from tests.golden_util import state_dict
    import os
    sd = state_dict()
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV).eval()
    gen = torch.Generator().manual_seed(31)
    left, right = torch.randn(1, 3, 96, 192, generator=gen), torch.randn(1, 3, 96, 192, generator=gen)
    dout = torch.randn(1, 96, 192, generator=gen)
    ld, rd = left.to(DEV).requires_grad_(True), right.to(DEV).requires_grad_(True)
    disp = m(ld, rd)
    disp.backward(dout.to(DEV))
    torch.cuda.synchronize()
    arch = {k: np.load(os.path.join(ARCH_DIR, f)) for k, f in (
        ("net_arch_fea", "feature_network_path.npy"), ("cell_arch_fea", "feature_genotype.npy"),
        ("net_arch_mat", "matching_network_path.npy"), ("cell_arch_mat", "matching_genotype.npy"))}
    sd64 = {k: torch.as_tensor(np.asarray(v)).double().requires_grad_(k.endswith(("conv.weight", "bn.weight",
                                                                                   "bn.bias")))
            if np.asarray(v).dtype.kind == "f" else torch.as_tensor(np.asarray(v)) for k, v in sd.items()}
    lr, rr = left.double().requires_grad_(True), right.double().requires_grad_(True)
    want = ref.leastereo_forward(sd64, lr, rr, 48, arch)
    want.backward(dout.double())
    assert float((disp.detach().cpu().double() - want.detach()).abs().max()) <= 1e-3
    params = dict(m.named_parameters())
    checked = 0
    for k, t in list(sd64.items()) + [("left", lr), ("right", rr)]:
        if not (isinstance(t, torch.Tensor) and t.requires_grad) or t.grad is None:
            continue
        got = (ld.grad if k == "left" else rd.grad if k == "right" else params[k].grad)
        assert got is not None, k
        r = t.grad
        err = float((got.detach().double().cpu() - r).abs().max())
        assert err <= 2e-3 * float(r.abs().max()) + 1e-9, f"{k}: {err:.3e} vs scale {float(r.abs().max()):.3e}"
        checked += 1
    assert checked > 300, checked


def test_whole_model_sgd_steps_then_eval_uses_updated_weights():
    """train.py's loop (zero_grad, forward in train mode, smooth_l1, backward, step) for
    three steps, then evaluation: the inference executors were built before training
    (an eval pass) and must see the optimizer's in-place updates (version counters)."""
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from tests.golden_util import state_dict
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV)
    m.load_state_dict(state_dict(), strict=True)
    m = m.to(DEV).eval()
    gen = torch.Generator().manual_seed(21)
    left = torch.randn(1, 3, 96, 192, generator=gen).to(DEV)
    right = torch.randn(1, 3, 96, 192, generator=gen).to(DEV)
    with torch.no_grad():
        before = m(left, right).clone()      # builds and caches the executors
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=1e-3, momentum=0.9)
    losses = []
    for _ in range(3):
        target = (torch.rand(1, 96, 192, generator=gen) * 40 + 1).to(DEV)
        opt.zero_grad()
        loss = F.smooth_l1_loss(m(left, right), target, reduction="mean")
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(v == v and abs(v) < 1e6 for v in losses), losses
    m.eval()
    with torch.no_grad():
        after = m(left, right)
        # the eval path equals the differentiable path in eval mode on the updated weights
        ld = left.clone().requires_grad_(True)
    with torch.enable_grad():
        diff_path = m(ld, right)
    assert not torch.equal(after, before)
    assert float((after - diff_path.detach()).abs().max()) <= 1e-3
