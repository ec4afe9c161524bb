"""GPU parity: the HIP path (through the C ABI) against the golden vectors of the
reference and against the CPU/torch oracle on the same seeded inputs.

Tolerances (floating point, BASELINE.json north_star: disparity within 1e-3 px
EPE of the PyTorch reference in fp32):
  cost volume            bit-exact (pure copy)
  ConvBR3d               |d| <= 1e-4 + 1e-4*|ref|  (fp32, K up to 3456, reassociated sums)
  trilinear resample     |d| <= 2e-6
  disparity regression   |d| <= 2e-5 px
  ConvBR2d / feature net |d| <= 1e-4 + 1e-4*|ref| (per op), 1e-4 (whole net vs golden)
  end to end             EPE <= 1e-3 px vs reference fp32 and fp64 disparities
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from leastereo_amd import _lib, kernels
from leastereo_amd.config import LEAStereoArgs, default_arch_args
from leastereo_amd.model import LEAStereo
from oracle import torch_ref as ref
from tests.golden_util import arch, c1_inputs, golden, meta, normal, state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = meta()["cases"]


def _cases(prefix):
    return sorted(k.split("/", 1)[1] for k in CASES if k.startswith(prefix + "/"))


@pytest.fixture(autouse=True, scope="module")
def _no_tf32():
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False


def _model(maxdisp):
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=maxdisp)), DEV)
    m.load_state_dict(state_dict(), strict=True)
    return m.to(DEV).eval()


# ------------------------------------------------------------------ per-op golden
@pytest.mark.parametrize("name", _cases("cost_volume"))
def test_cost_volume_golden(name):
    c = CASES["cost_volume/" + name]
    fl = normal(c["seeds"][0], c["shape"]).to(DEV)
    fr = normal(c["seeds"][1], c["shape"]).to(DEV)
    out = kernels.build_cost_volume(fl, fr, c["maxdisp"]).cpu().numpy()
    np.testing.assert_array_equal(out, golden("cost_volume")[name])


def _conv_params(module):
    sd = state_dict()
    w = sd[module + ".conv.weight"].to(DEV)
    packed = kernels.pack_conv_weight(w)
    if module + ".bn.weight" in sd and not module.endswith("last_3"):
        inv = 1.0 / torch.sqrt(sd[module + ".bn.running_var"] + 1e-5)
        scale = (inv * sd[module + ".bn.weight"]).to(DEV)
        shift = (sd[module + ".bn.bias"] - sd[module + ".bn.running_mean"] * inv * sd[module + ".bn.weight"]).to(DEV)
    else:
        scale = shift = None
    return w, packed, scale, shift


@pytest.mark.parametrize("name", _cases("convbr"))
def test_convbr_golden(name):
    c = CASES["convbr/" + name]
    x = normal(c["seed"], c["input"]).to(DEV)
    w, packed, scale, shift = _conv_params(c["module"])
    if not c["bn"]:
        scale = shift = None
    y = kernels.conv3d_bnrelu(x, packed, c["cout"], c["k"], scale, shift, relu=c["relu"])
    np.testing.assert_allclose(y.cpu().numpy(), golden("convbr")[name], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", _cases("resample"))
def test_resample_golden(name):
    c = CASES["resample/" + name]
    y = kernels.resample_trilinear(normal(c["seed"], c["input"]).to(DEV), c["size"], True)
    np.testing.assert_allclose(y.cpu().numpy(), golden("resample")[name], rtol=0, atol=2e-6)


@pytest.mark.parametrize("name", _cases("disp"))
def test_disparity_golden(name):
    c = CASES["disp/" + name]
    x = (normal(c["seed"], c["input"]) * c["gain"]).to(DEV)
    y = kernels.disparity_regression(x, c["maxdisp"])
    np.testing.assert_allclose(y.cpu().numpy(), golden("disp")[name], rtol=0, atol=2e-5)


# ------------------------------------------------------------- randomized vs torch fp32
@pytest.mark.parametrize("b,cin,cout,k,shape", [
    (1, 64, 32, 3, (6, 20, 70)), (2, 128, 64, 3, (5, 9, 40)), (1, 16, 16, 3, (7, 33, 17)),
    (1, 8, 8, 3, (3, 5, 100)), (1, 32, 1, 3, (4, 12, 64)), (1, 12, 20, 3, (3, 4, 5)),
    (1, 64, 16, 1, (3, 7, 11)), (2, 128, 32, 1, (4, 6, 130)), (1, 40, 8, 1, (2, 3, 5)),
    (1, 32, 64, 1, (1, 1, 1000)), (1, 256, 128, 1, (2, 5, 33)), (2, 12, 80, 3, (3, 6, 40)),
    (2, 16, 5, 3, (4, 9, 33)), (1, 7, 3, 3, (1, 4, 17)), (1, 8, 8, 3, (6, 40, 64))])
def test_conv_random_vs_torch(b, cin, cout, k, shape):
    g = torch.Generator().manual_seed(cin * 131 + cout)
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, k, k, k, generator=g) / np.sqrt(cin * k ** 3)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    res = torch.randn((b, cout) + shape, generator=g)
    refy = F.conv3d(x.double(), w.double(), None, 1, k // 2)
    refy = torch.relu(refy * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    refy = refy + res.double()
    out = res.to(DEV).clone()
    kernels.conv3d_bnrelu(x.to(DEV), kernels.pack_conv_weight(w.to(DEV)), cout, k, scale.to(DEV),
                          shift.to(DEV), relu=True, out=out, accumulate=True)
    np.testing.assert_allclose(out.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cin,cout,shape,acc", [(16, 16, (35, 96, 160), False),
                                                (16, 16, (35, 96, 160), True),
                                                (8, 8, (33, 48, 320), True),
                                                (32, 48, (9, 100, 326), False)])
def test_conv_two_plane_tiles_odd_depth(cin, cout, shape, acc):
    """Large volumes use 2 output planes per workgroup; odd D masks the last one.
    With ``acc`` the residual is prefetched into registers at workgroup start."""
    name = kernels.conv_kernel_name(1, cout, *shape, 3)
    # two output planes per workgroup: TD = 2, or the depth-paired tile (couts <= 8)
    assert name.endswith(", 2, 3, false>") or name.endswith(", 1, 4, false>"), name
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn((1, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    res = torch.randn((1, cout) + shape, generator=g)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    refy = F.conv3d(x.double(), w.double(), None, 1, 1)
    refy = torch.relu(refy * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    out = res.to(DEV).clone() if acc else None
    y = kernels.conv3d_bnrelu(x.to(DEV), kernels.pack_conv_weight(w.to(DEV)), cout, 3, scale.to(DEV),
                              shift.to(DEV), relu=True, out=out, accumulate=acc)
    if acc:
        refy = refy + res.double()
    np.testing.assert_allclose(y.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("c1,c2,cout,shape", [(64, 64, 64, (4, 10, 40)), (16, 12, 16, (3, 7, 33)),
                                              (4, 4, 8, (2, 3, 5))])
def test_conv_two_sources_is_cat(c1, c2, cout, shape):
    """conv(cat(x, x2)) without the cat (skip_model_3d.py:150,155)."""
    g = torch.Generator().manual_seed(c1 + c2)
    x = torch.randn((2, c1) + shape, generator=g)
    x2 = torch.randn((2, c2) + shape, generator=g)
    w = torch.randn(cout, c1 + c2, 3, 3, 3, generator=g) / np.sqrt((c1 + c2) * 27)
    refy = F.conv3d(torch.cat((x, x2), 1).double(), w.double(), None, 1, 1)
    y = kernels.conv3d_bnrelu(x.to(DEV), kernels.pack_conv_weight(w.to(DEV)), cout, 3, None, None,
                              relu=False, x2=x2.to(DEV))
    np.testing.assert_allclose(y.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("k,cin,cout,src,dst", [
    (1, 64, 8, (4, 6, 10), (8, 12, 20)),      # L1 -> L0 (cell10)
    (1, 32, 16, (8, 12, 20), (4, 6, 10)),     # L0 -> L1 (cell0/1/11)
    (1, 128, 16, (3, 5, 9), (5, 9, 17)),      # odd sizes up (2n-1)
    (1, 64, 32, (5, 9, 17), (3, 5, 9)),       # odd sizes down ((n+1)/2)
    (3, 32, 1, (4, 6, 40), (8, 12, 80)),      # head: Upsample + last_3
    (3, 16, 16, (5, 7, 9), (4, 5, 6))])       # generic size match
def test_conv_resampled_vs_torch(k, cin, cout, src, dst):
    g = torch.Generator().manual_seed(cin * 7 + k)
    x = torch.randn((2, cin) + src, generator=g)
    w = torch.randn(cout, cin, k, k, k, generator=g) / np.sqrt(cin * k ** 3)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    xi = F.interpolate(x.double(), dst, mode="trilinear", align_corners=True)
    refy = torch.relu(F.conv3d(xi, w.double(), None, 1, k // 2) * scale.double().view(1, -1, 1, 1, 1)
                      + shift.double().view(1, -1, 1, 1, 1))
    y = kernels.conv3d_bnrelu_resampled(x.to(DEV), dst, kernels.pack_conv_weight(w.to(DEV)), cout, k,
                                        scale.to(DEV), shift.to(DEV), relu=True)
    np.testing.assert_allclose(y.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cin,cin2,cout,shape,resid", [
    (2, 24, 0, 8, (8, 12, 20), False), (1, 48, 0, 16, (4, 6, 10), True),
    (2, 32, 16, 32, (5, 7, 12), False),     # virtual concat, D*H*W % 4 == 0
    (1, 64, 0, 48, (3, 5, 7), True),        # D*H*W odd: the vector form declines
    (3, 96, 32, 64, (2, 9, 20), False), (1, 8, 0, 16, (1, 1, 4), True)])
def test_conv1x1_vector_form_is_the_scalar_form(b, cin, cin2, cout, shape, resid):
    """lea_conv1x1_set_vector(1) (lane n owns NT consecutive voxels: vector loads and
    stores) stores exactly what the one-float-per-lane form stores, into a channel slice,
    with the residual epilogue and a second source; both against torch in float64."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(cin + cout + cin2)
    x = torch.randn((b, cin) + shape, device=DEV, generator=g)
    x2 = torch.randn((b, cin2) + shape, device=DEV, generator=g) if cin2 else None
    w = torch.randn(cout, cin + cin2, 1, 1, 1, device=DEV, generator=g) / np.sqrt(cin + cin2)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.1
    res = torch.randn((b, cout) + shape, device=DEV, generator=g) if resid else None
    base = torch.randn((b, cout + 8) + shape, device=DEV, generator=g)
    pw = kernels.pack_conv_weight(w)
    outs = []
    try:
        for on in (0, 1):
            assert lib.lea_conv1x1_set_vector(on) == 0
            y = base.clone()
            kernels.conv3d_bnrelu(x, pw, cout, 1, scale, shift, relu=True, out=y[:, 4:4 + cout], x2=x2,
                                  residual=res)
            outs.append(y)
    finally:
        lib.lea_conv1x1_set_vector(1)
    assert torch.equal(outs[0], outs[1])
    xin = torch.cat((x, x2), 1) if cin2 else x
    want = torch.relu(F.conv3d(xin.double(), w.double()) * scale.double().view(1, -1, 1, 1, 1)
                      + shift.double().view(1, -1, 1, 1, 1))
    if resid:
        want = want + res.double()
    np.testing.assert_allclose(outs[1][:, 4:4 + cout].cpu().double().numpy(), want.cpu().numpy(),
                               rtol=1e-4, atol=1e-4)
    assert torch.equal(outs[1][:, :4], base[:, :4]) and torch.equal(outs[1][:, 4 + cout:], base[:, 4 + cout:])


@pytest.mark.parametrize("cin,cout,src,dst", [
    (32, 32, (8, 12, 20), (4, 6, 10)),      # L0 -> L1 stacked share conv
    (64, 64, (5, 9, 17), (3, 5, 9)),        # L1 -> L2 stacked, odd sizes
    (24, 48, (6, 10, 14), (3, 5, 7)),       # padded 32-channel chunk, 48-row block
    (128, 16, (3, 5, 9), (5, 9, 17)),       # up-sampling, four chunks
    (8, 16, (4, 3, 1), (7, 5, 6))])         # width 1 -> 6 (the W pair clamps to one word)
def test_resampled_1x1_gather_matches_staged_engine(cin, cout, src, dst):
    """The gather-GEMM (lea_conv3d_set_rs_gather(1), the default for resampled 1x1 convs)
    stores what the register-staged engine stores (up to the MFMA summation order), into
    a channel slice, with and without the accumulate epilogue."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(cin + cout)
    x = torch.randn((2, cin) + src, device=DEV, generator=g)
    w = torch.randn(cout, cin, 1, 1, 1, device=DEV, generator=g) / np.sqrt(cin)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.1
    r = torch.randn((2, cout + 8) + dst, device=DEV, generator=g)
    pw = kernels.pack_conv_weight(w)
    outs = []
    try:
        for on in (0, 1):
            assert lib.lea_conv3d_set_rs_gather(on) == 0
            for acc in (False, True):
                y = r.clone()
                kernels.conv3d_bnrelu_resampled(x, dst, pw, cout, 1, scale, shift, True, y[:, 3:3 + cout], acc)
                outs.append(y)
    finally:
        lib.lea_conv3d_set_rs_gather(1)
    for a, b in ((outs[0], outs[2]), (outs[1], outs[3])):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-5, atol=1e-5)
    xi = F.interpolate(x.double(), dst, mode="trilinear", align_corners=True)
    want = torch.relu(F.conv3d(xi, w.double()) * scale.double().view(1, -1, 1, 1, 1)
                      + shift.double().view(1, -1, 1, 1, 1)) + r[:, 3:3 + cout].double()
    np.testing.assert_allclose(outs[3][:, 3:3 + cout].cpu().double().numpy(), want.cpu().numpy(),
                               rtol=1e-4, atol=1e-4)
    assert torch.equal(outs[3][:, :3], r[:, :3]) and torch.equal(outs[3][:, 3 + cout:], r[:, 3 + cout:])


@pytest.mark.parametrize("cout,cin,shape", [(1, 32, (6, 20, 130)), (2, 12, (3, 9, 64)),
                                            (1, 5, (2, 3, 7))])
def test_conv_small_cout_valu_engine(cout, cin, shape):
    """last_3-like convs (cout <= 2) run on the VALU engine."""
    g = torch.Generator().manual_seed(cout * 100 + cin)
    x = torch.randn((2, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    assert kernels.conv_kernel_name(2, cout, *shape, 3).startswith("conv3d_valu_kernel")
    refy = F.conv3d(x.double(), w.double(), None, 1, 1)
    y = kernels.conv3d_bnrelu(x.to(DEV), kernels.pack_conv_weight(w.to(DEV)), cout, 3, None, None,
                              relu=False)
    np.testing.assert_allclose(y.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cout,cin,src,dst", [(1, 32, (4, 6, 10), (8, 12, 20)),
                                              (2, 8, (3, 5, 9), (5, 9, 17)),
                                              (1, 32, (32, 96, 160), (64, 192, 320))])
def test_head_tapsum_upsample_vs_torch(cout, cin, src, dst):
    """last_3(Upsample(y)) via per-tap partial sums == conv3d(interpolate(y))."""
    g = torch.Generator().manual_seed(cout * 31 + cin)
    y = torch.randn((1, cin) + src, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    taps = w.permute(0, 2, 3, 4, 1).reshape(cout * 27, cin, 1, 1, 1).contiguous()
    q = kernels.conv3d_bnrelu(y.to(DEV), kernels.pack_conv_weight(taps.to(DEV)), cout * 27, 1,
                              None, None, relu=False)
    out = kernels.tapsum_upsample(q, cout, dst).cpu().double()
    yd = y.to(DEV).double() if src[0] > 8 else y.double()
    refy = F.conv3d(F.interpolate(yd, dst, mode="trilinear", align_corners=True),
                    w.to(yd.device).double(), None, 1, 1).cpu()
    np.testing.assert_allclose(out.numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cout,src,dst", [(1, 1, (32, 96, 160), (64, 192, 320)), (2, 2, (3, 5, 9), (5, 9, 17)),
                                           (1, 1, (4, 13, 7), (8, 26, 14)), (1, 1, (16, 48, 252), (32, 96, 504))])
def test_head_tapsum_rows_pass_is_the_gather_pass(b, cout, src, dst):
    """The fused tap-sum head (passes 1 + 2 in one launch, the default since r05), the
    row-staged pass 2 after pass 1 and the per-row gather pass produce identical bits, f32
    and bf16 (c8) partial sums alike; a non-float4 f32 layout too (odd W)."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(13)
    q = torch.randn((b, 27 * cout) + src, generator=g).to(DEV)
    qc = kernels.to_c8(torch.cat([q, torch.zeros((b, (-27 * cout) % 8) + src, device=DEV)], 1))
    out = {}
    for on in (2, 1, 0):
        assert lib.lea_tapsum_set_rows(on) == 0
        try:
            out[on] = (kernels.tapsum_upsample(q, cout, dst), kernels.tapsum_upsample_bf16(qc, cout, dst))
        finally:
            lib.lea_tapsum_set_rows(2)
    for on in (1, 0):
        assert torch.equal(out[2][0], out[on][0]) and torch.equal(out[2][1], out[on][1]), on
    assert not torch.isnan(out[2][0]).any()


def test_resample_affine_relu_epilogue_into_slice():
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 8, 4, 6, 10, generator=g)
    scale = torch.rand(8, generator=g) + 0.5
    shift = torch.randn(8, generator=g)
    big = torch.zeros(2, 24, 8, 12, 20, device=DEV)
    kernels.resample_trilinear(x.to(DEV), (8, 12, 20), True, big[:, 8:16], scale.to(DEV),
                               shift.to(DEV), relu=True)
    refy = torch.relu(F.interpolate(x, (8, 12, 20), mode="trilinear", align_corners=True)
                      * scale.view(1, -1, 1, 1, 1) + shift.view(1, -1, 1, 1, 1))
    np.testing.assert_allclose(big[:, 8:16].cpu().numpy(), refy.numpy(), atol=1e-5, rtol=0)
    assert big[:, :8].abs().sum().item() == 0 and big[:, 16:].abs().sum().item() == 0


def test_conv_channel_slices():
    """Input and output as channel slices of larger tensors (the free cat)."""
    g = torch.Generator().manual_seed(7)
    big_in = torch.randn(2, 48, 4, 6, 70, generator=g).to(DEV)
    x = big_in[:, 8:24]
    w = (torch.randn(16, 16, 3, 3, 3, generator=g) / 10).to(DEV)
    big_out = torch.zeros(2, 64, 4, 6, 70, device=DEV)
    kernels.conv3d_bnrelu(x, kernels.pack_conv_weight(w), 16, 3, None, None, relu=False,
                          out=big_out[:, 32:48])
    refy = F.conv3d(x.cpu().double(), w.cpu().double(), None, 1, 1)
    np.testing.assert_allclose(big_out[:, 32:48].cpu().double().numpy(), refy.numpy(), atol=1e-4, rtol=1e-4)
    assert big_out[:, :32].abs().sum().item() == 0 and big_out[:, 48:].abs().sum().item() == 0


def test_resample_vs_torch_random_sizes():
    g = torch.Generator().manual_seed(3)
    for src, dst in [((5, 9, 13), (3, 5, 7)), ((4, 6, 8), (8, 12, 16)), ((32, 96, 160), (64, 192, 320)),
                     ((3, 3, 3), (1, 1, 1)), ((1, 4, 5), (2, 7, 9)),
                     ((2, 2000, 40), (3, 3, 40)), ((16, 48, 80), (32, 96, 160))]:
        x = torch.randn((2, 3) + src, generator=g)
        for ac in (True, False):
            refy = F.interpolate(x, dst, mode="trilinear", align_corners=ac)
            y = kernels.resample_trilinear(x.to(DEV), dst, ac).cpu()
            np.testing.assert_allclose(y.numpy(), refy.numpy(), atol=3e-6, rtol=0)


@pytest.mark.parametrize("src,dst,ac,epi,ch", [
    ((32, 96, 160), (64, 192, 320), True, True, 3), ((16, 48, 80), (32, 96, 160), True, False, 3),
    ((5, 9, 13), (3, 5, 8), False, True, 3), ((4, 6, 8), (8, 12, 16), False, False, 3),
    ((3, 70, 9), (6, 141, 20), True, True, 3), ((8, 40, 100), (4, 20, 52), True, False, 3),
    ((16, 48, 80), (32, 96, 160), False, True, 3), ((40, 24, 36), (13, 48, 72), True, False, 3),
    ((48, 20, 40), (24, 40, 80), True, True, 16), ((9, 33, 20), (19, 64, 40), False, False, 24)])
def test_resample_kernels_are_bit_identical(src, dst, ac, epi, ch):
    """The separable resample (W-lerped source rows in LDS, the default for 16-byte output
    rows), the row-staged and the gather kernels give the same bits -- trilerp's expression
    tree in each -- with and without the BN/ReLU epilogue, up- and down-sampling, ragged
    row blocks (H 141), 3 to 24 channels, and match torch."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(sum(dst))
    x = torch.randn((2, ch) + src, generator=g)
    scale = (torch.rand(ch, generator=g) + 0.5).to(DEV) if epi else None
    shift = (torch.randn(ch, generator=g) * 0.1).to(DEV) if epi else None
    outs = []
    try:
        for mode in (0, 1, 2):
            assert lib.lea_resample_set_mode(mode) == 0
            outs.append(kernels.resample_trilinear(x.to(DEV), dst, ac, None, scale, shift, relu=epi).cpu())
    finally:
        lib.lea_resample_set_mode(0)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    want = F.interpolate(x, dst, mode="trilinear", align_corners=ac)
    if epi:
        want = torch.relu(want * scale.cpu().view(1, -1, 1, 1, 1) + shift.cpu().view(1, -1, 1, 1, 1))
    np.testing.assert_allclose(outs[0].numpy(), want.numpy(), atol=3e-6, rtol=0)


def test_disparity_vs_oracle_sizes():
    g = torch.Generator().manual_seed(5)
    for shape, md in [((1, 1, 64, 12, 20), 192), ((2, 1, 88, 5, 9), 264), ((1, 1, 16, 7, 4), 48)]:
        x = torch.randn(shape, generator=g) * 3
        refd = ref.disp_forward(x.double(), md)
        y = kernels.disparity_regression(x.to(DEV), md).cpu()
        assert torch.isfinite(y).all()
        # fp32 sums over maxdisp terms: error grows ~ md * 2^-24 * disparity; bar is 1e-3 px EPE
        err = np.abs(y.double().numpy() - refd.numpy())
        assert err.max() < 2e-3 and err.mean() < 1e-4, (err.max(), err.mean())


@pytest.mark.parametrize("shape,md", [((1, 1, 64, 12, 20), 192), ((2, 1, 32, 9, 13), 96), ((1, 1, 16, 7, 4), 48),
                                      ((1, 1, 8, 5, 6), 24), ((1, 1, 88, 4, 90), 264), ((2, 1, 4, 1, 3), 12)])
def test_disparity_register_form_matches_the_lds_form(shape, md):
    """The row-staged disparity kernel (the default: source rows H-lerped into LDS, two passes
    over the planes), the register kernel (D3 plane values in registers, compile-time depth
    axis, softmin shifted by the smallest plane value) and the online-softmin LDS kernel
    agree to fp32 summation noise, f32 and fast-exp alike, and all meet the oracle at the
    1e-3 px bar."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(shape, generator=g) * 3
    refd = ref.disp_forward(x.double(), md).numpy()
    for fast in (False, True):
        out = {}
        for on in (4, 3, 2, 1, 0):
            assert lib.lea_disparity_set_register_form(on) == 0
            try:
                out[on] = kernels.disparity_regression(x.to(DEV), md, fast).cpu().double().numpy()
            finally:
                lib.lea_disparity_set_register_form(4)
            err = np.abs(out[on] - refd)
            assert err.max() < 2e-3 and err.mean() < 1e-4, (fast, on, err.max(), err.mean())
        assert np.abs(out[1] - out[0]).max() < 1e-3 and np.abs(out[2] - out[1]).max() < 1e-3
        # the three-row staging (r06) forms the two-row kernel's LDS values: same bits
        assert np.array_equal(out[3], out[2]), np.abs(out[3] - out[2]).max()
        # D3 exponentials per pixel (form 4, the default): products of exp((m - v_k) / 3) for
        # the x3 depth up-sampling; a few ulp per softmin term from the per-od exponentials,
        # the same fp32 noise as between the other forms (each also meets the oracle bar above)
        assert np.abs(out[4] - out[3]).max() < 1e-3, np.abs(out[4] - out[3]).max()


@pytest.mark.parametrize("b,c,cout,maxdisp,hw", [(2, 32, 32, 48, (12, 40)), (1, 4, 16, 27, (5, 7)),
                                                  (1, 32, 32, 192, (30, 100)), (1, 8, 48, 9, (9, 18))])
def test_costvolume_stem0_is_bit_identical(b, c, cout, maxdisp, hw):
    """stem0 reading the cost volume in place == building it, then convolving."""
    g = torch.Generator().manual_seed(c + cout + maxdisp)
    fl = torch.randn((b, c) + hw, generator=g).to(DEV)
    fr = torch.randn((b, c) + hw, generator=g).to(DEV)
    w = (torch.randn(cout, 2 * c, 3, 3, 3, generator=g) / np.sqrt(2 * c * 27)).to(DEV)
    scale = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    packed = kernels.pack_conv_weight(w)
    want = kernels.conv3d_bnrelu(kernels.build_cost_volume(fl, fr, maxdisp), packed, cout, 3, scale,
                                 shift, relu=True)
    got = kernels.conv3d_bnrelu_costvolume(fl, fr, maxdisp, packed, cout, scale, shift, relu=True)
    assert torch.equal(got, want)
    refy = F.conv3d(ref.build_cost_volume(fl.cpu().double(), fr.cpu().double(), maxdisp),
                    w.cpu().double(), None, 1, 1)
    refy = torch.relu(refy * scale.cpu().double().view(1, -1, 1, 1, 1)
                      + shift.cpu().double().view(1, -1, 1, 1, 1))
    np.testing.assert_allclose(got.cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


# ------------------------------------------------------------------ 2D feature net
@pytest.mark.parametrize("b,cin,cout,hw,res", [
    (2, 3, 16, (96, 192), None), (1, 32, 32, (37, 53), "acc"), (2, 16, 48, (24, 40), "res"),
    (1, 8, 8, (5, 3), "res"), (3, 12, 24, (17, 100), None), (1, 64, 64, (20, 33), "acc")])
def test_conv2d_random_vs_torch(b, cin, cout, hw, res):
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn((b, cin) + hw, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + hw, generator=g)
    refy = F.conv2d(x.double(), w.double(), None, 1, 1)
    refy = torch.relu(refy * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1))
    if res:
        refy = refy + r.double()
    out = r.to(DEV).clone().unsqueeze(2) if res == "acc" else None
    y = kernels.conv2d_bnrelu(x.to(DEV).unsqueeze(2), kernels.pack_conv2d_weight(w.to(DEV)), cout,
                              scale.to(DEV), shift.to(DEV), relu=True, out=out,
                              accumulate=res == "acc",
                              residual=r.to(DEV).unsqueeze(2) if res == "res" else None)
    np.testing.assert_allclose(y.squeeze(2).cpu().double().numpy(), refy.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cin,cout,hw,res", [
    (2, 8, 8, (192, 320), "acc"), (2, 8, 16, (192, 320), None), (2, 16, 16, (96, 160), "res"),
    (2, 16, 32, (96, 160), "slice"), (1, 3, 16, (31, 45), None), (1, 12, 24, (17, 100), "acc"),
    (2, 5, 20, (9, 70), "res"), (1, 16, 8, (1, 1), None), (3, 4, 32, (33, 31), "slice")])
def test_conv2d_few_channel_tile_vs_torch(b, cin, cout, hw, res):
    """The few-channel 2D tile (cin <= 16, cout <= 32: the feature net's cell ops, r04) and
    the DMA / MFMA engine it replaces there, against float64 torch: the 1/3 and 1/6
    resolution cell shapes, ragged tiles, cin not a multiple of 4, the cell-sum epilogues
    (accumulate, residual) and an output slice of a wider tensor (the cell's channel slot)."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin * 11 + cout + hw[1])
    x = torch.randn((b, cin) + hw, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + hw, generator=g)
    refy = F.conv2d(x.double(), w.double(), None, 1, 1)
    refy = torch.relu(refy * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1))
    if res in ("acc", "res"):
        refy = refy + r.double()
    pw = kernels.pack_conv2d_weight(w.to(DEV))
    ys = {}
    try:
        for small in (1, 0):
            assert lib.lea_conv2d_set_small(small) == 0
            name = kernels.conv2d_kernel_name(b, cout, hw[0], hw[1], cin)
            assert name.startswith("conv2d_small_kernel<") == bool(small), name
            big = torch.full((b, cout + 16, 1) + hw, 7.0, device=DEV)
            out = (r.to(DEV).clone().unsqueeze(2) if res == "acc" else
                   big[:, 8:8 + cout] if res == "slice" else None)
            y = kernels.conv2d_bnrelu(x.to(DEV).unsqueeze(2), pw, cout, scale.to(DEV), shift.to(DEV),
                                      relu=True, out=out, accumulate=res == "acc",
                                      residual=r.to(DEV).unsqueeze(2) if res == "res" else None)
            if res == "slice":
                assert torch.all(big[:, :8] == 7.0) and torch.all(big[:, 8 + cout:] == 7.0)
            ys[small] = y.squeeze(2).cpu().double().numpy()
    finally:
        lib.lea_conv2d_set_small(1)
    for small, y in ys.items():
        np.testing.assert_allclose(y, refy.numpy(), rtol=1e-4, atol=1e-4, err_msg=f"small={small}")


@pytest.mark.parametrize("b,cin,cout,hw", [(2, 16, 32, (96, 192)), (1, 5, 20, (31, 46)),
                                           (1, 16, 32, (4, 3))])
def test_conv2d_stride3_vs_torch(b, cin, cout, hw):
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn((b, cin) + hw, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    refy = F.conv2d(x.double(), w.double(), None, 3, 1)
    refy = torch.relu(refy * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1))
    y = kernels.conv2d_s3_bnrelu(x.to(DEV).unsqueeze(2), w.to(DEV), scale.to(DEV), shift.to(DEV))
    assert y.shape[3:] == refy.shape[2:]
    np.testing.assert_allclose(y.squeeze(2).cpu().double().numpy(), refy.numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("b,cin,c,hw,res", [
    (2, 8, 8, (192, 320), True), (2, 16, 16, (96, 160), True), (1, 8, 8, (33, 70), False),
    (3, 5, 16, (17, 9), True), (1, 12, 8, (1, 1), False)])
def test_conv2d_pair_is_the_two_convs(b, cin, c, hw, res):
    """lea_conv2d_bnrelu_pair (a feature cell's two ops on s0 in one launch, r04): both halves
    equal their own lea_conv2d_bnrelu bit for bit -- the first with the residual (the skip
    term), the second without -- into two non-adjacent channel slots of one cat buffer, the
    slot between and the edges untouched."""
    g = torch.Generator().manual_seed(cin * 7 + c + hw[1])
    x = torch.randn((b, cin, 1) + hw, generator=g).to(DEV)
    w = (torch.randn(2 * c, cin, 3, 3, generator=g) / np.sqrt(cin * 9)).to(DEV)
    scale = (torch.rand(2 * c, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(2 * c, generator=g) * 0.1).to(DEV)
    r = torch.randn((b, c, 1) + hw, generator=g).to(DEV) if res else None
    buf = torch.full((b, 4 * c, 1) + hw, 7.0, device=DEV)
    kernels.conv2d_bnrelu_pair(x, kernels.pack_conv2d_weight(w), c, 2 * c, scale, shift, True,
                               buf[:, 0:c], buf[:, 2 * c:3 * c], r)
    y0 = kernels.conv2d_bnrelu(x, kernels.pack_conv2d_weight(w[:c].contiguous()), c, scale[:c].contiguous(),
                               shift[:c].contiguous(), relu=True, residual=r)
    y1 = kernels.conv2d_bnrelu(x, kernels.pack_conv2d_weight(w[c:].contiguous()), c, scale[c:].contiguous(),
                               shift[c:].contiguous(), relu=True)
    assert torch.equal(buf[:, 0:c], y0) and torch.equal(buf[:, 2 * c:3 * c], y1)
    assert torch.all(buf[:, c:2 * c] == 7.0) and torch.all(buf[:, 3 * c:] == 7.0)


def test_feature_net_pair_launch_is_bit_identical():
    """The feature executor with each cell's two s0 ops as one launch (the default) and as two
    launches (FeatureExecutor.PAIR_S0 = False) give the same feature maps bit for bit."""
    from leastereo_amd import executor
    m = _model(48)
    x = normal(78, (2, 3, 96, 192)).to(DEV)
    outs = {}
    old = executor.FeatureExecutor.PAIR_S0
    try:
        for pair in (True, False):
            executor.FeatureExecutor.PAIR_S0 = pair
            m.feature._executor = None
            with torch.no_grad():
                outs[pair] = m.feature(x)
            assert bool(m.feature.executor().s0_pair) == pair
    finally:
        executor.FeatureExecutor.PAIR_S0 = old
        m.feature._executor = None
    assert torch.equal(outs[True], outs[False])


def test_feature_net_golden():
    """HIP feature net vs the reference's own feature map (e2e fixture)."""
    m = _model(48)
    c = CASES["e2e/b1_h96_w192_md48"]
    x = normal(c["seeds"][0], (1, 3, 96, 192)).to(DEV)
    with torch.no_grad():
        f = m.feature(x)
    np.testing.assert_allclose(f.cpu().numpy(), golden("e2e")["b1_h96_w192_md48/fea_l"],
                               rtol=1e-4, atol=1e-4)


def test_feature_net_vs_oracle_c1_size():
    """288x576 (config 1 crop), batch 2: HIP feature net vs the oracle on the GPU."""
    m = _model(96)
    x = normal(77, (2, 3, 288, 576)).to(DEV)
    sd = {k: v.to(DEV) for k, v in state_dict().items()}
    with torch.no_grad():
        f = m.feature(x)
        a = arch()
        want = ref.feature_forward(sd, x, a["net_arch_fea"], a["cell_arch_fea"])
    assert f.shape == want.shape
    np.testing.assert_allclose(f.cpu().numpy(), want.cpu().numpy(), rtol=1e-3, atol=1e-3)


# ----------------------------------------------------------------------- end to end
@pytest.mark.parametrize("name", _cases("e2e"))
def test_e2e_golden(name):
    c = CASES["e2e/" + name]
    shape = (c["batch"], 3, c["height"], c["width"])
    left, right = normal(c["seeds"][0], shape).to(DEV), normal(c["seeds"][1], shape).to(DEV)
    m = _model(c["maxdisp"])
    g = golden("e2e")
    with torch.no_grad():
        if name + "/matching" in g:
            fl, fr = m.feature(left), m.feature(right)
            mat = m.matching(kernels.build_cost_volume(fl, fr, c["maxdisp"]))
            np.testing.assert_allclose(mat.cpu().numpy(), g[name + "/matching"], rtol=1e-3, atol=1e-3)
        disp = m(left, right).cpu()
    assert disp.shape == g[name + "/disp32"].shape
    e32 = ref.epe(disp, torch.from_numpy(g[name + "/disp32"]))
    e64 = ref.epe(disp, torch.from_numpy(g[name + "/disp64"]))
    assert e32 < 1e-3 and e64 < 1e-3, (e32, e64)


def test_c1_sceneflow_pair_vs_reference():
    """Config 1 (SceneFlow 0001, predict.py preprocessing, 288x576 D96) on the HIP
    model vs the reference model's disparity for the same inputs."""
    from leastereo_amd import predict as P
    c = meta()["c1"]
    left, right = c1_inputs()
    m = _model(c["maxdisp"])
    with torch.no_grad():
        d = m(left.to(DEV), right.to(DEV)).cpu().numpy()
    disp = P.crop_output(d, *c["full_hw"], *c["crop_hw"])
    assert ref.epe(torch.from_numpy(disp), torch.from_numpy(golden("c1_sceneflow")["disp"])) < 1e-3


def test_predict_cli_runs_on_a_list(tmp_path):
    """predict.py's list loop end to end on PNG files (sceneflow layout)."""
    from PIL import Image
    from leastereo_amd import predict as P
    g = golden("c1_sceneflow")
    for side in ("left", "right"):
        d = tmp_path / "frames_finalpass" / "S" / side
        d.mkdir(parents=True)
        Image.fromarray(g[side + "_u8"][:96, :192]).save(d / "0001.png")
    (tmp_path / "list.txt").write_text("S/left/0001.png\n")
    # a DataParallel-style checkpoint ('module.' keys), as predict.py:55-65 loads
    torch.save({"state_dict": {"module." + k: v for k, v in state_dict().items()}},
               tmp_path / "ckpt.pth")
    rc = P.main(["--sceneflow=1", "--maxdisp=48", "--crop_height=96", "--crop_width=192",
                 f"--data_path={tmp_path}/", f"--test_list={tmp_path}/list.txt",
                 f"--save_path={tmp_path}/out/", f"--resume={tmp_path}/ckpt.pth"])
    assert rc == 0
    out = np.load(tmp_path / "out" / "0.npy")
    assert out.shape == (96, 192) and np.isfinite(out).all()
    # the reference's turbo PNG of the prediction (predict.py:240,246-247)
    png = np.asarray(Image.open(tmp_path / "out" / "0.png"))
    assert png.shape[:2] == (96, 192)


def test_predict_cli_satellite_branch(tmp_path):
    """predict.py's --satellite loop (predict.py:187-211,258-264): <name>.png holds the
    disparity as skimage writes a float image, <name>_in.png the cropped left input."""
    from PIL import Image
    from leastereo_amd import predict as P
    g = golden("c1_sceneflow")
    d = tmp_path / "sat" / "tile_01"
    d.mkdir(parents=True)
    Image.fromarray(g["left_u8"][:90, :180]).save(d / "satiml.png")
    Image.fromarray(g["right_u8"][:90, :180]).save(d / "satimr.png")
    (tmp_path / "list.txt").write_text("tile_01\n")
    out = tmp_path / "out"
    out.mkdir()
    torch.save({"state_dict": state_dict()}, tmp_path / "ckpt.pth")
    rc = P.main(["--satellite=1", "--maxdisp=48", "--crop_height=96", "--crop_width=192",
                 f"--data_path={tmp_path}/sat/", f"--test_list={tmp_path}/list.txt",
                 f"--save_path={out}/", f"--resume={tmp_path}/ckpt.pth"])
    assert rc == 0
    m = _model(48)
    left, right, h, w = P.load_transform(*P.load_images(d / "satiml.png", d / "satimr.png"), 96, 192)
    with torch.no_grad():
        disp = P.crop_output(m(left, right).cpu().numpy(), h, w, 96, 192)
    assert disp.shape == (90, 180)
    np.testing.assert_array_equal(np.asarray(Image.open(out / "tile_01.png")), P.float_to_u8(disp))
    inp = np.asarray(Image.open(out / "tile_01_in.png"))
    assert inp.shape == (96, 192, g["left_u8"].shape[2])  # every layer of the image (predict.py:128-141)
    np.testing.assert_array_equal(inp, P.float_to_u8(P.crop_image(g["left_u8"][:90, :180], 96, 192)))


def test_batch_rows_are_independent():
    """A B=2 batch equals the two B=1 runs bit for bit (feature net, cost volume,
    matching, disparity): no cross-pair mixing, batch-invariant arithmetic."""
    m = _model(48)
    left = normal(901, (2, 3, 96, 192)).to(DEV)
    right = normal(902, (2, 3, 96, 192)).to(DEV)
    with torch.no_grad():
        fl, fr = m.feature(left), m.feature(right)
        both = m.disp(m.matching(kernels.build_cost_volume(fl, fr, 48)))
        one = torch.cat([m.disp(m.matching(kernels.build_cost_volume(fl[i:i + 1], fr[i:i + 1], 48)))
                         for i in range(2)])
        assert torch.equal(both, one)
        e2e_both = m(left, right)
        e2e_one = torch.cat([m(left[i:i + 1], right[i:i + 1]) for i in range(2)])
    assert torch.equal(e2e_both, e2e_one)


@pytest.mark.parametrize("b,h,w,maxdisp,oracle_dev", [(1, 1008, 1512, 264, "cpu"),
                                                      (2, 384, 1248, 192, "cpu")])
def test_large_configs_vs_torch_oracle(b, h, w, maxdisp, oracle_dev):
    """Config 5 (Middlebury 1008x1512, D264 -- D256 is illegal in the reference) and
    config 3's KITTI shape (384x1248 D192, here fp32, batch 2): HIP vs the oracle,
    EPE <= 1e-3 px per pair.  (MIOpen's 3D convs at these sizes take minutes, so
    the oracle runs on the host CPU.)"""
    m = _model(maxdisp)
    left = normal(4321 + h, (b, 3, h, w))
    right = normal(4322 + h, (b, 3, h, w))
    sd = {k: v.to(oracle_dev) for k, v in state_dict().items()}
    with torch.no_grad():
        disp = m(left.to(DEV), right.to(DEV)).cpu()
        want = ref.leastereo_forward(sd, left.to(oracle_dev), right.to(oracle_dev), maxdisp,
                                     arch()).cpu()
    assert disp.shape == (b, h, w) and torch.isfinite(disp).all()
    for i in range(b):
        assert ref.epe(disp[i], want[i]) < 1e-3


def test_full_size_c2_vs_torch_oracle():
    """576x960 D192 (the benchmark configuration): HIP vs the oracle's torch
    restatement in fp32 on the host CPU (MIOpen's 3D convs at this size take
    minutes), EPE <= 1e-3 px."""
    m = _model(192)
    left = normal(1234, (1, 3, 576, 960))
    right = normal(1235, (1, 3, 576, 960))
    with torch.no_grad():
        disp = m(left.to(DEV), right.to(DEV)).cpu()
        want = ref.leastereo_forward(state_dict(), left, right, 192, arch())
    assert torch.isfinite(disp).all()
    assert float(disp.min()) >= 0.0 and float(disp.max()) <= 191.0
    assert ref.epe(disp.cpu(), want.cpu()) < 1e-3


@pytest.mark.parametrize("precision,bound", [("f32", 1e-3), ("bf16", 0.25)])
def test_stem0_fallback_shape_vs_torch_oracle(precision, bound):
    """W3 = 66 (W = 198, legal: 66 -> 33 -> 17 -> 33 -> 66) is not a multiple of 4, so the
    f32 executor runs stem0 as the 3D conv on the in-place cost volume instead of the
    factored form (float4 rows); bf16 keeps the factored form.  Both vs the oracle at the
    f32 bar / the bf16 e2e bar (test_bf16_e2e_vs_reference_fixture)."""
    from leastereo_amd import executor
    assert not kernels.cv_stem_supported(32, 8, 66, False) and kernels.cv_stem_supported(32, 8, 66, True)
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=24)), DEV, precision=precision)
    m.load_state_dict(state_dict(), strict=True)
    m = m.to(DEV).eval()
    left = normal(5151, (1, 3, 48, 198))
    right = normal(5152, (1, 3, 48, 198))
    with torch.no_grad():
        disp = m(left.to(DEV), right.to(DEV)).cpu()
        want = ref.leastereo_forward(state_dict(), left, right, 24, arch())
    # (the reference's feature net returns 65 of the 66 columns here: its output is 195 wide)
    assert executor.CV_STEM and disp.shape == want.shape and torch.isfinite(disp).all()
    assert ref.epe(disp, want) < bound


@pytest.mark.parametrize("c8", [False, True])
def test_fused_feature_stems_vs_torch(c8):
    """lea_feature_stem_bnrelu (new_model_2d.py:93-94 fused) vs float64 torch of
    ConvBR(3->16, s1) then ConvBR(16->32, s3), edge rows / columns included (H, W not
    multiples of 3); c8: the bf16 output of the same f32 values."""
    g = torch.Generator().manual_seed(77)
    x = torch.randn(2, 3, 50, 131, generator=g)
    w0 = torch.randn(16, 3, 3, 3, generator=g) / np.sqrt(27)
    w1 = torch.randn(32, 16, 3, 3, generator=g) / np.sqrt(144)
    s0, t0 = torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g) * 0.1
    s1, t1 = torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g) * 0.1
    a = torch.relu(F.conv2d(x.double(), w0.double(), None, 1, 1) * s0.double().view(1, -1, 1, 1)
                   + t0.double().view(1, -1, 1, 1))
    want = torch.relu(F.conv2d(a, w1.double(), None, 3, 1) * s1.double().view(1, -1, 1, 1)
                      + t1.double().view(1, -1, 1, 1))
    got = kernels.feature_stem(x.to(DEV), w0.to(DEV), s0.to(DEV), t0.to(DEV), w1.to(DEV), s1.to(DEV),
                               t1.to(DEV), c8)
    if c8:
        got = kernels.from_c8(got)
        np.testing.assert_allclose(got[:, :, 0].cpu().double().numpy(), want.numpy(), rtol=1e-2, atol=1e-2)
    else:
        np.testing.assert_allclose(got[:, :, 0].cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
    # two sources: [x; x2] stacked without a concatenated copy, bit for bit
    x2 = torch.randn(2, 3, 50, 131, generator=g)
    both = kernels.feature_stem(x.to(DEV), w0.to(DEV), s0.to(DEV), t0.to(DEV), w1.to(DEV), s1.to(DEV),
                                t1.to(DEV), c8, x2.to(DEV))
    cat = kernels.feature_stem(torch.cat((x, x2), 0).to(DEV), w0.to(DEV), s0.to(DEV), t0.to(DEV),
                               w1.to(DEV), s1.to(DEV), t1.to(DEV), c8)
    assert torch.equal(both, cat)
    # one image per source: a single launch striding from x to x2
    one = kernels.feature_stem(x[:1].to(DEV), w0.to(DEV), s0.to(DEV), t0.to(DEV), w1.to(DEV), s1.to(DEV),
                               t1.to(DEV), c8, x2[1:].to(DEV))
    assert torch.equal(one, cat[[0, 3]])
    # a non-contiguous right image (a transposed view of the same values) on that path
    x2_nc = x2[1:].to(DEV).transpose(2, 3).contiguous().transpose(2, 3)
    assert not x2_nc.is_contiguous()
    one_nc = kernels.feature_stem(x[:1].to(DEV), w0.to(DEV), s0.to(DEV), t0.to(DEV), w1.to(DEV),
                                  s1.to(DEV), t1.to(DEV), c8, x2_nc)
    assert torch.equal(one_nc, cat[[0, 3]])
