"""GPU parity of the Winograd F(2,3)-along-W conv engine (csrc/conv3d_wino.hip)
against float64 torch, with the tolerance of the direct fp32 engine
(|d| <= 1e-4 + 1e-4 |ref|, test_gpu_parity.py) -- the transforms add a few fp32
roundings per product, far inside it -- and against the direct engine itself.
End to end the model runs on this engine by default, so test_gpu_parity.py's
e2e / config-1 / full-size cases cover it at EPE <= 1e-3 px."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from leastereo_amd import _lib, kernels

pytestmark = pytest.mark.gpu
DEV = "cuda"
WPRE_DEFAULT = 1  # lea_conv3d_wino2p_set_wpre's library default (csrc/conv3d_wino.hip g_wpre)
W44U_DEFAULT = 0  # lea_conv3d_wino44_set_upre's library default (csrc/conv3d_wino44.hip g_w44u)
W44G_DEFAULT = -1  # lea_conv3d_wino44_set_group's library default (g_w44g: auto)
W44_DEFAULT = 2  # lea_conv3d_wino44_set's library default (csrc/conv3d_wino44.hip g_w44)


def _ref(x, w, scale, shift, relu, res=None):
    y = F.conv3d(x.double(), w.double(), None, 1, 1)
    if scale is not None:
        y = y * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1)
    if relu:
        y = torch.relu(y)
    if res is not None:
        y = y + res.double()
    return y


@pytest.mark.parametrize("b,cin,cout,shape,mode", [
    (1, 64, 32, (6, 20, 70), None), (1, 32, 32, (5, 9, 320), "acc"), (2, 8, 24, (3, 7, 130), "res"),
    (1, 16, 16, (4, 5, 127), "acc"), (2, 128, 64, (5, 9, 40), "acc"), (1, 16, 16, (7, 33, 17), "acc"),
    (1, 16, 48, (4, 9, 40), None), (1, 32, 96, (3, 6, 21), "res"), (1, 8, 24, (3, 10, 17), None),
    (1, 12, 20, (3, 4, 5), "acc"), (2, 32, 32, (9, 13, 31), "res"), (1, 4, 12, (1, 1, 1), None),
    (1, 32, 32, (2, 3, 2), "acc"),
    # depth-paired (couts <= 8): odd D (the last pair's second plane masked), D = 1
    (1, 8, 8, (5, 9, 70), "res"), (2, 16, 8, (4, 7, 33), "acc"), (1, 8, 4, (1, 3, 64), None),
    (1, 32, 8, (6, 20, 130), None), (1, 8, 8, (3, 12, 320), "acc"), (1, 4, 6, (2, 5, 9), "res")])
def test_wino_vs_torch(b, cin, cout, shape, mode):
    """Odd and even W (the last pair half-masked), ragged H/D tiles, every epilogue."""
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None)
    out = r.to(DEV).clone() if mode == "acc" else None
    y = kernels.conv3d_bnrelu_wino(x.to(DEV), kernels.pack_conv_weight_wino(w.to(DEV)), cout,
                                   scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                   accumulate=mode == "acc",
                                   residual=r.to(DEV) if mode == "res" else None)
    np.testing.assert_allclose(y.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("f", [2, 4, 8])
@pytest.mark.parametrize("np_,td", [(1, 1), (1, 2), (2, 1), (2, 2)])
@pytest.mark.parametrize("cout", [16, 48, 64])
def test_wino_every_tile(np_, td, cout, f):
    """Every instantiated (F, rows, planes) tile on a ragged volume (W = 45: a partial
    last group of outputs for both F) with the accumulate epilogue."""
    if np_ == 2 and (cout == 48 or f != 2):
        pytest.skip("48-row blocks and F(4,3) tiles are instantiated with one row per wave (LDS budget)")
    if cout == 48 and (f == 4 or (f == 8 and td == 2)):
        pytest.skip("48-row blocks run F(2,3), or F(4,3) on row pairs one plane deep")
    lib = _lib.load()
    g = torch.Generator().manual_seed(np_ * 10 + td + cout)
    x = torch.randn((2, 32, 5, 11, 45), generator=g)
    w = torch.randn(cout, 32, 3, 3, 3, generator=g) / np.sqrt(32 * 27)
    r = torch.randn((2, cout, 5, 11, 45), generator=g)
    want = _ref(x, w, None, None, False, r)
    assert lib.lea_conv3d_wino_set_tile_override(np_, td, f) == 0
    try:
        name = kernels.wino_kernel_name(2, cout, 5, 11, 45)
        mt = {16: 1, 48: 3, 64: 2}[cout]
        ff, q = (4, 8) if f == 8 else (f, 16)
        assert name == f"conv3d_wino_kernel<{ff}, {q}, {mt}, {np_}, {td}, false>", name
        out = r.to(DEV).clone()
        kernels.conv3d_bnrelu_wino(x.to(DEV), kernels.pack_conv_weight_wino(w.to(DEV)), cout, None,
                                   None, relu=False, out=out, accumulate=True)
    finally:
        lib.lea_conv3d_wino_set_tile_override(0, 0, 0)
    np.testing.assert_allclose(out.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


def test_wino_two_sources_into_a_channel_slice():
    """conv1/conv2 shape: cat(x, x2) read in place, output into a slice of a cat buffer."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn((1, 64, 4, 10, 40), generator=g)
    x2 = torch.randn((1, 64, 4, 10, 40), generator=g)
    w = torch.randn(64, 128, 3, 3, 3, generator=g) / np.sqrt(128 * 27)
    want = _ref(torch.cat((x, x2), 1), w, None, None, False)
    big = torch.zeros((1, 96, 4, 10, 40), device=DEV)
    kernels.conv3d_bnrelu_wino(x.to(DEV), kernels.pack_conv_weight_wino(w.to(DEV)), 64, None, None,
                               relu=False, out=big[:, 16:80], x2=x2.to(DEV))
    np.testing.assert_allclose(big[:, 16:80].cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
    assert float(big[:, :16].abs().sum()) == 0 and float(big[:, 80:].abs().sum()) == 0


@pytest.mark.parametrize("b,c,cout,maxdisp,hw", [(1, 32, 32, 48, (12, 40)), (2, 16, 16, 27, (5, 19))])
def test_wino_costvolume_is_bit_identical_to_the_materialised_volume(b, c, cout, maxdisp, hw):
    """stem0 reading the cost volume in place == the same engine on the built volume (the
    F(4,3) x F(2,3) arithmetic: the materialised volume's conv is held off the r06 F(4,3) x F(4,3)
    tile, which the in-place read never takes)."""
    g = torch.Generator().manual_seed(c + maxdisp)
    fl = torch.randn((b, c) + hw, generator=g).to(DEV)
    fr = torch.randn((b, c) + hw, generator=g).to(DEV)
    w = (torch.randn(cout, 2 * c, 3, 3, 3, generator=g) / np.sqrt(2 * c * 27)).to(DEV)
    packed = kernels.pack_conv_weight_wino(w)
    scale = torch.rand(cout, device=DEV) + 0.5
    shift = torch.randn(cout, device=DEV) * 0.1
    cost = kernels.build_cost_volume(fl, fr, maxdisp)
    with kernels.wino_depth_f2():
        want = kernels.conv3d_bnrelu_wino(cost, packed, cout, scale, shift)
    got = kernels.conv3d_bnrelu_costvolume_wino(fl, fr, maxdisp, packed, cout, scale, shift)
    assert torch.equal(got, want)
    ref = _ref(cost.cpu(), w.cpu(), scale.cpu(), shift.cpu(), True)
    np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_wino_matches_the_direct_engine_at_full_size():
    """conv1/conv2 at config 2 (128 -> 64 at 32x96x160): Winograd vs direct engine."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn((1, 128, 32, 96, 160), device=DEV, generator=g)
    w = torch.randn(64, 128, 3, 3, 3, device=DEV, generator=g) / np.sqrt(128 * 27)
    a = kernels.conv3d_bnrelu(x, kernels.pack_conv_weight(w), 64, 3, None, None, relu=False)
    b = kernels.conv3d_bnrelu_wino(x, kernels.pack_conv_weight_wino(w), 64, None, None, relu=False)
    err = float((a - b).abs().max())
    assert err <= 1e-4 * float(a.abs().max()), err


@pytest.mark.parametrize("mode,name", [
    (0, "conv3d_wino_kernel<4, 16, 0, 1, 2, false, true, true>"),
    (1, "conv3d_wino2_kernel<16, 1, 1, 4, 2, 0, false>")])
def test_small_cout_tiles_match_the_direct_engine_at_full_size(mode, name):
    """The L0 8->8 cell op at config 2 (8 channels, 64x192x320) on both small-cout forms
    of the Winograd entries -- the depth-paired 1-D tile (couts of two planes per 16-row
    MFMA tile, mode 0, the default) and the W x D engine's 16-row block (mode 1) -- vs
    the direct engine.  Packing and launch share the mode."""
    lib = _lib.load()
    assert lib.lea_conv3d_wino_set_small_cout(mode) == 0
    try:
        assert kernels.wino_kernel_name(1, 8, 64, 192, 320) == name
        g = torch.Generator(device=DEV).manual_seed(4)
        x = torch.randn((1, 8, 64, 192, 320), device=DEV, generator=g)
        w = torch.randn(8, 8, 3, 3, 3, device=DEV, generator=g) / np.sqrt(8 * 27)
        a = kernels.conv3d_bnrelu(x, kernels.pack_conv_weight(w), 8, 3, None, None, relu=False)
        b = kernels.conv3d_bnrelu_wino(x, kernels.pack_conv_weight_wino(w), 8, None, None, relu=False)
        err = float((a - b).abs().max())
        assert err <= 1e-4 * float(a.abs().max()), err
    finally:
        lib.lea_conv3d_wino_set_small_cout(0)


def test_model_uses_the_winograd_engine():
    from leastereo_amd import executor
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV).to(DEV).eval()
    ex = m.matching.executor()
    wino = {n for n, p in ex.p.items() if p.wino is not None}
    assert executor.WINOGRAD and {"stem0", "stem1", "conv1", "conv2"} <= wino
    # the L0 8-channel cell ops run on the same engine
    assert any(ex.p[n].cout <= 8 and ex.p[n].k == 3 for n in wino)


@pytest.mark.parametrize("variant", [0, 1])
def test_e2e_golden_with_every_eligible_layer_on_winograd(monkeypatch, variant):
    """The reference's end-to-end golden case (96x192 D48) with the Winograd engine
    forced onto every eligible layer (the size threshold would keep this small
    case on the direct engine): EPE vs the reference fp32 / fp64 disparity, with the
    planner's engines (variant 0: W x D where it applies) and F(4,3) along W only."""
    monkeypatch.setattr(kernels, "WINO_MIN_VOXELS", 0)
    assert _lib.load().lea_conv3d_wino_set_variant(variant) == 0
    try:
        _e2e_golden_cases()
    finally:
        _lib.load().lea_conv3d_wino_set_variant(0)


def _e2e_golden_cases():
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from oracle import torch_ref as ref
    from tests.golden_util import golden, meta, normal, state_dict
    for name, c in meta()["cases"].items():
        if not name.startswith("e2e/"):
            continue
        key = name.split("/", 1)[1]
        m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=c["maxdisp"])), DEV)
        m.load_state_dict(state_dict(), strict=True)
        m = m.to(DEV).eval()
        shape = (c.get("batch", 1), 3, c["height"], c["width"])
        with torch.no_grad():
            d = m(normal(c["seeds"][0], shape).to(DEV), normal(c["seeds"][1], shape).to(DEV)).cpu()
        g = golden("e2e")
        assert ref.epe(d, torch.from_numpy(g[key + "/disp32"])) < 1e-3
        assert ref.epe(d, torch.from_numpy(g[key + "/disp64"])) < 1e-3


def test_graphed_forward_replays_the_eager_result():
    """LEAStereo.graphed: the forward captured into a HIP graph replays to the eager
    output bit for bit, for new inputs copied into its static buffers."""
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from tests.golden_util import normal, state_dict
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), DEV)
    m.load_state_dict(state_dict(), strict=True)
    m = m.to(DEV).eval()
    g = m.graphed(2, 96, 192)
    for seed in (5, 6):
        x = normal(seed, (2, 3, 96, 192)).to(DEV)
        y = normal(seed + 10, (2, 3, 96, 192)).to(DEV)
        with torch.no_grad():
            want = m(x, y)
        got = g(x, y)
        torch.cuda.synchronize()
        assert torch.equal(got, want)


# ---- F(4,3) along W x F(2,3) along D (csrc/conv3d_wino2.hip) ----

@pytest.fixture
def wino_variant():
    lib = _lib.load()

    def use(v):
        assert lib.lea_conv3d_wino_set_variant(v) == 0
    yield use
    lib.lea_conv3d_wino_set_variant(0)


@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("b,cin,cout,shape,mode", [
    (1, 64, 32, (6, 20, 70), None), (1, 32, 32, (5, 9, 320), "acc"), (2, 8, 24, (3, 7, 130), "res"),
    (1, 16, 16, (4, 5, 127), "acc"), (2, 128, 64, (5, 9, 40), "acc"), (1, 16, 16, (7, 33, 17), "acc"),
    (1, 12, 20, (3, 4, 5), "acc"), (2, 32, 32, (9, 13, 31), "res"), (1, 4, 12, (1, 1, 1), None),
    (1, 32, 32, (2, 3, 2), "acc"), (1, 32, 96, (3, 6, 21), "res"), (1, 16, 16, (1, 6, 64), None)])
def test_wino2_vs_torch(wino_variant, variant, b, cin, cout, shape, mode):
    """The W x D engine's tiles: odd D (the last pair's / quad's planes masked), D = 1,
    W not a multiple of 4, ragged H tiles, every epilogue, couts padding a block."""
    wino_variant(variant)
    name = kernels.wino_kernel_name(b, cout, *shape, cin=cin)
    # (the planner's default, variant 5, puts the pipelined layers on the r06 F(4,3) x F(4,3) tile)
    assert name.startswith(("conv3d_wino2", "conv3d_wino44")), name
    g = torch.Generator().manual_seed(cin * 7 + cout + variant)
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None)
    out = r.to(DEV).clone() if mode == "acc" else None
    y = kernels.conv3d_bnrelu_wino(x.to(DEV), kernels.pack_conv_weight_wino(w.to(DEV)), cout,
                                   scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                   accumulate=mode == "acc",
                                   residual=r.to(DEV) if mode == "res" else None)
    np.testing.assert_allclose(y.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6, 7])
def test_wino2_keeps_the_1d_engine_where_it_has_no_tile(wino_variant, variant):
    """48-row blocks, and couts <= 8 in the default (depth-paired) mode, stay on F(4,3)
    along W; couts <= 8 in mode 1 take the W x D engine's 16-row block."""
    wino_variant(variant)
    lib = _lib.load()
    assert kernels.wino_kernel_name(1, 8, 64, 192, 320).startswith("conv3d_wino_kernel<")
    assert lib.lea_conv3d_wino_set_small_cout(1) == 0
    try:
        assert kernels.wino_kernel_name(1, 8, 64, 192, 320).startswith("conv3d_wino2_kernel<")
    finally:
        lib.lea_conv3d_wino_set_small_cout(0)
    assert kernels.wino_kernel_name(1, 48, 32, 96, 160).startswith("conv3d_wino_kernel<")


@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6, 7])
def test_wino2_costvolume_and_two_sources(wino_variant, variant):
    """stem0 on the in-place cost volume == the same tile on the built volume (bit for
    bit); conv1/conv2's two-source read into a channel slice."""
    wino_variant(variant)
    g = torch.Generator().manual_seed(5 + variant)
    fl = torch.randn((2, 32, 12, 40), generator=g).to(DEV)
    fr = torch.randn((2, 32, 12, 40), generator=g).to(DEV)
    w = (torch.randn(32, 64, 3, 3, 3, generator=g) / np.sqrt(64 * 27)).to(DEV)
    packed = kernels.pack_conv_weight_wino(w)
    scale = torch.rand(32, device=DEV) + 0.5
    shift = torch.randn(32, device=DEV) * 0.1
    cost = kernels.build_cost_volume(fl, fr, 45)
    with kernels.wino_depth_f2():  # the in-place read's F(4,3) x F(2,3) arithmetic (r06 tile held off)
        want = kernels.conv3d_bnrelu_wino(cost, packed, 32, scale, shift)
    got = kernels.conv3d_bnrelu_costvolume_wino(fl, fr, 45, packed, 32, scale, shift)
    assert torch.equal(got, want)
    ref = _ref(cost.cpu(), w.cpu(), scale.cpu(), shift.cpu(), True)
    np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    x = torch.randn((1, 64, 4, 10, 40), generator=g)
    x2 = torch.randn((1, 64, 4, 10, 40), generator=g)
    w2 = torch.randn(64, 128, 3, 3, 3, generator=g) / np.sqrt(128 * 27)
    want = _ref(torch.cat((x, x2), 1), w2, None, None, False)
    big = torch.zeros((1, 96, 4, 10, 40), device=DEV)
    kernels.conv3d_bnrelu_wino(x.to(DEV), kernels.pack_conv_weight_wino(w2.to(DEV)), 64, None, None,
                               relu=False, out=big[:, 16:80], x2=x2.to(DEV))
    np.testing.assert_allclose(big[:, 16:80].cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
    assert float(big[:, :16].abs().sum()) == 0 and float(big[:, 80:].abs().sum()) == 0


@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6, 7])
def test_wino2_matches_the_direct_engine_at_full_size(wino_variant, variant):
    """conv1/conv2 and stem0 at config 2 on the W x D engine vs the direct engine."""
    wino_variant(variant)
    g = torch.Generator(device=DEV).manual_seed(3)
    for cin, cout, shape in ((128, 64, (32, 96, 160)), (64, 32, (64, 192, 320))):
        x = torch.randn((1, cin) + shape, device=DEV, generator=g)
        w = torch.randn(cout, cin, 3, 3, 3, device=DEV, generator=g) / np.sqrt(cin * 27)
        a = kernels.conv3d_bnrelu(x, kernels.pack_conv_weight(w), cout, 3, None, None, relu=False)
        b = kernels.conv3d_bnrelu_wino(x, kernels.pack_conv_weight_wino(w), cout, None, None, relu=False)
        err = float((a - b).abs().max())
        assert err <= 1e-4 * float(a.abs().max()), (cin, cout, err)


@pytest.mark.parametrize("b,cin,cout,shape,small", [
    (1, 16, 16, (11, 20, 40), 0),   # W x D engine, 16-row blocks; 6 depth pairs
    (2, 8, 24, (9, 8, 70), 0),      # W x D engine with the transform pass (32-row block)
    (1, 16, 48, (7, 12, 33), 0),    # 1-D engine, 48-row block, one plane per group
    (1, 8, 8, (13, 10, 64), 0),     # 1-D engine, depth-paired
    (1, 8, 8, (5, 6, 40), 1)])      # W x D engine with an 8-cout block (small-cout mode 1)
def test_depth_walk_is_bit_identical(b, cin, cout, shape, small):
    """Workgroups walking 1, 2, 3 or 4 depth groups (lea_conv3d_wino2_set_walk) run the
    same per-group arithmetic: outputs identical bit for bit, accumulate mode included,
    for walks that do and do not divide the number of groups."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(cin * 7 + cout)
    x = torch.randn((b, cin) + shape, device=DEV, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device=DEV, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, device=DEV, generator=g)
    assert lib.lea_conv3d_wino_set_small_cout(small) == 0
    try:
        pw = kernels.pack_conv_weight_wino(w)
        outs = []
        for walk in (1, 2, 3, 4):
            assert lib.lea_conv3d_wino2_set_walk(walk) == 0
            y = r.clone()
            kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, True)
            outs.append(y)
    finally:
        lib.lea_conv3d_wino2_set_walk(0)
        lib.lea_conv3d_wino_set_small_cout(0)
    for y in outs[1:]:
        assert torch.equal(y, outs[0])
    want = F.conv3d(x.double(), w.double(), None, 1, 1)
    want = torch.relu(want * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1)) + r.double()
    np.testing.assert_allclose(outs[0].cpu().double().numpy(), want.cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cin,cout,shape,small,variant", [
    (1, 16, 16, (11, 20, 40), 0, 0),   # W x D engine, 16-row blocks, partial row tiles
    (2, 8, 24, (9, 8, 68), 0, 0),      # W x D engine with the transform pass, 24 of 32 couts
    (1, 16, 48, (7, 12, 36), 0, 0),    # 1-D engine, 48-row block
    (1, 8, 8, (13, 10, 64), 0, 0),     # 1-D engine, depth-paired, odd depth
    (1, 32, 32, (5, 10, 20), 0, 1),    # 1-D engine, 32-row block, two planes
    (1, 8, 8, (5, 6, 40), 1, 0)])      # W x D engine with an 8-cout block (small-cout mode 1)
def test_buffer_epilogue_is_bit_identical(b, cin, cout, shape, small, variant):
    """The buffer-addressed epilogue (out-of-range lanes dropped, residual loads issued
    together; lea_conv3d_wino_set_epi_buf) stores exactly what the per-group epilogue
    stores, into a channel slice of a larger buffer, with and without the residual.  (The
    two-chunk 8 -> 24 shape runs on the F(4,3) x F(4,3) tile by default, which has the
    buffer epilogue only: this test keeps it on the W x D engine it is about, mode 1.)"""
    lib = _lib.load()
    assert lib.lea_conv3d_wino44_set(1) == 0
    g = torch.Generator(device=DEV).manual_seed(cin * 5 + cout + shape[2])
    x = torch.randn((b, cin) + shape, device=DEV, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device=DEV, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.1
    r = torch.randn((b, cout + 8) + shape, device=DEV, generator=g)
    assert lib.lea_conv3d_wino_set_small_cout(small) == 0
    assert lib.lea_conv3d_wino_set_variant(variant) == 0
    try:
        pw = kernels.pack_conv_weight_wino(w)
        outs = []
        for on in (0, 1):
            assert lib.lea_conv3d_wino_set_epi_buf(on) == 0
            for acc in (False, True):
                y = r.clone()
                kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y[:, 4:4 + cout], acc)
                outs.append(y)
    finally:
        lib.lea_conv3d_wino_set_epi_buf(1)
        lib.lea_conv3d_wino_set_variant(0)
        lib.lea_conv3d_wino_set_small_cout(0)
        lib.lea_conv3d_wino44_set(int(os.environ.get("LEASTEREO_WINO44") or W44_DEFAULT))
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])
    assert torch.equal(outs[3][:, :4], r[:, :4]) and torch.equal(outs[3][:, 4 + cout:], r[:, 4 + cout:])
    want = F.conv3d(x.double(), w.double(), None, 1, 1)
    want = torch.relu(want * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    np.testing.assert_allclose(outs[3][:, 4:4 + cout].cpu().double().numpy(),
                               (want + r[:, 4:4 + cout].double()).cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cin,c1,cout,shape,mode", [
    (1, 32, 32, 32, (5, 9, 320), "acc"), (2, 128, 64, 64, (5, 9, 40), "res"),
    (1, 64, 64, 32, (4, 7, 36), None), (1, 8, 8, 24, (3, 6, 68), "acc"),
    (1, 32, 32, 96, (3, 6, 20), "res"), (2, 16, 8, 32, (7, 13, 4), None),
    (1, 32, 32, 32, (1, 1, 4), None), (1, 4, 4, 32, (2, 3, 8), "res"), (2, 8, 8, 64, (9, 5, 72), "acc"),
    # the depth-paired 1-D tile (couts <= 8, 64-wide rows): odd D, partial rows, 2 sources
    (1, 8, 8, 8, (5, 9, 320), "acc"), (2, 16, 8, 8, (4, 7, 124), "res"), (1, 8, 8, 6, (3, 5, 60), None),
    (1, 32, 32, 8, (6, 20, 188), None)])
def test_wd_halo16_is_bit_identical_to_dword_pieces(b, cin, c1, cout, shape, mode):
    """The transform-pass W x D tile with its halo staged as 16-byte pieces (rows of whole
    16-byte blocks: W % 4 == 0) -- as the one-barrier pipeline (conv3d_wino2p_kernel, weights
    from the per-lane copy, the default) and the two-barrier tile (PV = 2) -- and the
    depth-paired 1-D kernel with 16-byte pieces (fenced schedule, the default, and the compiler's)
    equal the dword-piece staging bit for bit
    (same values in LDS, same transforms, same accumulation order) and float64 torch at the
    engine bar; ragged H / D / W tiles (W = 36, 68, 4, 124, 60, 188: partial rows), a single
    item (cin 4, one pair), two sources (cin1 = c1), every epilogue."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin + cout + shape[2])
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None)
    xs = x.to(DEV)
    x1, x2 = (xs[:, :c1].contiguous(), xs[:, c1:].contiguous()) if c1 < cin else (xs, None)
    pw = kernels.pack_conv_weight_wino(w.to(DEV))
    outs = {}
    assert lib.lea_conv3d_wino44_set(0) == 0  # this test is the F(4,3) x F(2,3) kernel's
    # (halo16, pipeline, fence, W-transformed per-lane weights: r06 lea_conv3d_wino2p_set_wpre)
    for on, pipe, fence, wpre in ((1, 1, 1, 0), (1, 0, 1, 0), (0, 1, 1, 0), (1, 1, 0, 0), (1, 1, 1, 1)):
        assert lib.lea_conv3d_wino2_set_halo16(on) == 0 and lib.lea_conv3d_wino2_set_pipeline(pipe) == 0
        assert lib.lea_conv3d_wino_set_fence(fence) == 0 and lib.lea_conv3d_wino2p_set_wpre(wpre) == 0
        try:
            name = kernels.wino_kernel_name(b, cout, *shape, cin=cin)
            if cout <= 8:
                want_name = "conv3d_wino_kernel<4, 16, 0, 1, 2, false%s>" % (
                    (", true, true" if fence else ", true") if on else "")
                assert name == want_name, name
            elif on and pipe and cin > 8:  # (one or two chunks per pair: the two-barrier tile)
                assert name == "conv3d_wino2p_kernel", name
            else:
                assert name.startswith("conv3d_wino2_kernel<8, 2, 1, 4, 2, %d," % (2 if on else 1)), name
            out = r.to(DEV).clone() if mode == "acc" else None
            outs[(on, pipe, fence, wpre)] = kernels.conv3d_bnrelu_wino(
                x1, pw, cout, scale.to(DEV), shift.to(DEV), relu=True, out=out, accumulate=mode == "acc", x2=x2,
                residual=r.to(DEV) if mode == "res" else None)
        finally:
            lib.lea_conv3d_wino2_set_halo16(1)
            lib.lea_conv3d_wino2_set_pipeline(1)
            lib.lea_conv3d_wino_set_fence(1)
            lib.lea_conv3d_wino2p_set_wpre(int(os.environ.get("LEASTEREO_WINO2P_WPRE") or WPRE_DEFAULT))
    lib.lea_conv3d_wino44_set(int(os.environ.get("LEASTEREO_WINO44") or W44_DEFAULT))
    base = outs[(0, 1, 1, 0)]
    assert all(torch.equal(o, base) for o in outs.values()), [k for k, o in outs.items() if not torch.equal(o, base)]
    np.testing.assert_allclose(outs[(1, 1, 1, 0)].cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,cin,c1,cout,shape,mode", [
    (1, 16, 16, 16, (11, 20, 40), "acc"), (2, 16, 16, 16, (5, 9, 36), "res"),
    (1, 32, 16, 16, (4, 13, 68), None), (1, 16, 16, 16, (1, 1, 4), None),
    (2, 64, 64, 16, (3, 8, 32), "acc"), (1, 16, 16, 16, (7, 33, 164), "res"),
    (1, 16, 16, 12, (6, 10, 44), "acc")])
def test_lane_halo16_is_bit_identical_to_dword_pieces(b, cin, c1, cout, shape, mode):
    """The per-lane 16-cout W x D tile with its halo staged as 16-byte pieces into the
    interleaved-row, bank-conflict-free layout (PV = 4, r04; lea_conv3d_wino2_set_lane_halo16),
    and its fenced-schedule form (PV = 5, the default) equal the dword-piece tile (PV = 0) bit for bit -- same staged values, same transforms,
    same accumulation order -- and float64 torch at the engine bar: ragged H (partial 8-row
    tiles), odd D, W not a multiple of 32, one item, two sources, couts padding the block,
    every epilogue."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin * 3 + cout + shape[2])
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None)
    xs = x.to(DEV)
    x1, x2 = (xs[:, :c1].contiguous(), xs[:, c1:].contiguous()) if c1 < cin else (xs, None)
    pw = kernels.pack_conv_weight_wino(w.to(DEV))
    outs = {}
    for on in (1, 2, 0):
        assert lib.lea_conv3d_wino2_set_lane_halo16(on) == 0
        try:
            name = kernels.wino_kernel_name(b, cout, *shape, cin=cin)
            assert name == "conv3d_wino2_kernel<8, 1, 1, 4, 2, %d, false>" % {1: 4, 2: 5, 0: 0}[on], name
            out = r.to(DEV).clone() if mode == "acc" else None
            outs[on] = kernels.conv3d_bnrelu_wino(x1, pw, cout, scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                                  accumulate=mode == "acc", x2=x2,
                                                  residual=r.to(DEV) if mode == "res" else None)
        finally:
            lib.lea_conv3d_wino2_set_lane_halo16(2)
    assert torch.equal(outs[1], outs[0]) and torch.equal(outs[2], outs[0])
    np.testing.assert_allclose(outs[1].cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


# ------------------------------------------------------------------ F(2,3) x F(2,3) tile
@pytest.mark.parametrize("b,cin,cout,shape,mode,split", [
    (1, 16, 16, (32, 96, 160), "acc", 0),    # the L1 cells' 16 -> 16 op at C2
    (1, 16, 16, (16, 48, 80), "res", 0),     # a partial 32-column tile (W = 80)
    (2, 16, 16, (5, 9, 20), None, 0),        # odd D, H not a multiple of 8, W < 32
    (1, 32, 16, (4, 7, 36), "acc", 0),       # 8 chunks, W = 36 (a 4-column tail tile)
    (1, 16, 12, (3, 10, 24), "res", 0),      # a partial cout block (12 of 16 rows)
    (1, 16, 16, (6, 11, 40), "acc", 8),      # two sources (cat of 8 + 8 channels)
    (1, 64, 16, (2, 3, 4), None, 0),         # one row, one column tile, one depth pair
])
def test_wino22_vs_torch(b, cin, cout, shape, mode, split):
    """conv3d_wino22_kernel (16-cout blocks on F(2,3) x F(2,3), the packer's U, 4 waves per
    SIMD) against float64 torch with the engines' tolerance, every epilogue, ragged tiles;
    and the same layer on the default per-lane F(4,3) x F(2,3) tile within the same bar."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin * 11 + cout + shape[2])
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None).numpy()
    packed = kernels.pack_conv_weight_wino(w.to(DEV))
    xd = x.to(DEV)
    x1, x2 = (xd[:, :split].contiguous(), xd[:, split:].contiguous()) if split else (xd, None)
    got = {}
    try:
        for on in (1, 0):
            assert lib.lea_conv3d_wino_set_w22(on) == 0
            name = kernels.wino_kernel_name(b, cout, *shape)
            assert (name == "conv3d_wino22_kernel") == bool(on), name
            out = r.to(DEV).clone() if mode == "acc" else None
            got[on] = kernels.conv3d_bnrelu_wino(x1, packed, cout, scale.to(DEV), shift.to(DEV), relu=True,
                                                 out=out, accumulate=mode == "acc", x2=x2,
                                                 residual=r.to(DEV) if mode == "res" else None)
            np.testing.assert_allclose(got[on].cpu().double().numpy(), want, rtol=1e-4, atol=1e-4)
    finally:
        lib.lea_conv3d_wino_set_w22(0)


def test_wino22_writes_only_its_channel_slice():
    """Output into channels [16, 32) of a 48-channel buffer: the other channels untouched."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(22)
    x = torch.randn((1, 16, 4, 9, 40), generator=g).to(DEV)
    w = (torch.randn(16, 16, 3, 3, 3, generator=g) / np.sqrt(16 * 27)).to(DEV)
    big = torch.full((1, 48, 4, 9, 40), 3.0, device=DEV)
    try:
        assert lib.lea_conv3d_wino_set_w22(1) == 0
        kernels.conv3d_bnrelu_wino(x, kernels.pack_conv_weight_wino(w), 16, None, None, relu=False,
                                   out=big[:, 16:32])
    finally:
        lib.lea_conv3d_wino_set_w22(0)
    want = F.conv3d(x.double(), w.double(), None, 1, 1)
    np.testing.assert_allclose(big[:, 16:32].cpu().double().numpy(), want.cpu().numpy(), rtol=1e-4, atol=1e-4)
    assert bool((big[:, :16] == 3.0).all()) and bool((big[:, 32:] == 3.0).all())


@pytest.mark.parametrize("b,cin,c1,cout,shape,mode", [
    (1, 32, 32, 32, (5, 9, 320), "acc"), (2, 128, 64, 64, (5, 9, 40), "res"), (1, 64, 64, 32, (4, 7, 36), None),
    (1, 32, 32, 96, (3, 6, 20), "res"), (2, 16, 8, 32, (7, 13, 4), None), (1, 32, 32, 32, (1, 1, 4), None),
    (1, 16, 16, 32, (8, 12, 32), "acc"), (1, 128, 64, 64, (16, 10, 96), None), (1, 32, 32, 32, (6, 5, 68), "res"),
    (2, 12, 12, 40, (9, 3, 12), "acc")])
def test_wino44_vs_float64(b, cin, c1, cout, shape, mode):
    """The F(4,3) x F(4,3) tile (r06, lea_conv3d_wino44_set: the pipelined W x D kernel's layers;
    the W points split over two waves that swap accumulators in the epilogue) against float64
    torch at the engine bar (|d| <= 1e-4 + 1e-4 |ref|) and against the F(4,3) x F(2,3) kernel:
    ragged D (not a multiple of 4: masked planes), H (odd), W (partial 32-wide tiles), a single
    item, two sources, couts padded to the 32-cout block (40, 96), every epilogue."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin + 3 * cout + shape[2])
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if mode else None)
    xs = x.to(DEV)
    x1, x2 = (xs[:, :c1].contiguous(), xs[:, c1:].contiguous()) if c1 < cin else (xs, None)
    pw = kernels.pack_conv_weight_wino(w.to(DEV))
    outs = {}
    for on, upre, grp in ((0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 2), (1, 0, 3), (1, 0, 16)):
        assert lib.lea_conv3d_wino44_set(on) == 0 and lib.lea_conv3d_wino44_set_upre(upre) == 0
        assert lib.lea_conv3d_wino44_set_group(grp) == 0
        try:
            name = kernels.wino_kernel_name(b, cout, *shape, cin=cin)
            if cin > 8:
                assert name == ("conv3d_wino44_kernel" if on else "conv3d_wino2p_kernel"), name
            out = r.to(DEV).clone() if mode == "acc" else None
            outs[(on, upre, grp)] = kernels.conv3d_bnrelu_wino(
                x1, pw, cout, scale.to(DEV), shift.to(DEV), relu=True, out=out, accumulate=mode == "acc", x2=x2,
                residual=r.to(DEV) if mode == "res" else None).cpu().double()
        finally:
            lib.lea_conv3d_wino44_set(int(os.environ.get("LEASTEREO_WINO44") or W44_DEFAULT))
            lib.lea_conv3d_wino44_set_upre(int(os.environ.get("LEASTEREO_WINO44_UPRE") or W44U_DEFAULT))
            lib.lea_conv3d_wino44_set_group(W44G_DEFAULT)
    np.testing.assert_allclose(outs[(1, 0, 0)].numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(outs[(1, 0, 0)].numpy(), outs[(0, 0, 0)].numpy(), rtol=1e-4, atol=1e-4)
    # U precomputed by the packer (lea_conv3d_wino44_set_upre): the kernel's own operations, same bits
    assert torch.equal(outs[(1, 1, 0)], outs[(1, 0, 0)])
    # grouped workgroup orders (lea_conv3d_wino44_set_group; 3: partial edge groups): same bits
    assert all(torch.equal(outs[(1, 0, g)], outs[(1, 0, 0)]) for g in (2, 3, 16))


@pytest.mark.parametrize("mode,b,cin,cout,shape,res", [
    (2, 1, 8, 24, (9, 8, 68), "acc"), (2, 2, 8, 32, (5, 6, 40), None),
    (3, 1, 16, 16, (11, 20, 40), "acc"), (3, 2, 16, 16, (5, 9, 36), "res"), (3, 1, 32, 16, (4, 13, 68), None),
    (3, 1, 16, 12, (6, 10, 44), "acc")])
def test_wino44_modes_vs_float64(mode, b, cin, cout, shape, res):
    """lea_conv3d_wino44_set modes 2 (the two-chunk layers on the F(4,3) x F(4,3) tile) and 3
    (also the 16-cout layers, as half-empty 32-cout blocks) against float64 torch."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin + 5 * cout + shape[2])
    x = torch.randn((b, cin) + shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = torch.randn((b, cout) + shape, generator=g)
    want = _ref(x, w, scale, shift, True, r if res else None)
    pw = kernels.pack_conv_weight_wino(w.to(DEV))
    assert lib.lea_conv3d_wino44_set(mode) == 0
    try:
        assert kernels.wino_kernel_name(b, cout, *shape, cin=cin) == "conv3d_wino44_kernel"
        out = r.to(DEV).clone() if res == "acc" else None
        y = kernels.conv3d_bnrelu_wino(x.to(DEV), pw, cout, scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                       accumulate=res == "acc", residual=r.to(DEV) if res == "res" else None)
    finally:
        lib.lea_conv3d_wino44_set(int(os.environ.get("LEASTEREO_WINO44") or W44_DEFAULT))
    np.testing.assert_allclose(y.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cin,cout,shape", [(32, 32, (64, 192, 320)), (128, 64, (32, 96, 160)),
                                            (128, 32, (34, 98, 156))])
def test_wino44_grouped_order_on_large_grids(cin, cout, shape):
    """The grouped workgroup order the F(4,3) x F(4,3) tile takes by itself on grids of >= 2048
    workgroups (lea_conv3d_wino44_set_group(-1): stem1 and conv1/2 at C2, 3840 workgroups; the
    third shape, 2205 workgroups, ragged in every axis: partial boxes at every edge) writes the linear order's
    bits, and every output is written (against float64 on a sampled window)."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(cin + cout)
    x = torch.randn((1, cin) + shape, device=DEV, generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device=DEV, generator=g) / np.sqrt(cin * 27)
    scale = torch.rand(cout, device=DEV, generator=g) + 0.5
    shift = torch.randn(cout, device=DEV, generator=g) * 0.1
    pw = kernels.pack_conv_weight_wino(w)
    outs = []
    try:
        for grp in (0, -1, 16):
            assert lib.lea_conv3d_wino44_set_group(grp) == 0
            y = torch.full((1, cout) + shape, float("nan"), device=DEV)
            kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y)
            outs.append(y)
    finally:
        lib.lea_conv3d_wino44_set_group(W44G_DEFAULT)
    assert kernels.wino_kernel_name(1, cout, *shape, cin=cin) == "conv3d_wino44_kernel"
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[1], outs[0]) and torch.equal(outs[2], outs[0])
    # a window at the far corner (the last, partial box) against float64
    d0, h0, w0 = shape[0] - 6, shape[1] - 7, shape[2] - 40
    xs = x[:, :, d0 - 1:, h0 - 1:, w0 - 1:].double().cpu()
    want = F.conv3d(F.pad(xs, (0, 1, 0, 1, 0, 1)), w.double().cpu())
    want = torch.relu(want * scale.double().cpu().view(1, -1, 1, 1, 1) + shift.double().cpu().view(1, -1, 1, 1, 1))
    np.testing.assert_allclose(outs[0][:, :, d0:, h0:, w0:].double().cpu().numpy(), want.numpy(),
                               rtol=1e-4, atol=1e-4)
