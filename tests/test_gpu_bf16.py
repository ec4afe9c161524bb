"""GPU parity of the bf16 path (configs 3/4) against float64 torch on the same
bf16-rounded inputs and weights.

Tolerances: activations and weights are bf16 (8-bit mantissa), sums are f32 and
outputs are rounded to bf16 again, so per op |d| <= 1e-2 * max|ref| (two bf16
ulps at the output scale); layout converters and the cost-volume stem0 are exact.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from leastereo_amd import kernels
from oracle import torch_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _close(got, want, rel=1e-2):
    got, want = got.double().cpu(), want.double().cpu()
    scale = float(want.abs().max()) + 1e-6
    err = float((got - want).abs().max())
    assert err <= rel * scale, (err, scale)


def test_c8_round_trip_is_exact_bf16_rounding():
    x = torch.randn(2, 24, 3, 5, 7, device=DEV)
    y = kernels.from_c8(kernels.to_c8(x))
    assert torch.equal(y, _bf(x))


@pytest.mark.parametrize("b,cin,cout,k,shape,mode", [
    (1, 8, 8, 3, (5, 9, 40), None), (1, 16, 16, 3, (4, 12, 33), "acc"), (2, 32, 32, 3, (3, 8, 20), None),
    (1, 64, 32, 3, (6, 20, 70), None), (1, 16, 48, 3, (4, 9, 40), None), (1, 32, 96, 3, (3, 6, 21), "res"),
    (1, 8, 24, 3, (3, 10, 17), None), (2, 64, 8, 1, (3, 7, 11), None), (1, 32, 16, 1, (4, 6, 40), None),
    (1, 128, 32, 1, (2, 5, 33), None), (1, 32, 32, 1, (3, 4, 50), None)])
def test_conv_bf16_vs_torch(b, cin, cout, k, shape, mode):
    g = torch.Generator().manual_seed(cin * 13 + cout + k)
    x = _bf(torch.randn((b, cin) + shape, generator=g))
    w = _bf(torch.randn(cout, cin, k, k, k, generator=g) / np.sqrt(cin * k ** 3))
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = _bf(torch.randn((b, cout) + shape, generator=g))
    want = F.conv3d(x.double(), w.double(), None, 1, k // 2)
    want = torch.relu(want * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    if mode:
        want = want + r.double()
    xc = kernels.to_c8(x.to(DEV))
    rc = kernels.to_c8(r.to(DEV))
    out = rc.clone() if mode == "acc" else None
    y = kernels.conv3d_bnrelu_bf16(xc, kernels.pack_conv_weight_bf16(w.to(DEV)), cout, k,
                                   scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                   accumulate=mode == "acc", residual=rc if mode == "res" else None)
    _close(kernels.from_c8(y), want)


def test_conv_bf16_two_sources_and_block_slices():
    """cat(x, x2) read in place; output into a block slice of a bigger buffer."""
    g = torch.Generator().manual_seed(5)
    x = _bf(torch.randn(1, 64, 4, 9, 40, generator=g))
    x2 = _bf(torch.randn(1, 64, 4, 9, 40, generator=g))
    w = _bf(torch.randn(64, 128, 3, 3, 3, generator=g) / np.sqrt(128 * 27))
    want = F.conv3d(torch.cat((x, x2), 1).double(), w.double(), None, 1, 1)
    big = torch.zeros(1, 12, 4, 9, 40, 8, device=DEV, dtype=torch.bfloat16)
    kernels.conv3d_bnrelu_bf16(kernels.to_c8(x.to(DEV)), kernels.pack_conv_weight_bf16(w.to(DEV)), 64,
                               3, None, None, relu=False, out=big[:, 2:10], x2=kernels.to_c8(x2.to(DEV)))
    _close(kernels.from_c8(big[:, 2:10].contiguous()), want)
    assert float(big[:, :2].float().abs().sum()) == 0 and float(big[:, 10:].float().abs().sum()) == 0


@pytest.mark.parametrize("c,cout,maxdisp,hw", [(32, 32, 48, (12, 40)), (16, 16, 27, (5, 19))])
def test_costvolume_stem0_bf16_is_bit_identical(c, cout, maxdisp, hw):
    g = torch.Generator().manual_seed(c + maxdisp)
    fl = torch.randn((2, c) + hw, generator=g).to(DEV)
    fr = torch.randn((2, c) + hw, generator=g).to(DEV)
    w = (torch.randn(cout, 2 * c, 3, 3, 3, generator=g) / np.sqrt(2 * c * 27)).to(DEV)
    packed = kernels.pack_conv_weight_bf16(w)
    scale = torch.rand(cout, device=DEV) + 0.5
    shift = torch.randn(cout, device=DEV) * 0.1
    cost = kernels.to_c8(kernels.build_cost_volume(fl, fr, maxdisp))
    want = kernels.conv3d_bnrelu_bf16(cost, packed, cout, 3, scale, shift)
    got = kernels.conv3d_bnrelu_costvolume_bf16(kernels.to_c8(fl), kernels.to_c8(fr), maxdisp, packed,
                                                cout, scale, shift)
    assert torch.equal(got, want)


@pytest.mark.parametrize("src,dst,ac", [((4, 6, 10), (8, 12, 20), True), ((9, 13, 17), (5, 7, 9), True),
                                        ((4, 6, 10), (12, 18, 30), False)])
def test_resample_bf16_vs_torch(src, dst, ac):
    g = torch.Generator().manual_seed(3)
    x = _bf(torch.randn((2, 16) + src, generator=g))
    scale = torch.rand(16, generator=g) + 0.5
    shift = torch.randn(16, generator=g) * 0.1
    want = torch.relu(F.interpolate(x.double(), dst, mode="trilinear", align_corners=ac)
                      * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    y = kernels.resample_trilinear_bf16(kernels.to_c8(x.to(DEV)), dst, ac, None, scale.to(DEV),
                                        shift.to(DEV), relu=True)
    _close(kernels.from_c8(y), want)


@pytest.mark.parametrize("src,dst,ac", [((16, 24, 40), (32, 48, 80), True), ((5, 7, 9), (9, 13, 17), True),
                                        ((8, 12, 20), (16, 24, 40), False), ((9, 13, 17), (5, 7, 9), True),
                                        ((16, 48, 80), (32, 96, 160), True)])
def test_resample_bf16_is_the_f32_kernel_rounded(src, dst, ac):
    """The c8 resample (up and down) evaluates the f32 engine's trilinear expression
    in the same order: bit-identical after rounding to bf16."""
    g = torch.Generator().manual_seed(5)
    x = _bf(torch.randn((1, 16) + src, generator=g)).to(DEV)
    scale = (torch.rand(16, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(16, generator=g) * 0.1).to(DEV)
    got = kernels.from_c8(kernels.resample_trilinear_bf16(kernels.to_c8(x), dst, ac, None, scale, shift,
                                                          relu=True))
    want = kernels.resample_trilinear(x, dst, ac, None, scale, shift, relu=True)
    assert torch.equal(got, want.to(torch.bfloat16).float())


@pytest.mark.parametrize("b,c,src,dst,ac", [(2, 24, (5, 7, 9), (9, 13, 17), True),
                                            (1, 8, (32, 96, 160), (64, 192, 320), True),
                                            (2, 16, (16, 48, 80), (32, 96, 160), True),
                                            (1, 16, (8, 12, 20), (16, 24, 70), False),
                                            (1, 8, (3, 40, 33), (5, 79, 130), True)])
def test_resample_bf16_cols_kernel_is_the_gather_kernel(b, c, src, dst, ac):
    """The up-sampling column walker (resample_c8_cols_kernel: source rows W-lerped once per
    wave into registers) gives the per-output gather kernel's bits, into a channel slice too
    (odd sizes, a partial last column tile, the last source row pairing with itself)."""
    from leastereo_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(b * 100 + c)
    x = kernels.to_c8(torch.randn((b, c) + src, generator=g).to(DEV))
    scale = (torch.rand(c, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(c, generator=g) * 0.1).to(DEV)
    outs = []
    try:
        for cols in (0, 1, 2):  # gather, column walker R = 8, R = 16
            assert lib.lea_resample_bf16_set_cols(cols) == 0
            big = torch.full((b, c // 8 + 2) + tuple(dst) + (8,), 7.0, device=DEV, dtype=torch.bfloat16)
            kernels.resample_trilinear_bf16(x, dst, ac, big[:, 1:1 + c // 8], scale, shift, relu=True)
            outs.append(big)
    finally:
        lib.lea_resample_bf16_set_cols(1)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert bool((outs[1][:, 0] == 7.0).all()) and bool((outs[1][:, -1] == 7.0).all())


def test_tapsum_bf16_matches_f32_on_same_values():
    g = torch.Generator().manual_seed(9)
    q = _bf(torch.randn(1, 32, 8, 12, 20, generator=g)).to(DEV)  # 27 taps + 5 pad channels
    got = kernels.tapsum_upsample_bf16(kernels.to_c8(q), 1, (16, 24, 40))
    want = kernels.tapsum_upsample(q[:, :27].contiguous(), 1, (16, 24, 40))
    np.testing.assert_allclose(got.cpu().numpy(), want.cpu().numpy(), rtol=1e-6, atol=1e-6)


# ----------------------------------------------------------------------- end to end
def _model(maxdisp, precision):
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from tests.golden_util import state_dict
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=maxdisp)), DEV, precision=precision)
    m.load_state_dict(state_dict(), strict=True)
    return m.to(DEV).eval()


def test_bf16_e2e_vs_reference_fixture():
    """bf16 matching net vs the reference's f32 disparity (e2e fixture).  No bf16
    tolerance is stated upstream; measured r01: 0.06 px EPE (disparity std 3.6 px)."""
    from tests.golden_util import golden, meta, normal
    c = meta()["cases"]["e2e/b1_h96_w192_md48"]
    left = normal(c["seeds"][0], (1, 3, 96, 192)).to(DEV)
    right = normal(c["seeds"][1], (1, 3, 96, 192)).to(DEV)
    with torch.no_grad():
        d = _model(48, "bf16")(left, right).cpu()
    assert torch.isfinite(d).all()
    assert ref.epe(d, torch.from_numpy(golden("e2e")["b1_h96_w192_md48/disp32"])) < 0.25


def _bf16_noise(cfg):
    """The reference network's own bf16 noise at this config (tests/golden/bf16_noise.json,
    tools/gen_bf16_noise.py: /root/reference's LEAStereo imported and run with bf16 feature +
    matching nets and an f32 Disp vs itself in f32, EPE px of each of the 8 pairs the test
    runs, and pair 0's relative L2 distance per stage; the oracle restatement gives the same
    figures bit for bit, bf16_noise_oracle.json / agreement_with_oracle)."""
    import json
    import os
    from tests.golden_util import GOLD
    with open(os.path.join(GOLD, "bf16_noise.json")) as f:
        return json.load(f)["cases"][cfg]


def _bf16_measured(cfg):
    """The HIP bf16 path's own measured figures at this config (tests/golden/
    bf16_hip_measured.json, written by this test under LEA_BF16_RECORD=1 on the GPU box):
    the worst pair's EPE and pair 0's per-stage relative L2 distance to the f32 oracle."""
    import json
    import os
    from tests.golden_util import GOLD
    path = os.path.join(GOLD, "bf16_hip_measured.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)["cases"].get(cfg)


# regression bar: the HIP bf16 path may drift at most this factor above its own recorded
# figures (worst pair's EPE, each stage's relative L2) ...
BF16_MEASURED_FACTOR = 1.2
# ... and may never be noisier than the reference network run in bf16 at its worst pair /
# at the same stage (the reference-anchored bar; HIP accumulates and normalises in f32)
BF16_REFERENCE_FACTOR = 1.0


def bf16_bars(cfg, e_bf, stages, measured=True):
    """The bf16 acceptance rule, as a function so the test can also show it REJECTS an
    injected error: returns the list of violated bars (empty = pass); ``measured=False``
    applies the reference-anchored bars only (when re-recording the HIP figures)."""
    noise, meas = _bf16_noise(cfg), (_bf16_measured(cfg) if measured else None)
    bad = []
    if max(e_bf) > BF16_REFERENCE_FACTOR * max(noise["epe_px"]):
        bad.append(f"EPE {max(e_bf):.4f} > {BF16_REFERENCE_FACTOR} x reference bf16 worst pair "
                   f"{max(noise['epe_px']):.4f}")
    if meas is not None and max(e_bf) > BF16_MEASURED_FACTOR * meas["epe_max"]:
        bad.append(f"EPE {max(e_bf):.4f} > {BF16_MEASURED_FACTOR} x recorded worst pair {meas['epe_max']:.4f}")
    for k, v in stages.items():
        ref_v = noise["stage_rel_l2_pair0"].get(k)
        if ref_v is not None and v > BF16_REFERENCE_FACTOR * ref_v:
            bad.append(f"stage {k}: rel L2 {v:.3e} > reference bf16 {ref_v:.3e}")
        if meas is not None and k in meas["stage_rel_l2_pair0"] and v > BF16_MEASURED_FACTOR * meas[
                "stage_rel_l2_pair0"][k]:
            bad.append(f"stage {k}: rel L2 {v:.3e} > {BF16_MEASURED_FACTOR} x recorded "
                       f"{meas['stage_rel_l2_pair0'][k]:.3e}")
    return bad


def _record(name, values):
    """Measured EPEs land in gpurun_out/ when the suite runs on the GPU box."""
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "bf16_epe.jsonl"), "a") as f:
            f.write(json.dumps({"test": name, "epe_px": values}) + "\n")


def _rel_l2(a, r):
    a, r = a.double(), r.double()
    return float(torch.linalg.vector_norm(a - r) / torch.linalg.vector_norm(r).clamp_min(1e-30))


def _stages_pair0(mb, left, right, md, sd, a):
    """Pair 0 through the HIP bf16 model with the executors' stage taps, then through the
    f32 oracle with its taps: relative L2 per stage (feature maps, stem0/1, conv1/2, each
    cell, the matching cost; oracle/torch_ref.matching_forward names them)."""
    hip = {}
    ex = mb.matching.executor()
    ex.tap = lambda k, t: hip.__setitem__(k, t.cpu())
    try:
        with torch.no_grad():
            mb(left, right)
            fx = mb.feature(left)
            fy = mb.feature(right)
            hip["fea_l"], hip["fea_r"] = (kernels.from_c8(f)[:, :, 0].cpu() if f.dim() == 6 else f.cpu()
                                          for f in (fx, fy))
    finally:
        ex.tap = None
    out = {}
    with torch.no_grad():
        ref.leastereo_forward(sd, left.cpu(), right.cpu(), md, a,
                              tap=lambda k, t: out.__setitem__(k, _rel_l2(hip.pop(k), t)))
    return out


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_bf16_batch8_vs_oracle(cfg):
    """Configs 3 (KITTI 384x1248 D192, bf16, batch 8) and 4 (576x960 D192, bf16, the
    8 pairs of one GPU's shard): every pair of the batch vs the f32 CPU oracle
    (oracle/torch_ref.leastereo_forward) and pair 0 stage by stage (relative L2), under
    bf16_bars: no noisier than the reference network itself run in bf16 (its worst pair
    of the same 8, its same stage) and within 1.2 x the HIP path's recorded figures; the
    rule rejects the same outputs with their error doubled (checked here on every run);
    the f32 HIP path on the same batch vs the oracle at the f32 bar (1e-3 px); and the
    batch equals eight single-pair runs bit for bit."""
    import json
    import os
    from tests.golden_util import arch, normal, state_dict
    case = _bf16_noise(cfg)
    h, w, md, seed = case["height"], case["width"], case["maxdisp"], case["seed"]
    pairs = [(normal(seed + 2 * i, (1, 3, h, w)), normal(seed + 2 * i + 1, (1, 3, h, w)))
             for i in range(8)]
    left = torch.cat([p[0] for p in pairs]).to(DEV)
    right = torch.cat([p[1] for p in pairs]).to(DEV)
    mb, mf = _model(md, "bf16"), _model(md, "f32")
    sd, a = state_dict(), arch()
    with torch.no_grad():
        db, df = mb(left, right).cpu(), mf(left, right).cpu()
        one = torch.cat([mb(left[i:i + 1], right[i:i + 1]) for i in range(8)]).cpu()
        want = torch.cat([ref.leastereo_forward(sd, l, r, md, a) for l, r in pairs])
    assert torch.equal(db, one)
    e_bf = [ref.epe(db[i], want[i]) for i in range(8)]
    e_f32 = [ref.epe(df[i], want[i]) for i in range(8)]
    stages = _stages_pair0(mb, left[:1], right[:1], md, sd, a)
    _record(f"bf16_batch8_vs_oracle[{cfg}]", {"bf16": e_bf, "f32": e_f32, "stages": stages,
                                              "reference_bf16": case["epe_px"]})
    assert max(e_f32) < 1e-3, e_f32
    assert not bf16_bars(cfg, e_bf, stages, measured=False), bf16_bars(cfg, e_bf, stages, measured=False)
    if os.environ.get("LEA_BF16_RECORD"):  # (re)record this path's figures, GPU box only
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                            "bf16_hip_measured.json")
        rec = json.load(open(path)) if os.path.exists(path) else {
            "what": "HIP bf16 path vs the f32 oracle: worst pair EPE (px) of the 8 pairs and pair 0's "
                    "relative L2 per stage (tests/test_gpu_bf16.py under LEA_BF16_RECORD=1)", "cases": {}}
        rec["cases"][cfg] = {"epe_max": max(e_bf), "epe_px": e_bf, "stage_rel_l2_pair0": stages}
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
        return  # (the error-injection checks below need the recorded figures)
    bad = bf16_bars(cfg, e_bf, stages)
    assert not bad, bad
    assert _bf16_measured(cfg) is not None, "tests/golden/bf16_hip_measured.json lacks " + cfg
    # the rule is sharp enough to see a doubled error: the same disparities / stages with
    # twice their distance to the oracle must fail it
    e2 = [ref.epe(want[i] + 2 * (db[i] - want[i]), want[i]) for i in range(8)]
    assert bf16_bars(cfg, e2, {k: 2 * v for k, v in stages.items()}), "bars do not reject a 2x error"
    assert bf16_bars(cfg, e_bf, {k: (2 * v if k == "cell10" else v) for k, v in stages.items()}), \
        "bars do not reject a 2x error in one stage"


def test_conv2d_bf16_vs_torch():
    g = torch.Generator().manual_seed(17)
    for b, cin, cout, hw, mode in [(2, 32, 32, (24, 40), None), (4, 8, 8, (19, 33), "res"),
                                   (1, 16, 16, (9, 20), "acc")]:
        x = _bf(torch.randn((b, cin) + hw, generator=g))
        w = _bf(torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9))
        scale = torch.rand(cout, generator=g) + 0.5
        shift = torch.randn(cout, generator=g) * 0.1
        r = _bf(torch.randn((b, cout) + hw, generator=g))
        want = F.conv2d(x.double(), w.double(), None, 1, 1)
        want = torch.relu(want * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1))
        if mode:
            want = want + r.double()
        rc = kernels.to_c8(r.to(DEV))
        y = kernels.conv2d_bnrelu_bf16(kernels.to_c8(x.to(DEV)), kernels.pack_conv2d_weight_bf16(w.to(DEV)),
                                       cout, scale.to(DEV), shift.to(DEV), relu=True,
                                       out=rc.clone() if mode == "acc" else None,
                                       accumulate=mode == "acc", residual=rc if mode == "res" else None)
        _close(kernels.from_c8(y)[:, :, 0], want)


def test_bf16_feature_net_vs_f32():
    """bf16 feature maps (c8) vs the f32 feature net on the same images."""
    from tests.golden_util import normal
    mb, mf = _model(48, "bf16"), _model(48, "f32")
    x = normal(31, (2, 3, 96, 192)).to(DEV)
    with torch.no_grad():
        fb = kernels.from_c8(mb.feature(x))[:, :, 0]
        ff = mf.feature(x)
    _close(fb, ff, rel=5e-2)


# ---- D-streaming kernel for the single-chunk 3x3x3 layers (cin <= 16) ----

@pytest.mark.parametrize("b,cin,cout,shape,mode", [
    (1, 8, 8, (64, 24, 40), "acc"), (2, 8, 8, (9, 13, 37), "res"), (1, 16, 16, (32, 12, 33), "acc"),
    (2, 16, 16, (7, 9, 20), None), (1, 8, 24, (16, 17, 50), None), (1, 16, 48, (12, 9, 40), None),
    (1, 8, 8, (4, 3, 5), "acc"), (1, 16, 16, (5, 8, 16), "res"), (3, 8, 16, (6, 10, 31), "acc"),
    # two K chunks (cin = 32: stem1, the L2 cells and their sibling groups)
    (1, 32, 32, (16, 12, 40), "acc"), (2, 32, 16, (9, 13, 37), None), (1, 32, 32, (24, 20, 48), None),
    (1, 32, 24, (6, 9, 20), "res")])
def test_stream_kernel_is_the_tile_kernel(b, cin, cout, shape, mode):
    """The streaming kernel (ring of planes along D, weights in registers, residual by
    LDS-DMA; one or two K chunks) computes the tile kernel's sums in the same order:
    bit-identical outputs,
    on odd D (a half last step), ragged H/W, column segments along D, every epilogue,
    an output block slice, and vs float64 torch within the bf16 tolerance."""
    from leastereo_amd import _lib
    lib = _lib.load()
    d, h, w = shape
    g = torch.Generator().manual_seed(cin + cout + d)
    x = _bf(torch.randn((b, cin) + shape, generator=g))
    wt = _bf(torch.randn(cout, cin, 3, 3, 3, generator=g) / np.sqrt(cin * 27))
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = _bf(torch.randn((b, cout) + shape, generator=g))
    xc, rc = kernels.to_c8(x.to(DEV)), kernels.to_c8(r.to(DEV))
    packed = kernels.pack_conv_weight_bf16(wt.to(DEV))
    outs = []
    for variant in (0, 1):
        assert lib.lea_conv3d_bf16_set_variant(variant) == 0
        try:
            name = kernels.conv_kernel_name_bf16(b, cout, cin, d, h, w, 3)
            assert name.startswith("conv_bf16_stream_kernel<" if variant == 0 else "conv_bf16_kernel<"), name
            big = torch.zeros((b, cout // 8 + 2, d, h, w, 8), device=DEV, dtype=torch.bfloat16)
            big[:, 1:1 + cout // 8] = rc
            out = big[:, 1:1 + cout // 8]
            kernels.conv3d_bnrelu_bf16(xc, packed, cout, 3, scale.to(DEV), shift.to(DEV), relu=True,
                                       out=out if mode == "acc" else (out if mode is None else out),
                                       accumulate=mode == "acc", residual=rc if mode == "res" else None)
            torch.cuda.synchronize()
            assert float(big[:, 0].float().abs().sum()) == 0 and float(big[:, -1].float().abs().sum()) == 0
            outs.append(out.clone())
        finally:
            lib.lea_conv3d_bf16_set_variant(0)
    assert torch.equal(outs[0], outs[1])
    want = F.conv3d(x.double(), wt.double(), None, 1, 1)
    want = torch.relu(want * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    if mode:
        want = want + r.double()
    _close(kernels.from_c8(outs[0]), want)


@pytest.mark.parametrize("b,cin,cout,src,dst", [
    (2, 32, 16, (8, 12, 20), (4, 6, 10)), (1, 64, 64, (9, 13, 17), (5, 7, 9)),
    (1, 128, 32, (6, 10, 14), (3, 5, 7)), (3, 32, 32, (1, 12, 40), (1, 6, 20)),
    (1, 64, 16, (7, 9, 11), (7, 9, 11))])
def test_conv1x1_resampled_is_resample_then_conv(b, cin, cout, src, dst):
    """lea_conv1x1_resampled_bf16 == lea_resample3d_trilinear_bf16 + the k = 1 tile
    kernel, bit for bit (the same bf16 rounding of the interpolated words, the same
    MFMA chunk order); the same-size case is the plain 1x1."""
    g = torch.Generator().manual_seed(cin + cout + src[0])
    x = kernels.to_c8(torch.randn((b, cin) + src, generator=g).to(DEV))
    w = (torch.randn(cout, cin, 1, 1, 1, generator=g) / np.sqrt(cin)).to(DEV)
    scale = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    packed = kernels.pack_conv_weight_bf16(w)
    want = kernels.conv3d_bnrelu_bf16(kernels.resample_trilinear_bf16(x, dst, True), packed, cout, 1,
                                      scale, shift, relu=True)
    got = kernels.conv1x1_resampled_bf16(x, dst, packed, cout, scale, shift, relu=True)
    assert torch.equal(got, want)
    big = torch.zeros((b, cout // 8 + 2) + tuple(dst) + (8,), device=DEV, dtype=torch.bfloat16)
    kernels.conv1x1_resampled_bf16(x, dst, packed, cout, scale, shift, relu=True, out=big[:, 1:1 + cout // 8])
    assert torch.equal(big[:, 1:1 + cout // 8], want)
    assert float(big[:, 0].float().abs().sum()) == 0 and float(big[:, -1].float().abs().sum()) == 0


@pytest.mark.parametrize("b,cin,cout,shape,mode,cin2", [
    (1, 32, 16, (8, 12, 20), None, 0), (2, 64, 32, (5, 9, 17), "acc", 0), (1, 128, 64, (4, 6, 10), None, 0),
    (3, 24, 8, (3, 5, 7), "res", 0), (1, 64, 96, (2, 8, 9), None, 0), (2, 8, 24, (6, 7, 5), "acc", 0),
    (1, 64, 32, (4, 12, 16), None, 32), (2, 48, 16, (3, 4, 33), "res", 16)])
def test_stream_1x1_is_the_tile_kernel(b, cin, cout, shape, mode, cin2):
    """The streamed 1x1 (conv1x1_c8_kernel: B words loaded per lane, no staging) stores
    what the k = 1 tile kernel stores, bit for bit: padded chunks (cin % 32 != 0), several
    cout blocks, two sources (a block-slice cat), residual and accumulate epilogues, an
    output block slice; and matches float64 torch within the bf16 tolerance."""
    from leastereo_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin * 3 + cout + b)
    x = _bf(torch.randn((b, cin) + shape, generator=g))
    wt = _bf(torch.randn(cout, cin, 1, 1, 1, generator=g) / np.sqrt(cin))
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    r = _bf(torch.randn((b, cout) + shape, generator=g))
    xc, rc = kernels.to_c8(x.to(DEV)), kernels.to_c8(r.to(DEV))
    x1, x2 = (xc[:, : (cin - cin2) // 8], xc[:, (cin - cin2) // 8:]) if cin2 else (xc, None)
    packed = kernels.pack_conv_weight_bf16(wt.to(DEV))
    outs = []
    for on in (1, 0):
        assert lib.lea_conv3d_bf16_set_stream1x1(on) == 0
        try:
            name = kernels.conv_kernel_name_bf16(b, cout, cin, *shape, 1)
            assert name.startswith("conv1x1_c8_kernel<" if on else "conv_bf16_kernel<1,"), name
            big = torch.zeros((b, cout // 8 + 2) + shape + (8,), device=DEV, dtype=torch.bfloat16)
            big[:, 1:1 + cout // 8] = rc
            out = big[:, 1:1 + cout // 8]
            kernels.conv3d_bnrelu_bf16(x1, packed, cout, 1, scale.to(DEV), shift.to(DEV), relu=True, out=out,
                                       accumulate=mode == "acc", x2=x2, residual=rc if mode == "res" else None)
            torch.cuda.synchronize()
            assert float(big[:, 0].float().abs().sum()) == 0 and float(big[:, -1].float().abs().sum()) == 0
            outs.append(out.clone())
        finally:
            lib.lea_conv3d_bf16_set_stream1x1(1)
    assert torch.equal(outs[0], outs[1])
    want = F.conv3d(x.double(), wt.double())
    want = torch.relu(want * scale.double().view(1, -1, 1, 1, 1) + shift.double().view(1, -1, 1, 1, 1))
    if mode:
        want = want + r.double()
    _close(kernels.from_c8(outs[0]), want)


@pytest.mark.parametrize("split", [3, 2, 1, 0])
@pytest.mark.parametrize("c,shape", [(16, (6, 9, 40)), (8, (5, 12, 33)), (16, (4, 4, 16)), (8, (8, 20, 64)),
                                     (8, (4, 9, 17))])
def test_pair_sum_bf16_vs_torch(c, shape, split):
    """LEA_PAIR_SUM on the bf16 engine (a matching-cell step: relu(BN_a(conv_a(xa))) +
    relu(BN_b(conv_b(xb))) in one launch) -- the split-wave pair kernel (split 1; split 2 with
    the plane-paired tile for the 8 -> 8 steps; split 3, the default: that tile for the 8 -> 8
    steps, the 16-channel ones as split 0) and the D-streaming kernel with both convs per wave
    (split 0) -- against float64 torch on the same bf16 operands, written into a block slice of
    a cat buffer; odd D / ragged H, W."""
    from leastereo_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(c * 3 + shape[0])
    xa, xb = _bf(torch.randn((2, c) + shape, generator=g)), _bf(torch.randn((2, c) + shape, generator=g))
    wa = _bf(torch.randn(c, c, 3, 3, 3, generator=g) / np.sqrt(c * 27))
    wb = _bf(torch.randn(c, c, 3, 3, 3, generator=g) / np.sqrt(c * 27))
    sc, sh = torch.rand(2 * c, generator=g) + 0.5, torch.randn(2 * c, generator=g) * 0.1

    def branch(x, w, s, t):
        y = F.conv3d(x.double(), w.double(), None, 1, 1)
        return torch.relu(y * s.double().view(1, -1, 1, 1, 1) + t.double().view(1, -1, 1, 1, 1))
    want = branch(xa, wa, sc[:c], sh[:c]) + branch(xb, wb, sc[c:], sh[c:])
    packed = torch.cat([kernels.pack_conv_weight_bf16(wa.to(DEV)), kernels.pack_conv_weight_bf16(wb.to(DEV))])
    big = torch.full((2, c // 8 + 2) + shape + (8,), 5.0, device=DEV, dtype=torch.bfloat16)
    out = big[:, 1:1 + c // 8]
    xa8, xb8 = kernels.to_c8(xa.to(DEV)), kernels.to_c8(xb.to(DEV))
    assert kernels.pair_sum_supported_bf16(xa8, xb8, out)
    try:
        assert lib.lea_conv3d_bf16_set_pair_split(split) == 0
        kernels.conv3d_bnrelu_bf16(xa8, packed, c, 3, sc.to(DEV), sh.to(DEV), True, out, x2=xb8, pair_sum=True)
    finally:
        lib.lea_conv3d_bf16_set_pair_split(3)
    _close(kernels.from_c8(out.contiguous()), want)
    assert bool((big[:, 0] == 5.0).all()) and bool((big[:, -1] == 5.0).all())
