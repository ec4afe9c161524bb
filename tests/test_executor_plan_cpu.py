"""The cell-graph executors' launch plans, checked on the CPU.

``FeatureExecutor`` (new_model_2d.py:140-165) turns a searched cell into a few fused
launches: the s1 sibling group (one conv writing consecutive cat slots), the s0 pair
(two ops on s0 in one launch writing two slots, lea_conv2d_bnrelu_pair), skip terms as
epilogue residuals and the remaining ops accumulating into their slots.  Which launch
writes a slot first and which accumulate depends on the genotype, so a plan that is
right for the shipped genotype can be wrong for another (a genotype whose
s1 group covers a step of the s0 pair).

These tests replace the library's launches by plain torch ops with the same contract
(packed weights = the raw weights; ``out``/``accumulate``/``residual`` semantics of
kernels.py) and run the executor in float64 on CPU against the oracle
(oracle/torch_ref.feature_forward, itself pinned to the reference's fixtures): the
executor's graph logic is then the only thing under test.  The HIP arithmetic is
covered by the -m gpu tests.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from leastereo_amd import executor as ex
from leastereo_amd import kernels
from leastereo_amd.config import LEAStereoArgs, default_arch_args
from leastereo_amd.model import LEAStereo
from leastereo_amd.weights import synthetic_state_dict
from oracle import torch_ref as ref
from tests.golden_util import arch, normal


def _act(z, scale, shift, relu):
    if scale is not None:
        z = z * scale.view(1, -1, 1, 1, 1).to(z.dtype) + shift.view(1, -1, 1, 1, 1).to(z.dtype)
    return z.clamp_min(0) if relu else z


def _emit(y, out, accumulate, residual):
    if residual is not None:
        y = y + residual
    if out is None:
        return y
    if accumulate:
        out.add_(y)
    else:
        out.copy_(y)
    return out


class FakeKernels:
    """torch stand-ins for the launches the f32 feature executor issues."""

    def __init__(self):
        self.log = []

    @staticmethod
    def pack_conv2d_weight(w):
        return w.detach().clone()

    @staticmethod
    def pack_conv_weight(w):
        return w.detach().clone()

    def conv2d_bnrelu(self, x, packed, cout, scale, shift, relu=True, out=None, accumulate=False,
                      residual=None):
        self.log.append(("conv2d", out.data_ptr() if out is not None else None, accumulate))
        z = F.conv2d(x[:, :, 0], packed.to(x.dtype), padding=1).unsqueeze(2)
        return _emit(_act(z, scale, shift, relu), out, accumulate, residual)

    def conv2d_bnrelu_pair(self, x, packed, c1, cout, scale, shift, relu, out1, out2, residual=None):
        self.log.append(("pair", out1.data_ptr(), out2.data_ptr()))
        y = _act(F.conv2d(x[:, :, 0], packed.to(x.dtype), padding=1).unsqueeze(2), scale, shift, relu)
        _emit(y[:, :c1], out1, False, residual)
        _emit(y[:, c1:], out2, False, None)

    def conv2d_s3_bnrelu(self, x, w, scale, shift, relu=True):
        z = F.conv2d(x[:, :, 0], w.to(x.dtype), stride=3, padding=1).unsqueeze(2)
        return _act(z, scale, shift, relu)

    def conv3d_bnrelu(self, x, packed, cout, k, scale, shift, relu=True, out=None, accumulate=False,
                      x2=None, residual=None):
        if x2 is not None:
            x = torch.cat((x, x2), 1)
        z = F.conv3d(x, packed.to(x.dtype), padding=k // 2)
        return _emit(_act(z, scale, shift, relu), out, accumulate, residual)

    def conv3d_bnrelu_resampled(self, x, size, packed, cout, k, scale, shift, relu=True, out=None,
                                accumulate=False):
        x = F.interpolate(x, size=tuple(size), mode="trilinear", align_corners=True)
        return self.conv3d_bnrelu(x, packed, cout, k, scale, shift, relu, out, accumulate)

    @staticmethod
    def pack_conv_weight_wino(w):
        return w.detach().clone()

    def conv3d_bnrelu_wino(self, x, packed, cout, scale, shift, relu=True, out=None, accumulate=False,
                           x2=None, residual=None, pair_sum=False):
        self.log.append(("wino", out.data_ptr() if out is not None else None, accumulate, pair_sum))
        if not pair_sum:
            return self.conv3d_bnrelu(x, packed, cout, 3, scale, shift, relu, out, accumulate, x2, residual)
        ca = x.shape[1]
        ya = _act(F.conv3d(x, packed[:, :ca].to(x.dtype), padding=1), scale[:cout], shift[:cout], relu)
        yb = _act(F.conv3d(x2, packed[:, ca:].to(x.dtype), padding=1), scale[cout:], shift[cout:], relu)
        return _emit(ya + yb, out, False, None)

    def tapsum_upsample(self, q, cout, size, scale=None, shift=None, relu=False):
        """sum over the 27 taps of the up-sampled per-tap partial sums, shifted by the tap
        (channel co * 27 + tap): conv3x3x3(upsample(y)) by linearity."""
        d, h, w = (int(v) for v in size)
        up = F.pad(F.interpolate(q, size=(d, h, w), mode="trilinear", align_corners=True), (1, 1, 1, 1, 1, 1))
        y = sum(up[:, co * 27 + (kd * 3 + kh) * 3 + kw::27 * cout][:, :1, kd:kd + d, kh:kh + h, kw:kw + w]
                for co in range(cout) for kd in range(3) for kh in range(3) for kw in range(3)) \
            if cout == 1 else None
        return _act(y, scale, shift, relu)

    def resample_trilinear(self, x, size, align_corners=True, out=None, scale=None, shift=None,
                           relu=False):
        y = _act(F.interpolate(x, size=tuple(size), mode="trilinear", align_corners=align_corners),
                 scale, shift, relu)
        return _emit(y, out, False, None)


@pytest.fixture
def fake(monkeypatch):
    fk = FakeKernels()
    for name in ("pack_conv2d_weight", "pack_conv_weight", "conv2d_bnrelu", "conv2d_bnrelu_pair",
                 "conv2d_s3_bnrelu", "conv3d_bnrelu", "conv3d_bnrelu_resampled", "resample_trilinear",
                 "pack_conv_weight_wino", "conv3d_bnrelu_wino", "tapsum_upsample"):
        monkeypatch.setattr(kernels, name, getattr(fk, name))
    # the stems as two convs (the fused stem kernel has no stand-in here)
    monkeypatch.setattr(ex.FeatureExecutor, "FUSED_STEM", False)
    return fk


# The shipped genotype, and ones whose s1 sibling group overlaps the steps of the s0 pair
# (rows: (state index, primitive), genotypes_2d.py; primitive 1 = 3x3 conv, 0 = skip)
GENOTYPES = {
    "shipped": None,
    # s0 convs at steps 0 and 2 (a pair), s1 convs at steps 0 and 1 (a group covering step 0)
    "group_covers_pair": [[0, 1], [1, 1], [3, 1], [4, 1], [5, 1], [8, 1]],
    # s1 convs at steps 0, 1, 2 (a group covering both pair steps)
    "group_covers_both": [[0, 1], [1, 1], [3, 1], [2, 1], [5, 1], [6, 1]],
    # s1 group at steps 1, 2 beside an s0 pair at steps 0 and 2, skip terms mixed in
    "skips_and_group": [[0, 1], [1, 0], [3, 1], [4, 1], [5, 1], [6, 1]],
}


@pytest.mark.parametrize("pair_s0", [True, False])
@pytest.mark.parametrize("geno", sorted(GENOTYPES))
def test_feature_executor_plan_matches_oracle(tmp_path, fake, monkeypatch, geno, pair_s0):
    monkeypatch.setattr(ex.FeatureExecutor, "PAIR_S0", pair_s0)
    args = LEAStereoArgs(maxdisp=48)
    a = arch()
    if GENOTYPES[geno] is not None:
        a["cell_arch_fea"] = np.array(GENOTYPES[geno])
        args.cell_arch_fea = str(tmp_path / "fea_geno.npy")
        np.save(args.cell_arch_fea, a["cell_arch_fea"])
    args = default_arch_args(args)
    m = LEAStereo(args, "cpu")
    sd = synthetic_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()}, bn_file=None)
    m.load_state_dict(sd, strict=True)
    m = m.double().eval()
    fe = ex.FeatureExecutor(m.feature)
    if geno == "shipped" and pair_s0:
        assert fe.s0_pair, "the shipped genotype's cells run their s0 pair as one launch"
    for i, pair in fe.s0_pair.items():  # a pair never shares a step with the s1 group
        assert not ({k for k, _ in fe.s1_group.get(i, [])} & {k for k, _ in pair})
    x = normal(901, (2, 3, 48, 96)).double()
    with torch.no_grad():
        got = fe.run(x)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        want = ref.feature_forward(sd64, x, a["net_arch_fea"], a["cell_arch_fea"])
    assert got.shape == want.shape
    err = float((got - want).abs().max())
    # folded BN is f32 by design (model.ConvBR.folded_bn): ~1e-7 relative per layer; a plan
    # error (a dropped or doubled term) is O(1)
    assert err <= 1e-5 * float(want.abs().max()), err


# The matching net's cells (skip_model_3d.py:41-75): the shipped genotype (every step two conv
# terms: LEA_PAIR_SUM launches when PAIR_STEPS) and one with a skip term (that cell keeps the
# s1 group + accumulating launches)
MATCHING_GENOTYPES = {"shipped": None, "with_skip": [[1, 1], [0, 1], [3, 1], [4, 0], [8, 1], [6, 1]]}


@pytest.mark.parametrize("pair_steps", [True, False])
@pytest.mark.parametrize("split48", [True, False])
@pytest.mark.parametrize("geno", sorted(MATCHING_GENOTYPES))
def test_matching_executor_plan_matches_oracle(tmp_path, fake, monkeypatch, geno, split48, pair_steps):
    monkeypatch.setattr(ex.MatchingExecutor, "PAIR_STEPS", pair_steps)
    monkeypatch.setattr(ex.MatchingExecutor, "SPLIT_S1_GROUP48", split48)
    monkeypatch.setattr(ex, "CV_STEM", False)
    args = LEAStereoArgs(maxdisp=48)
    a = arch()
    if MATCHING_GENOTYPES[geno] is not None:
        a["cell_arch_mat"] = np.array(MATCHING_GENOTYPES[geno])
        args.cell_arch_mat = str(tmp_path / "mat_geno.npy")
        np.save(args.cell_arch_mat, a["cell_arch_mat"])
    args = default_arch_args(args)
    m = LEAStereo(args, "cpu")
    sd = synthetic_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()}, bn_file=None)
    m.load_state_dict(sd, strict=True)
    m = m.double().eval()
    me = ex.MatchingExecutor(m.matching)
    if pair_steps and geno == "shipped":
        assert len(me.pair_steps) == len(m.matching.cells), "every shipped cell runs as pair launches"
    if geno == "with_skip":
        assert 0 not in me.pair_steps  # every cell has the skip term at step 1
    x = normal(903, (1, 64, 16, 32, 64)).double()  # the e2e case's cost volume shape (96x192 D48)
    with torch.no_grad():
        got = me.run(x)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        want = ref.matching_forward(sd64, x, a["net_arch_mat"], a["cell_arch_mat"])
    pairs = [e for e in fake.log if e[0] == "wino" and e[3]]
    assert bool(pairs) == (pair_steps and geno == "shipped")
    assert got.shape == want.shape
    err = float((got - want).abs().max())
    assert err <= 1e-5 * float(want.abs().max()), err
