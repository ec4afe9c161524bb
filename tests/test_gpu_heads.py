"""Every head branch of both searched networks, f32 and bf16, against the float64
oracle.

The shipped SceneFlow architecture ends the feature net at level 0 (the head is
last_3 alone) and the matching net at level 1 (last_6 then the up-sampled last_3),
so the other branches of new_model_2d.py:156-163 and skip_model_3d.py:166-173 --
last levels 1/2/3 (feature) and 0/2/3 (matching) -- only run for other level paths.
These tests build such paths (the matching net's skip fusions need cells 1, 4 and 8
at level 1, skip_model_3d.py:150,155) and compare each subnet's output with
oracle/torch_ref.py in float64 on the same inputs and weights.

Weights: the synthetic recipe without the calibrated BN file (its tensors have the
shipped architecture's shapes): kaiming convs, random BN affine, identity running
statistics.  Bars: f32 max |d| <= 1e-4 * max |ref| + 1e-6 (the per-conv bar of the
engines, compounded over the net, measured well inside it); bf16 mean |d| <= 2e-2
* mean |ref| (bf16 storage between ~40 layers, f32 accumulation).
"""
import numpy as np
import pytest
import torch

from leastereo_amd import kernels
from leastereo_amd.config import LEAStereoArgs, default_arch_args
from leastereo_amd.model import LEAStereo
from leastereo_amd.weights import synthetic_state_dict
from oracle import torch_ref as ref
from tests.golden_util import arch, normal

pytestmark = pytest.mark.gpu
DEV = "cuda"

FEATURE_PATHS = {1: [1, 1, 0, 1, 1, 1], 2: [1, 2, 2, 1, 2, 2], 3: [1, 2, 3, 3, 2, 3]}
MATCHING_PATHS = {0: [1, 1, 2, 2, 1, 2, 2, 2, 1, 0, 0, 0], 2: [0, 1, 2, 2, 1, 1, 2, 2, 1, 2, 2, 2],
                  3: [1, 1, 2, 2, 1, 2, 3, 2, 1, 2, 3, 3]}


def _model(tmp_path, maxdisp, precision, fea=None, mat=None):
    args = LEAStereoArgs(maxdisp=maxdisp)
    if fea is not None:
        args.net_arch_fea = str(tmp_path / "fea.npy")
        np.save(args.net_arch_fea, np.array(fea))
    if mat is not None:
        args.net_arch_mat = str(tmp_path / "mat.npy")
        np.save(args.net_arch_mat, np.array(mat))
    args = default_arch_args(args)
    m = LEAStereo(args, DEV, precision=precision)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = synthetic_state_dict(shapes, bn_file=None)
    m.load_state_dict(sd, strict=True)
    a = arch()
    if fea is not None:
        a["net_arch_fea"] = np.array(fea)
    if mat is not None:
        a["net_arch_mat"] = np.array(mat)
    return m.to(DEV).eval(), sd, a


def _check(got, want, precision):
    got, want = got.double().cpu(), want.double().cpu()
    assert got.shape == want.shape and torch.isfinite(got).all()
    if precision == "f32":
        err, scale = float((got - want).abs().max()), float(want.abs().max())
        assert err <= 1e-4 * scale + 1e-6, (err, scale)
    else:
        err, scale = float((got - want).abs().mean()), float(want.abs().mean())
        assert err <= 2e-2 * scale, (err, scale)


@pytest.mark.parametrize("precision", ["f32", "bf16"])
@pytest.mark.parametrize("level", sorted(FEATURE_PATHS))
def test_feature_head_branch(tmp_path, level, precision):
    path = FEATURE_PATHS[level]
    assert path[-1] == level
    m, sd, a = _model(tmp_path, 48, precision, fea=path)
    x = normal(611 + level, (2, 3, 96, 192))
    with torch.no_grad():
        got = m.feature(x.to(DEV))
        if precision == "bf16":
            got = kernels.from_c8(got)[:, :, 0]
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        want = ref.feature_forward(sd64, x.double(), a["net_arch_fea"], a["cell_arch_fea"])
    _check(got, want, precision)


@pytest.mark.parametrize("precision", ["f32", "bf16"])
@pytest.mark.parametrize("level", sorted(MATCHING_PATHS))
def test_matching_head_branch(tmp_path, level, precision):
    path = MATCHING_PATHS[level]
    assert path[-1] == level and path[1] == path[4] == path[8] == 1
    m, sd, a = _model(tmp_path, 48, precision, mat=path)
    m.check_shape(96, 192)
    g = torch.Generator().manual_seed(700 + level)
    fl = torch.randn(1, 32, 32, 64, generator=g)
    fr = torch.randn(1, 32, 32, 64, generator=g)
    with torch.no_grad():
        got = m.matching.executor().run_features(fl.to(DEV), fr.to(DEV), 48)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        cost = ref.build_cost_volume(fl.double(), fr.double(), 48)
        want = ref.matching_forward(sd64, cost, a["net_arch_mat"], a["cell_arch_mat"])
    _check(got, want, precision)
