"""Host-side checks of the drop-in module (CPU, no kernel launches)."""
import numpy as np
import pytest
import torch

from leastereo_amd import arch as A
from leastereo_amd.config import LEAStereoArgs, default_arch_args
from leastereo_amd.model import LEAStereo
from oracle import torch_ref as ref
from tests.golden_util import arch, golden, meta, normal, shapes, state_dict


def _model(maxdisp=48):
    args = default_arch_args(LEAStereoArgs(maxdisp=maxdisp))
    return LEAStereo(args, "cpu")


def test_state_dict_key_set_and_shapes_match_reference():
    m = _model()
    mine = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert mine == shapes()
    assert list(mine) == list(shapes()), "registration order differs from the reference"
    m.load_state_dict(state_dict(), strict=True)


def test_cell_specs_match_survey_table():
    specs = _model().matching.specs
    assert [(s.level, s.c_out, s.c_prev, s.c_prev_prev, s.downup) for s in specs] == [
        (1, 16, 32, 32, -1), (1, 16, 64, 32, 0), (2, 32, 64, 64, -1), (2, 32, 128, 64, 0),
        (1, 16, 128, 128, 1), (2, 32, 64, 128, -1), (2, 32, 128, 64, 0), (2, 32, 128, 128, 0),
        (1, 16, 128, 128, 1), (1, 16, 64, 128, 0), (0, 8, 64, 64, 1), (1, 16, 32, 64, -1)]


def test_ops_iteration_order():
    plan = A.ops_in_iteration_order(arch()["cell_arch_mat"], 3)
    assert plan == [[(0, 0), (1, 1)], [(2, 1), (3, 2)], [(4, 1), (5, 3)]]
    plan = A.ops_in_iteration_order(arch()["cell_arch_fea"], 3)
    assert plan == [[(0, 0), (1, 1)], [(2, 1), (3, 2)], [(4, 0), (5, 3)]]


def test_network_layer_to_space_matches_oracle():
    for key in ("net_arch_fea", "net_arch_mat"):
        np.testing.assert_array_equal(A.network_layer_to_space(arch()[key]),
                                      ref.network_layer_to_space(arch()[key]))


@pytest.mark.parametrize("maxdisp,ok", [(192, True), (264, True), (408, True), (96, True),
                                        (256, False), (252, False), (258, False)])
def test_shape_legality(maxdisp, ok):
    m = _model(maxdisp)
    if ok:
        m.check_shape(576, 960)
    else:
        with pytest.raises(ValueError):
            m.check_shape(576, 960)


def test_shape_legality_spatial():
    m = _model(192)
    for h, w in ((576, 960), (384, 1248), (1008, 1512), (288, 576)):
        m.check_shape(h, w)
    with pytest.raises(ValueError):
        m.check_shape(540, 960)


def test_feature_net_refuses_cpu():
    """No torch fallback: the feature net runs on the HIP kernels only."""
    m = _model(48)
    with pytest.raises(RuntimeError):
        m.feature(torch.zeros(1, 3, 96, 192))


def test_forward_refuses_cpu():
    m = _model(48)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 96, 192), torch.zeros(1, 3, 96, 192))
