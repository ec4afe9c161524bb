"""Host-side checks of the ConvBR3d training drop-in (leastereo_amd/training.py); the
numerics are in tests/test_gpu_training.py."""
import pytest
import torch

from leastereo_amd import _lib
from leastereo_amd.training import ConvBR3d


def test_state_dict_keys_match_reference_convbr():
    """models/operations_3d.py:31-39: conv (bias-free Conv3d) + bn (BatchNorm3d)."""
    m = ConvBR3d(16, 32, 3, 1, 1)
    assert list(m.state_dict()) == ["conv.weight", "bn.weight", "bn.bias", "bn.running_mean",
                                    "bn.running_var", "bn.num_batches_tracked"]
    assert tuple(m.conv.weight.shape) == (32, 16, 3, 3, 3)
    assert m.bn.eps == 1e-5 and m.bn.momentum == 0.1
    assert torch.all(m.bn.weight == 1) and torch.all(m.bn.bias == 0)


@pytest.mark.parametrize("k,stride,pad", [(3, 2, 1), (3, 1, 0), (5, 1, 2)])
def test_unsupported_shapes_raise(k, stride, pad):
    with pytest.raises(NotImplementedError):
        ConvBR3d(4, 4, k, stride, pad)


def test_cpu_tensor_raises_no_fallback():
    m = ConvBR3d(4, 4, 3, 1, 1)
    with pytest.raises(_lib.HipKernelError):
        m(torch.randn(1, 4, 2, 3, 4))


def test_train_step_golden_matches_model_shapes():
    """tests/golden/train_step.npz (the reference's own float64 train step) names
    parameters of this model with its shapes, and carries a noise figure per quantity."""
    from leastereo_amd.config import LEAStereoArgs, default_arch_args
    from leastereo_amd.model import LEAStereo
    from tests.golden_util import golden
    g = golden("train_step")
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=48)), "cpu")
    params = dict(m.named_parameters())
    n = 0
    for k, v in g.items():
        if k.startswith("grad/"):
            name = k[5:]
            shape = tuple(params[name].shape)
            if name.endswith(("conv1.conv.weight", "conv2.conv.weight")):
                shape = (8,) + shape[1:]
            assert tuple(v.shape) == shape, k
            assert "noise/" + k in g
            n += 1
    assert n == 15 and g["disp"].shape == (1, 96, 192) and 0 < float(g["noise/disp"]) < 0.05
