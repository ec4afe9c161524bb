"""Pin the CPU oracle (oracle/torch_ref.py) against golden vectors produced by
running the reference itself (tools/gen_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import torch_ref as ref
from tests.golden_util import arch, golden, meta, normal, state_dict

CASES = meta()["cases"]


def _cases(prefix):
    return sorted(k.split("/", 1)[1] for k in CASES if k.startswith(prefix + "/"))


def test_weight_recipe_hash():
    sd = state_dict()
    assert len(sd) == meta()["n_tensors"] == 918


@pytest.mark.parametrize("name", _cases("cost_volume"))
def test_cost_volume_bit_exact(name):
    c = CASES["cost_volume/" + name]
    fl = normal(c["seeds"][0], c["shape"])
    fr = normal(c["seeds"][1], c["shape"])
    out = ref.build_cost_volume(fl, fr, c["maxdisp"]).numpy()
    np.testing.assert_array_equal(out, golden("cost_volume")[name])


@pytest.mark.parametrize("name", _cases("convbr"))
def test_convbr(name):
    c = CASES["convbr/" + name]
    x = normal(c["seed"], c["input"])
    out = ref.conv_br(x, state_dict(), c["module"], bn=c["bn"], relu=c["relu"]).numpy()
    np.testing.assert_allclose(out, golden("convbr")[name], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", _cases("resample"))
def test_resample(name):
    c = CASES["resample/" + name]
    out = ref.resample_ac(normal(c["seed"], c["input"]), c["size"]).numpy()
    np.testing.assert_allclose(out, golden("resample")[name], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", _cases("disp"))
def test_disp(name):
    c = CASES["disp/" + name]
    x = normal(c["seed"], c["input"]) * c["gain"]
    out = ref.disp_forward(x, c["maxdisp"]).numpy()
    np.testing.assert_allclose(out, golden("disp")[name], rtol=0, atol=1e-5)


def test_scale_dimension_and_levels():
    assert [ref.scale_dimension(n, 0.5) for n in (64, 65, 85)] == [32, 33, 43]
    assert [ref.scale_dimension(n, 2) for n in (32, 33)] == [64, 65]
    lv = ref.cell_levels(ref.network_layer_to_space(arch()["net_arch_mat"]))
    assert [l for l, _ in lv] == [1, 1, 2, 2, 1, 2, 2, 2, 1, 1, 0, 1]
    assert [d for _, d in lv] == [-1, 0, -1, 0, 1, -1, 0, 0, 1, 0, 1, -1]


@pytest.mark.parametrize("name", _cases("e2e"))
def test_e2e(name):
    c = CASES["e2e/" + name]
    shape = (c["batch"], 3, c["height"], c["width"])
    left, right = normal(c["seeds"][0], shape), normal(c["seeds"][1], shape)
    g = golden("e2e")
    with torch.no_grad():
        st = ref.leastereo_forward(state_dict(), left, right, c["maxdisp"], arch(), return_stages=True)
    if name + "/fea_l" in g:
        np.testing.assert_allclose(st["fea_l"].numpy(), g[name + "/fea_l"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(st["matching"].numpy(), g[name + "/matching"], rtol=1e-4, atol=1e-3)
    d32 = st["disp"]
    assert ref.epe(d32, torch.from_numpy(g[name + "/disp32"])) < 1e-4
    assert ref.epe(d32, torch.from_numpy(g[name + "/disp64"])) < 1e-4
