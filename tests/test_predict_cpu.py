"""predict.py plumbing (config 1): the restated host steps and the oracle on the
SceneFlow sample pair, against the fixture made by the reference model
(tools/gen_golden_c1.py)."""
import os

import numpy as np
import pytest
import torch

from leastereo_amd import predict as P
from oracle import predict_ref as PR
from oracle import torch_ref as ref
from tests.golden_util import arch, c1_inputs, golden, meta, state_dict

SF = "/root/reference/dataset/sceneflow_part/frames_finalpass/35mm_forward_fast"


def _write_pfm(path, img, little=True):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(b"Pf\n")
        f.write(f"{w} {h}\n".encode())
        f.write(b"-1.0\n" if little else b"1.0\n")
        f.write(np.flipud(img).astype("<f4" if little else ">f4").tobytes())


@pytest.mark.parametrize("little", [True, False])
def test_read_pfm_round_trip(tmp_path, little):
    img = np.arange(12, dtype=np.float32).reshape(3, 4) / 7
    p = tmp_path / "x.pfm"
    _write_pfm(p, img, little)
    got, h, w = P.read_pfm(str(p))
    assert (h, w) == (3, 4)
    np.testing.assert_array_equal(got, img)


def test_test_transform_pads_top_left_and_crop_output_undoes_it():
    data = np.random.default_rng(0).standard_normal((6, 5, 7)).astype(np.float32)
    left, right, h, w = PR.test_transform(data, 8, 12)
    assert left.shape == (1, 3, 8, 12) and (h, w) == (5, 7)
    assert torch.equal(left[0, :, 3:, 5:], torch.from_numpy(data[0:3]))
    assert torch.equal(right[0, :, 3:, 5:], torch.from_numpy(data[3:6]))
    assert float(left[0, :, :3].abs().sum()) == 0 and float(left[0, :, :, :5].abs().sum()) == 0
    pred = np.arange(96, dtype=np.float32).reshape(1, 8, 12)
    np.testing.assert_array_equal(P.crop_output(pred, h, w, 8, 12), pred[0, 3:, 5:])


def test_test_transform_centre_crop():
    data = np.random.default_rng(1).standard_normal((6, 540, 960)).astype(np.float32)
    left, right, h, w = PR.test_transform(data, 288, 576)
    assert (h, w) == (540, 960)
    np.testing.assert_array_equal(left[0].numpy(), data[0:3, 126:414, 192:768])
    np.testing.assert_array_equal(P.crop_output(np.ones((1, 288, 576)), h, w, 288, 576).shape, (288, 576))


def test_sceneflow_list_names():
    l, r, g = P.sceneflow_names("/d/", "TEST/A/0000/left/0006.png\n")
    assert l == "/d/frames_finalpass/TEST/A/0000/left/0006.png"
    assert r == "/d/frames_finalpass/TEST/A/0000/right/0006.png"
    assert g == "/d/disparity/TEST/A/0000/left/0006.pfm"


@pytest.mark.skipif(not os.path.isdir(SF), reason="reference sample images absent")
def test_load_data_matches_fixture_statistics():
    """Restated load_data on the reference's sample PNGs == the fixture's crop
    standardised with its stored whole-image statistics (container only)."""
    full = PR.load_data(f"{SF}/left/0001.png", f"{SF}/right/0001.png")
    left, right, _, _ = PR.test_transform(full, 288, 576)
    want_l, want_r = c1_inputs()
    assert torch.equal(left, want_l) and torch.equal(right, want_r)


def test_c1_oracle_matches_reference_disparity():
    """Config 1 (288x576 D96) through the oracle on CPU vs the reference's output."""
    left, right = c1_inputs()
    c = meta()["c1"]
    with torch.no_grad():
        d = ref.leastereo_forward(state_dict(), left, right, c["maxdisp"], arch())
    disp = P.crop_output(d.numpy(), *c["full_hw"], *c["crop_hw"])
    assert ref.epe(torch.from_numpy(disp), torch.from_numpy(golden("c1_sceneflow")["disp"])) < 1e-3


def test_float_png_conversion_is_imageios():
    """skimage.io.imsave of a float image (predict.py:207,211) through imageio's 8-bit
    conversion (restated; parity unpinned -- neither library is importable here)."""
    a = np.array([[0.0, 0.5], [1.0, 0.25]], np.float32)          # already in [0, 1]
    np.testing.assert_array_equal(P.float_to_u8(a), [[0, 127], [255, 64]])
    d = np.array([[10.0, 20.0], [30.0, 50.0]], np.float32)      # min-max normalised
    np.testing.assert_array_equal(P.float_to_u8(d), [[0, 64], [127, 255]])
    assert P.float_to_u8(np.full((2, 2), 7.0)).tolist() == [[7, 7], [7, 7]]


def test_crop_image_pads_bottom_right_or_centre_crops():
    img = (np.arange(5 * 7 * 3) % 251).astype(np.uint8).reshape(5, 7, 3)
    pad = P.crop_image(img, 8, 12)
    assert pad.shape == (8, 12, 3) and pad.dtype == np.float32
    np.testing.assert_array_equal(pad[3:, 5:], img)
    assert pad[:3].sum() == 0 and pad[:, :5].sum() == 0
    crop = P.crop_image(img, 3, 4)
    assert crop.dtype == np.uint8
    np.testing.assert_array_equal(crop, img[1:4, 1:5])


def test_satellite_and_plot_outputs(tmp_path):
    l, r, s, i = P.satellite_names("/d/", "/o/", "tile_07\n")
    assert (l, r, s, i) == ("/d/tile_07/satiml.png", "/d/tile_07/satimr.png", "/o/tile_07.png",
                            "/o/tile_07_in.png")
    from PIL import Image
    disp = np.linspace(0, 200, 12 * 16, dtype=np.float32).reshape(12, 16)
    P.plot_disparity(str(tmp_path / "d.png"), disp, 192)
    png = np.asarray(Image.open(tmp_path / "d.png"))
    assert png.shape[:2] == (12, 16)
    import matplotlib
    want = (matplotlib.colormaps["turbo"](np.clip(disp / 192, 0, 1)) * 255).round().astype(np.uint8)
    assert np.abs(png[..., :3].astype(int) - want[..., :3]).max() <= 1
    P.save_float_png(str(tmp_path / "f.png"), disp)
    got = np.asarray(Image.open(tmp_path / "f.png"))
    np.testing.assert_array_equal(got, P.float_to_u8(disp))
