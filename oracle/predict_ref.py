"""ORACLE (test infrastructure only; imported by tests/, tools/gen_golden*.py and
bench.py's cpu_baseline leg, never by the product): numpy restatement of the
reference's predict.py host preprocessing, the checker for
``lea_standardize_crop_u8`` (leastereo_amd/csrc/evalio.hip).

  * ``standardize``    predict.py:171-183 (per-channel (x - mean) / std, float64,
                       stored float32)
  * ``load_data``      predict.py:162-184 (PIL decode + standardize)
  * ``test_transform`` predict.py:144-159

Pinning: predict.py cannot be imported (argv parse at import time),
so these are the same numpy expressions line for line; the config-1 fixture
(tests/golden/c1_sceneflow.npz, tools/gen_golden_c1.py) carries their output on
the reference's own SceneFlow sample pair, fed to the imported reference model.
"""
from __future__ import annotations

import numpy as np
import torch


def standardize(rgb_left: np.ndarray, rgb_right: np.ndarray) -> np.ndarray:
    """predict.py:171-183 -> [6, H, W] float32."""
    h, w = rgb_left.shape[:2]
    out = np.zeros([6, h, w], "float32")
    for i, img in enumerate((rgb_left, rgb_right)):
        for c in range(3):
            x = img[:, :, c]
            out[3 * i + c] = (x - np.mean(x[:])) / np.std(x[:])
    return out


def load_data(leftname, rightname) -> np.ndarray:
    """predict.py:162-184."""
    from PIL import Image
    return standardize(np.asarray(Image.open(leftname)), np.asarray(Image.open(rightname)))


def test_transform(temp_data: np.ndarray, crop_height: int, crop_width: int):
    """predict.py:144-159 -> (left [1,3,ch,cw], right [1,3,ch,cw], h, w)."""
    _, h, w = np.shape(temp_data)
    if h <= crop_height and w <= crop_width:
        temp = temp_data
        temp_data = np.zeros([6, crop_height, crop_width], "float32")
        temp_data[:, crop_height - h: crop_height, crop_width - w: crop_width] = temp
    else:
        start_x = int((w - crop_width) / 2)
        start_y = int((h - crop_height) / 2)
        temp_data = temp_data[:, start_y: start_y + crop_height, start_x: start_x + crop_width]
    left = np.ones([1, 3, crop_height, crop_width], "float32")
    left[0] = temp_data[0:3]
    right = np.ones([1, 3, crop_height, crop_width], "float32")
    right[0] = temp_data[3:6]
    return torch.from_numpy(left), torch.from_numpy(right), h, w
