"""predict.py of the reference, on the MI355X model (config 1 plumbing).

Restates the host-side steps around ``LEAStereo.forward`` (predict.py:144-243):
  * ``load_data``      predict.py:162-184  per-channel standardisation of both PNGs
                       (population std, float64 arithmetic, stored float32)
  * ``test_transform`` predict.py:144-159  zero-pad top-left up to the crop, else
                       centre-crop; split into left/right [1, 3, H, W]
  * ``crop_output``    predict.py:236-239  undo the padding on the disparity
  * ``read_pfm``       dataloaders/datasets/common.py:8-40
  * ``main``           predict.py:249-286  the list-file loop (SceneFlow naming)
The model runs on the HIP kernels; everything here is numpy/PIL file plumbing.

    python predict.py --sceneflow=1 --maxdisp=192 --crop_height=576 --crop_width=960 \
        --data_path=./dataset/SceneFlow/ --test_list=./lists/sceneflow_test.list \
        --save_path=./predict/ [--resume ckpt.pth] [arch flags as the reference]
"""
from __future__ import annotations

import os
import re
import sys
import time

import numpy as np
import torch


def read_pfm(path):
    """dataloaders/datasets/common.py:8-40: (image [H, W] float, height, width)."""
    with open(path, "rb") as f:
        kind = f.readline().decode("latin-1")
        if "PF" in kind:
            channels = 3
        elif "Pf" in kind:
            channels = 1
        else:
            raise ValueError(f"{path}: not a PFM file")
        width, height = (int(v) for v in re.findall(r"\d+", f.readline().decode("latin-1")))
        little = "-" in f.readline().decode("latin-1")
        data = np.frombuffer(f.read(width * height * channels * 4),
                             dtype="<f4" if little else ">f4").astype(np.float64)
    if channels != 1:
        raise ValueError(f"{path}: {channels}-channel PFM (the reference reshapes to [H, W])")
    return np.flipud(data.reshape(height, width)), height, width


def standardize(rgb_left: np.ndarray, rgb_right: np.ndarray) -> np.ndarray:
    """predict.py:171-183: channel c of each image -> (x - mean) / std in float64,
    stored float32 into a [6, H, W] array."""
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
    left = np.asarray(Image.open(leftname))
    right = np.asarray(Image.open(rightname))
    return standardize(left, right)


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


def crop_output(pred: np.ndarray, height: int, width: int, crop_height: int, crop_width: int):
    """predict.py:236-239 (the reference's ``or``: a crop on either axis triggers it)."""
    if height <= crop_height or width <= crop_width:
        return pred[0, crop_height - height: crop_height, crop_width - width: crop_width]
    return pred[0]


def predict_pair(model, leftname, rightname, crop_height, crop_width, device="cuda"):
    """test() of predict.py:213-243 without the plotting: disparity [h', w'] numpy."""
    left, right, h, w = test_transform(load_data(leftname, rightname), crop_height, crop_width)
    with torch.no_grad():
        pred = model(left.to(device), right.to(device))
    return crop_output(pred.cpu().numpy(), h, w, crop_height, crop_width)


def load_checkpoint(model, path):
    """predict.py:52-67: checkpoint['state_dict'] with an optional 'module.' prefix,
    loaded with a loader that executes nothing from the file."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = {(k.split(".", 1)[1] if k.startswith("module") else k): v
          for k, v in ckpt["state_dict"].items()}
    model.load_state_dict(sd, strict=True)


def sceneflow_names(data_path, line):
    """predict.py:267-273: left, right and GT names of one sceneflow list line."""
    cur = line.rstrip("\n")
    leftname = data_path + "frames_finalpass/" + cur
    rightname = data_path + "frames_finalpass/" + cur[: len(cur) - 13] + "right/" + cur[len(cur) - 8:]
    gtname = data_path + "disparity/" + cur[: len(cur) - 3] + "pfm"
    return leftname, rightname, gtname


def main(argv=None):
    from .config import default_arch_args, obtain_predict_args
    from .model import LEAStereo
    opt = default_arch_args(obtain_predict_args(argv))
    if not torch.cuda.is_available():
        raise RuntimeError("leastereo_amd runs on a ROCm device only")
    model = LEAStereo(opt, "cuda")
    if opt.resume:
        if not os.path.isfile(opt.resume):
            raise FileNotFoundError(opt.resume)
        load_checkpoint(model, opt.resume)
    model = model.cuda().eval()
    os.makedirs(opt.save_path, exist_ok=True)
    with open(opt.test_list) as f:
        lines = f.readlines()
    for index, line in enumerate(lines):
        if not opt.sceneflow:
            raise NotImplementedError("only the --sceneflow list layout is restated")
        leftname, rightname, gtname = sceneflow_names(opt.data_path, line)
        t0 = time.time()
        disp = predict_pair(model, leftname, rightname, opt.crop_height, opt.crop_width)
        print(f"Processing time: {time.time() - t0:.4f}")
        np.save(os.path.join(opt.save_path, f"{index}.npy"), disp.astype(np.float32))
        if os.path.isfile(gtname):
            gt, _, _ = read_pfm(gtname)
            ch, cw = disp.shape
            h, w = gt.shape
            y0, x0 = max(int((h - ch) / 2), 0), max(int((w - cw) / 2), 0)
            gt = gt[y0:y0 + ch, x0:x0 + cw]
            print(f"{index}: EPE vs GT {np.mean(np.abs(disp - gt)):.4f} px")
    return 0


if __name__ == "__main__":
    sys.exit(main())
