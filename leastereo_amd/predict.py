"""predict.py of the reference, on the MI355X model (config 1 plumbing).

Restates the host-side steps around ``LEAStereo.forward`` (predict.py:144-243):
  * ``load_images``    predict.py:163-169  PIL decode (uint8, stays uint8)
  * ``load_transform`` predict.py:144-184  load_data's per-channel standardisation
                       (whole-image float64 statistics, stored float32) fused with
                       test_transform's pad/centre-crop, on the device
                       (``lea_standardize_crop_u8``; numpy checker: oracle/predict_ref.py)
  * ``crop_output``    predict.py:236-239  undo the padding on the disparity
  * ``read_pfm``       dataloaders/datasets/common.py:8-40
  * ``plot_disparity`` predict.py:246-247  turbo-coloured PNG, vmin 0, vmax 192
  * ``save_float_png`` / ``crop_image``  predict.py:128-141,207-211  the satellite
                       branch's skimage.io.imsave of float arrays (imageio's min-max
                       8-bit conversion, restated: skimage / imageio are absent here)
  * ``main``           predict.py:249-286  the list-file loop: --sceneflow writes
                       {index}.png and {index}_gt.png (and {index}.npy, the raw
                       disparity), --satellite writes {name}.png and {name}_in.png
Arithmetic runs on the HIP kernels; what stays on the host is file I/O (PIL, PFM, PNG).

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


def load_images(leftname, rightname):
    """The PIL decode of predict.py:163-169: two uint8 [H, W, 3|4] arrays."""
    from PIL import Image
    left = np.asarray(Image.open(leftname))
    right = np.asarray(Image.open(rightname))
    if left.shape != right.shape or left.ndim != 3 or left.dtype != np.uint8:
        raise ValueError(f"{leftname}, {rightname}: need two 8-bit colour images of one size, "
                         f"got {left.shape} {left.dtype} and {right.shape} {right.dtype}")
    return left, right


def load_transform(left_u8, right_u8, crop_height, crop_width, device="cuda"):
    """load_data (predict.py:162-184) + test_transform (:144-159) on the device:
    the uint8 images go up as they were decoded (a quarter of the float32 bytes)
    and ``lea_standardize_crop_u8`` standardises with whole-image statistics and
    pads or crops in one pass.  Returns (left, right [1, 3, ch, cw], h, w)."""
    from . import kernels
    h, w = left_u8.shape[:2]
    lt = torch.from_numpy(np.ascontiguousarray(left_u8)).to(device, non_blocking=True)
    rt = torch.from_numpy(np.ascontiguousarray(right_u8)).to(device, non_blocking=True)
    left, right = kernels.standardize_crop_u8(lt, rt, crop_height, crop_width)
    return left, right, h, w


def crop_output(pred: np.ndarray, height: int, width: int, crop_height: int, crop_width: int):
    """predict.py:236-239 (the reference's ``or``: a crop on either axis triggers it)."""
    if height <= crop_height or width <= crop_width:
        return pred[0, crop_height - height: crop_height, crop_width - width: crop_width]
    return pred[0]


def predict_pair(model, leftname, rightname, crop_height, crop_width, device="cuda"):
    """test() of predict.py:213-243 without the plotting: disparity [h', w'] numpy."""
    left, right, h, w = load_transform(*load_images(leftname, rightname), crop_height, crop_width,
                                       device)
    with torch.no_grad():
        pred = model(left, right)
    return crop_output(pred.cpu().numpy(), h, w, crop_height, crop_width)


def plot_disparity(savename, data, max_disp=192):
    """predict.py:246-247: ``plt.imsave(savename, data, vmin=0, vmax=max_disp, cmap='turbo')``."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.imsave(savename, data, vmin=0, vmax=max_disp, cmap="turbo")


def float_to_u8(img: np.ndarray) -> np.ndarray:
    """What skimage.io.imsave (predict.py:207,211) writes for a float array: its imageio
    plugin's ``image_as_uint(im, bitdepth=8)`` -- values already in [0, 1] scale by 255,
    anything else is min-max normalised first -- ``* 255 + 0.499999999`` then truncated
    (imageio 2.x, a third-party dependency absent here; restated from its source)."""
    im = np.asarray(img, dtype=np.float64)
    mi, ma = float(np.nanmin(im)), float(np.nanmax(im))
    if not (mi >= 0 and ma <= 1):
        if not (np.isfinite(mi) and np.isfinite(ma)):
            raise ValueError("image values are not finite")
        if ma == mi:  # imageio returns the values cast as they are
            return im.astype(np.uint8)
        im = (im - mi) / (ma - mi)
    return (im * 255.0 + 0.499999999).astype(np.uint8)


def save_float_png(savename, img):
    """skimage.io.imsave(savename, img) of predict.py:207,211 (PNG)."""
    from PIL import Image
    a = np.asarray(img)
    if a.dtype != np.uint8:
        a = float_to_u8(a)
    Image.fromarray(a).save(savename)


def crop_image(image, crop_height, crop_width):
    """predict.py:128-141: zero-pad the HWC image into the bottom-right of the crop
    (float32 result) when it fits, else centre-crop (its own dtype)."""
    data = np.moveaxis(np.asarray(image), [2], [0])
    n_layers, h, w = data.shape
    if h <= crop_height and w <= crop_width:
        result = np.zeros([n_layers, crop_height, crop_width], "float32")
        result[:, crop_height - h: crop_height, crop_width - w: crop_width] = data
    else:
        start_x = (w - crop_width) // 2
        start_y = (h - crop_height) // 2
        result = data[:, start_y: start_y + crop_height, start_x: start_x + crop_width]
    return np.moveaxis(result, [0], [2])


def satellite_names(data_path, save_path, line):
    """predict.py:258-263: the list line minus its last character names a directory
    holding satiml.png / satimr.png; outputs <save_path><name>.png and <name>_in.png."""
    cur = line[:-1]
    return (data_path + cur + "/satiml.png", data_path + cur + "/satimr.png",
            save_path + cur + ".png", save_path + cur + "_in.png")


def test_satellite(model, leftname, rightname, savename, in_savename, crop_height, crop_width):
    """predict.py:187-211: the disparity as a PNG (min-max 8-bit, as skimage writes a
    float image) and the left input cropped / padded to the crop."""
    from PIL import Image
    disp = predict_pair(model, leftname, rightname, crop_height, crop_width)
    save_float_png(savename, disp)
    save_float_png(in_savename, crop_image(Image.open(leftname), crop_height, crop_width))
    return disp


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
    from . import metrics
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
    if not (opt.sceneflow or opt.satellite):
        raise NotImplementedError("predict.py has list layouts for --sceneflow and --satellite only "
                                  "(the reference's other dataset flags write nothing)")
    for index, line in enumerate(lines):
        if opt.satellite:  # predict.py:258-264
            test_satellite(model, *satellite_names(opt.data_path, opt.save_path, line),
                           opt.crop_height, opt.crop_width)
        if not opt.sceneflow:
            continue
        print(f"Running for sceneflow {index}")
        leftname, rightname, gtname = sceneflow_names(opt.data_path, line)
        gt = None
        if os.path.isfile(gtname):  # predict.py:275-277 (the reference requires it)
            gt, _, _ = read_pfm(gtname)
            plot_disparity(opt.save_path + f"{index:d}_gt.png", gt, 192)
        t0 = time.time()
        disp = predict_pair(model, leftname, rightname, opt.crop_height, opt.crop_width)
        print(f"Processing time: {time.time() - t0:.4f}")
        plot_disparity(opt.save_path + f"{index:d}.png", disp, 192)  # predict.py:240
        np.save(os.path.join(opt.save_path, f"{index}.npy"), disp.astype(np.float32))
        if gt is not None:
            ch, cw = disp.shape
            h, w = gt.shape
            y0, x0 = max(int((h - ch) / 2), 0), max(int((w - cw) / 2), 0)
            gt = np.ascontiguousarray(gt[y0:y0 + ch, x0:x0 + cw], dtype=np.float32)
            m = metrics.evaluate(disp, gt, opt.maxdisp)[0]  # evaluation.py:287-307, device
            print(f"{index}: EPE vs GT {m['epe']:.4f} px, 3px error {m['three_px_error']:.3f}, "
                  f"bad 1.0 {m['bad_1']:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
