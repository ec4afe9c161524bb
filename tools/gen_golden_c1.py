#!/usr/bin/env python3
"""Config-1 plumbing fixture (BASELINE configs[0]).

SceneFlow sample pair 0001 shipped in the reference (dataset/sceneflow_part),
preprocessed by the restated predict.py steps (oracle/predict_ref.py), centre-
cropped to 288x576, run through the *reference* LEAStereo (imported from
/root/reference, CPU, maxdisp 96, the synthetic weight recipe).  Container only.

Stored (tests/golden/c1_sceneflow.npz; the full images are not needed later):
  left_u8 / right_u8   the 288x576 RGB crops of the two PNGs
  mean / std           float64 per-channel statistics of the FULL images (load_data
                       standardises with whole-image statistics before the crop)
  gt                   the GT disparity crop (reference read_pfm of disparity/.../0001.pfm)
  disp                 reference fp32 disparity [288, 576]
and a "c1" entry in tests/golden/meta.json.  The reference's own read_pfm is used
to cross-check the restated one.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_c1.py
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from leastereo_amd import predict as P  # noqa: E402
from oracle import predict_ref as PR  # noqa: E402
from leastereo_amd.weights import synthetic_state_dict  # noqa: E402
from tools.gen_golden import GOLD, ref_model  # noqa: E402

SF = os.path.join(REF, "dataset", "sceneflow_part")
PAIR = "35mm_forward_fast/left/0001.png"
CROP = (288, 576)
MAXDISP = 96


def main():
    from PIL import Image
    left_name = os.path.join(SF, "frames_finalpass", PAIR)
    right_name = left_name.replace("/left/", "/right/")
    gt_name = os.path.join(SF, "disparity", PAIR[:-3] + "pfm")
    left = np.asarray(Image.open(left_name))
    right = np.asarray(Image.open(right_name))
    h, w = left.shape[:2]
    full = PR.load_data(left_name, right_name)
    li, ri, h2, w2 = PR.test_transform(full, *CROP)
    assert (h2, w2) == (h, w)
    y0, x0 = int((h - CROP[0]) / 2), int((w - CROP[1]) / 2)

    sys.path.insert(0, REF)
    from dataloaders.datasets.common import read_pfm as ref_read_pfm  # common.py:8
    gt_ref, _, _ = ref_read_pfm(gt_name)
    gt, _, _ = P.read_pfm(gt_name)
    assert np.array_equal(gt, gt_ref), "restated read_pfm differs from the reference's"

    m = ref_model(MAXDISP)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(synthetic_state_dict(shapes), strict=True)
    m.eval()
    with torch.no_grad():
        pred = m(li, ri).numpy()
    disp = P.crop_output(pred, h, w, *CROP).astype(np.float32)
    gt_crop = gt[y0:y0 + CROP[0], x0:x0 + CROP[1]].astype(np.float32)
    stats = []
    for img in (left, right):
        for c in range(3):
            x = img[:, :, c]
            stats.append((np.mean(x[:]), np.std(x[:])))
    np.savez_compressed(
        os.path.join(GOLD, "c1_sceneflow.npz"),
        left_u8=left[y0:y0 + CROP[0], x0:x0 + CROP[1]], right_u8=right[y0:y0 + CROP[0], x0:x0 + CROP[1]],
        mean=np.array([s[0] for s in stats], np.float64), std=np.array([s[1] for s in stats], np.float64),
        gt=gt_crop, disp=disp)
    meta_path = os.path.join(GOLD, "meta.json")
    meta = json.load(open(meta_path))
    meta["c1"] = {"pair": "dataset/sceneflow_part/frames_finalpass/" + PAIR, "full_hw": [h, w],
                  "crop_hw": list(CROP), "crop_origin": [y0, x0], "maxdisp": MAXDISP,
                  "epe_vs_gt_px": float(np.mean(np.abs(disp - gt_crop))),
                  "note": "synthetic weights: the GT EPE is plumbing, not accuracy"}
    json.dump(meta, open(meta_path, "w"), indent=1, sort_keys=True)
    print("c1 fixture written; EPE vs GT", meta["c1"]["epe_vs_gt_px"])


if __name__ == "__main__":
    main()
