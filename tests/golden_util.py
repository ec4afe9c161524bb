"""Shared fixture helpers: load golden vectors and regenerate their inputs/weights."""
import functools
import json
import os

import numpy as np
import torch

from leastereo_amd.weights import seeded_normal, state_dict_sha256, synthetic_state_dict

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ARCH_DIR = os.path.join(os.path.dirname(GOLD), "..", "leastereo_amd", "data", "architecture")


@functools.lru_cache(None)
def meta():
    with open(os.path.join(GOLD, "meta.json")) as f:
        return json.load(f)


@functools.lru_cache(None)
def golden(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))


def shapes():
    return {k: tuple(v) for k, v in meta()["state_dict_shapes"]}


@functools.lru_cache(None)
def state_dict():
    sd = synthetic_state_dict(shapes())
    assert state_dict_sha256(sd) == meta()["state_dict_sha256"], "weight recipe drifted"
    return sd


def arch():
    d = os.path.abspath(ARCH_DIR)
    return {"net_arch_fea": np.load(os.path.join(d, "feature_network_path.npy")),
            "cell_arch_fea": np.load(os.path.join(d, "feature_genotype.npy")),
            "net_arch_mat": np.load(os.path.join(d, "matching_network_path.npy")),
            "cell_arch_mat": np.load(os.path.join(d, "matching_genotype.npy"))}


def normal(seed, shape):
    return torch.from_numpy(seeded_normal(seed, shape))


def c1_inputs():
    """Config-1 fixture -> (left, right) [1, 3, 288, 576] float32 exactly as
    predict.py's load_data + test_transform make them (whole-image statistics)."""
    g = golden("c1_sceneflow")
    planes = []
    for i, img in enumerate((g["left_u8"], g["right_u8"])):
        for c in range(3):
            planes.append(((img[:, :, c] - g["mean"][3 * i + c]) / g["std"][3 * i + c]).astype(np.float32))
    x = np.stack(planes)
    return torch.from_numpy(x[None, 0:3].copy()), torch.from_numpy(x[None, 3:6].copy())
