"""Deterministic synthetic weights (the trained checkpoints are absent upstream).

Recipe: every ``*.conv.weight`` is drawn from numpy's portable
PCG64 stream seeded by (seed, crc32(key)) and scaled by the kaiming fan-out std
the reference initialiser uses (models/operations_3d.py:49-55,
nn.init.kaiming_normal_(mode='fan_out', nonlinearity='relu')).  BatchNorm
affine parameters and running statistics come from ``data/synthetic_bn.npz``,
which ``tools/gen_golden.py`` calibrated by one train-mode pass of the
*reference* model (momentum 1.0) and then conditioned
(``running_var >= 2``, ``matching.last_3.conv.weight *= 2``) so that fp32
disparities are well conditioned (fp32-vs-fp64 EPE recorded in the fixtures).

The key set is the reference state_dict's key set, so the result loads with
``load_state_dict(strict=True)`` into both the reference and this package.
"""
from __future__ import annotations

import hashlib
import os
import zlib

import numpy as np
import torch

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
BN_FILE = os.path.join(DATA_DIR, "synthetic_bn.npz")
DEFAULT_SEED = 20201101
LAST3_GAIN = 2.0


def seeded_normal(seed: int, shape) -> np.ndarray:
    """Portable N(0,1) float32 array (fixture inputs are regenerated from seeds)."""
    return np.random.default_rng(seed).standard_normal(tuple(shape), dtype=np.float32)


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng([seed, zlib.crc32(key.encode())])


def conv_weight(key: str, shape, seed: int = DEFAULT_SEED) -> np.ndarray:
    fan_out = shape[0] * int(np.prod(shape[2:]))
    std = np.sqrt(2.0 / fan_out)
    return (_rng(seed, key).standard_normal(shape) * std).astype(np.float32)


def bn_affine(key: str, c: int, seed: int = DEFAULT_SEED):
    """Pre-calibration BN affine (gamma, beta): mildly random so the folded
    epilogue scale/shift is exercised (defaults would be 1/0)."""
    r = _rng(seed, key + "#affine")
    gamma = r.uniform(0.75, 1.25, c).astype(np.float32)
    beta = (0.1 * r.standard_normal(c)).astype(np.float32)
    return gamma, beta


def synthetic_state_dict(shapes, seed: int = DEFAULT_SEED, bn_file: str | None = BN_FILE):
    """shapes: ordered mapping key -> tuple(shape) of the reference state_dict."""
    bn = None
    if bn_file is not None:
        if not os.path.exists(bn_file):
            raise FileNotFoundError(f"{bn_file} missing: run tools/gen_golden.py")
        bn = np.load(bn_file, allow_pickle=False)
    sd = {}
    for key, shape in shapes.items():
        shape = tuple(shape)
        if key.endswith("conv.weight"):
            w = conv_weight(key, shape, seed)
            if key == "matching.last_3.conv.weight" and bn is not None:
                w = w * np.float32(LAST3_GAIN)
            sd[key] = torch.from_numpy(w)
        elif bn is not None and key in bn.files:
            arr = bn[key]
            sd[key] = torch.from_numpy(np.array(arr))
        elif key.endswith("num_batches_tracked"):
            sd[key] = torch.tensor(0, dtype=torch.long)
        elif key.endswith("bn.weight"):
            sd[key] = torch.from_numpy(bn_affine(key[:-len(".weight")], shape[0], seed)[0])
        elif key.endswith("bn.bias"):
            sd[key] = torch.from_numpy(bn_affine(key[:-len(".bias")], shape[0], seed)[1])
        elif key.endswith("running_mean"):
            sd[key] = torch.zeros(shape, dtype=torch.float32)
        elif key.endswith("running_var"):
            sd[key] = torch.ones(shape, dtype=torch.float32)
        else:
            raise KeyError(f"no synthetic recipe for {key}")
    return sd


def state_dict_sha256(sd) -> str:
    h = hashlib.sha256()
    for key in sorted(sd.keys()):
        t = sd[key].detach().cpu().contiguous()
        h.update(key.encode())
        h.update(t.numpy().tobytes())
    return h.hexdigest()
