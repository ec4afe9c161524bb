"""Architecture decoding: searched level path + genotype -> static cell table.

Restates models/decoding_formulas.py:6-30 (network_layer_to_space) and the cell
constructor arithmetic of retrain/skip_model_3d.py:96-130 /
retrain/new_model_2d.py:99-133, plus the shape-legality rule the matching net
implies.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

FILTER_PARAM = {0: 1, 1: 2, 2: 4, 3: 8}
PRIMITIVES_3D = ("skip_connect", "3d_conv_3x3")  # models/genotypes_3d.py:5-8
PRIMITIVES_2D = ("skip_connect", "conv_3x3")     # models/genotypes_2d.py:5-8


def network_layer_to_space(net_arch) -> np.ndarray:
    """decoding_formulas.py:6-30: level path -> one-hot [L, 4 levels, 3 samples]."""
    path = [int(v) for v in net_arch]
    space = np.zeros((len(path), 4, 3))
    for i, layer in enumerate(path):
        if i == 0:
            space[0][layer][0] = 1
            continue
        delta = layer - path[i - 1]
        if delta not in (-1, 0, 1):
            raise ValueError(f"level path {path} jumps by {delta} at layer {i}")
        space[i][layer][{1: 0, 0: 1, -1: 2}[delta]] = 1
    return space


@dataclass(frozen=True)
class CellSpec:
    level: int
    downup: int          # -1 down (x0.5), 0, +1 up (x2)
    c_out: int           # filter_multiplier * {1,2,4,8}[level]
    c_prev: int          # channels of s1 (preprocess input)
    c_prev_prev: int     # channels of s0 (pre_preprocess input)


def cell_specs(network_arch: np.ndarray, filter_multiplier: int, block_multiplier: int):
    """The per-cell constants newMatching/newFeature.__init__ derive (skip_model_3d.py:96-130)."""
    initial_fm = filter_multiplier * block_multiplier
    specs = []
    n = network_arch.shape[0]
    for i in range(n):
        level = int(np.argmax(network_arch[i].sum(axis=1)))
        prev_level = int(np.argmax(network_arch[i - 1].sum(axis=1)))
        prev_prev_level = int(np.argmax(network_arch[i - 2].sum(axis=1)))
        if i == 0:
            downup = -level
            fpp = fp = initial_fm / block_multiplier
        else:
            downup = int(np.argmax(network_arch[i].sum(axis=0))) - 1
            fpp = (initial_fm / block_multiplier if i == 1
                   else filter_multiplier * FILTER_PARAM[prev_prev_level])
            fp = filter_multiplier * FILTER_PARAM[prev_level]
        specs.append(CellSpec(level, downup, filter_multiplier * FILTER_PARAM[level],
                              int(block_multiplier * fp), int(block_multiplier * fpp)))
    return specs


def ops_in_iteration_order(cell_arch: np.ndarray, steps: int):
    """Cell DAG as consumed by Cell.forward (skip_model_3d.py:55-72).

    Returns, per step, the list of (op_index, state_index) pairs summed into the
    new state.  ``_ops.k`` is built from cell_arch row k but applied to the k-th
    *matched* branch in iteration order.
    """
    branches = set(int(b) for b in cell_arch[:, 0])
    plan, offset, k, n_states = [], 0, 0, 2
    for _ in range(steps):
        terms = []
        for j in range(n_states):
            if offset + j in branches:
                terms.append((k, j))
                k += 1
        if not terms:
            raise ValueError("a cell step has no incoming branch")
        plan.append(terms)
        offset += n_states
        n_states += 1
    return plan


def scale_dimension(dim: int, scale: float) -> int:
    """skip_model_3d.py:38-39."""
    return int((float(dim) - 1.0) * scale + 1.0) if dim % 2 == 1 else int(float(dim) * scale)


def check_matching_shape(d3: int, h3: int, w3: int, specs) -> None:
    """Raise if the cost-volume size cannot run the matching net.

    The reference fails at torch.cat (skip_model_3d.py:150,155) when a level
    round trip changes a size (e.g. maxdisp=256 -> D3=85); this reports it up front.
    """
    sizes = [(d3, h3, w3)]
    cur = (d3, h3, w3)
    for s in specs:
        if s.downup != 0:
            sc = 0.5 if s.downup < 0 else 2
            cur = tuple(scale_dimension(n, sc) for n in cur)
        sizes.append(cur)
    # skip fusions concat cell1/cell4 and cell4/cell8 outputs
    if len(specs) >= 9 and (sizes[2] != sizes[5] or sizes[5] != sizes[9]):
        raise ValueError(
            f"cost volume {(d3, h3, w3)} is not legal for this matching net: level round trip "
            f"gives {sizes[2]} / {sizes[5]} / {sizes[9]} at the skip fusions "
            "(reference fails in torch.cat at skip_model_3d.py:150,155)")
