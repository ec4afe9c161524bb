"""CPU oracle: a from-scratch functional restatement of LEAStereo's inference path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``leastereo_amd``) never
imports it and never falls back to it.

Parity pinning: this restatement is checked against golden vectors produced by
running the reference itself (``/root/reference``, imported in the build
container by ``tools/gen_golden.py``) on the same seeded inputs and weights; the
vectors live in ``tests/golden/`` and ``tests/test_oracle_golden.py`` holds the
check.  Every function cites the reference file:line it restates.

All functions take a flat ``state_dict`` (the reference's key names, e.g.
``matching.cells.3._ops.2.conv.weight``) so the oracle shares no code with the
product's ``nn.Module`` tree.  Works in fp32 and fp64 (dtype follows inputs).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5  # torch.nn.BatchNorm{2,3}d default, used by ConvBR (operations_3d.py:38)
FILTER_PARAM = {0: 1, 1: 2, 2: 4, 3: 8}  # skip_model_3d.py:96 / new_model_2d.py:97


# ---------------------------------------------------------------- architecture
def network_layer_to_space(net_arch) -> np.ndarray:
    """Level path -> one-hot [L,4,3] (models/decoding_formulas.py:6-30)."""
    net_arch = [int(v) for v in net_arch]
    space = np.zeros((len(net_arch), 4, 3))
    prev = None
    for i, layer in enumerate(net_arch):
        if i == 0:
            space[0][layer][0] = 1
        else:
            if layer == prev + 1:
                sample = 0
            elif layer == prev:
                sample = 1
            elif layer == prev - 1:
                sample = 2
            else:  # the reference leaves `sample` stale here; never hit by a legal path
                raise ValueError("level path jumps by more than one level")
            space[i][layer][sample] = 1
        prev = layer
    return space


def cell_levels(network_space: np.ndarray):
    """Per-cell (level, downup) exactly as the cell constructors derive them.

    skip_model_3d.py:97-128 / new_model_2d.py:99-131: ``level`` is argmax over
    the level axis; cell 0 gets ``downup = -level``, the rest
    ``argmax(sum over levels) - 1``.
    """
    out = []
    for i in range(network_space.shape[0]):
        level = int(np.argmax(network_space[i].sum(axis=1)))
        if i == 0:
            downup = -level
        else:
            downup = int(np.argmax(network_space[i].sum(axis=0))) - 1
        out.append((level, downup))
    return out


def scale_dimension(dim: int, scale: float) -> int:
    """skip_model_3d.py:38-39 (identical in new_model_2d.py:38-39)."""
    return int((float(dim) - 1.0) * scale + 1.0) if dim % 2 == 1 else int(float(dim) * scale)


# ------------------------------------------------------------------ primitives
def conv_br(x, sd, prefix, stride=1, bn=True, relu=True):
    """ConvBR: conv (no bias) -> BN (eval) -> ReLU.

    models/operations_3d.py:31-47 (3D) and models/operations_2d.py:31-47 (2D).
    Padding is k//2 for every ConvBR on the inference path.
    """
    w = sd[prefix + ".conv.weight"].to(x.dtype)
    k = w.shape[-1]
    if w.dim() == 5:
        y = F.conv3d(x, w, None, stride, k // 2)
    else:
        y = F.conv2d(x, w, None, stride, k // 2)
    if bn:
        y = F.batch_norm(y, sd[prefix + ".bn.running_mean"].to(x.dtype),
                         sd[prefix + ".bn.running_var"].to(x.dtype),
                         sd[prefix + ".bn.weight"].to(x.dtype),
                         sd[prefix + ".bn.bias"].to(x.dtype), False, 0.0, BN_EPS)
    if relu:
        y = F.relu(y)
    return y


def resample_ac(x, size):
    """Trilinear/bilinear, align_corners=True (skip_model_3d.py:48,50,162)."""
    mode = "trilinear" if x.dim() == 5 else "bilinear"
    return F.interpolate(x, list(size), mode=mode, align_corners=True)


def cell_forward(sd, prefix, s0, s1, downup, cell_arch, primitives, steps=3, block_multiplier=4):
    """Cell.forward, skip_model_3d.py:41-75 (new_model_2d.py:41-75 for 2D).

    primitives[i] is the op kind of ``_ops.i`` ('conv' or 'skip'); ops are
    consumed in *iteration* order of the matched branch indices (:57-68).
    """
    prev_input = s1
    sp = s1.shape[2:]
    if downup != 0:
        scale = 0.5 if downup == -1 else 2
        s1 = resample_ac(s1, [scale_dimension(n, scale) for n in sp])
    if tuple(s0.shape[2:]) != tuple(s1.shape[2:]):
        s0 = resample_ac(s0, s1.shape[2:])
    c_out = sd[prefix + ".preprocess.conv.weight"].shape[0]
    if s0.shape[1] != c_out:
        s0 = conv_br(s0, sd, prefix + ".pre_preprocess")
    s1 = conv_br(s1, sd, prefix + ".preprocess")
    states = [s0, s1]
    branches = set(int(b) for b in cell_arch[:, 0])
    offset = 0
    ops_index = 0
    for _ in range(steps):
        new_states = []
        for j, h in enumerate(states):
            if offset + j in branches:
                if primitives[ops_index] == "conv":
                    new_states.append(conv_br(h, sd, f"{prefix}._ops.{ops_index}"))
                else:
                    new_states.append(h)
                ops_index += 1
        s = new_states[0]
        for t in new_states[1:]:
            s = s + t
        offset += len(states)
        states.append(s)
    return prev_input, torch.cat(states[-block_multiplier:], dim=1)


def _head(sd, prefix, last_output, ref_spatial, mode_dims):
    """Level-dependent head (skip_model_3d.py:161-173 / new_model_2d.py:151-163)."""
    h = ref_spatial[-2]
    lvl_h = last_output.shape[-2]
    full = list(ref_spatial)
    half = [n // 2 for n in ref_spatial]
    quarter = [n // 4 for n in ref_spatial]
    if lvl_h == h:
        y = last_output
    elif lvl_h == h // 2:
        y = resample_ac(conv_br(last_output, sd, prefix + ".last_6"), full)
    elif lvl_h == h // 4:
        y = resample_ac(conv_br(resample_ac(conv_br(last_output, sd, prefix + ".last_12"), half),
                                sd, prefix + ".last_6"), full)
    elif lvl_h == h // 8:
        y = conv_br(last_output, sd, prefix + ".last_24")
        y = resample_ac(y, quarter)
        y = conv_br(y, sd, prefix + ".last_12")
        y = resample_ac(y, half)
        y = resample_ac(conv_br(y, sd, prefix + ".last_6"), full)
    else:
        raise ValueError("unsupported last-level size")
    return y


def _primitives(cell_arch, names):
    return [names[int(p)] for p in cell_arch[:, 1]]


# ----------------------------------------------------------------- subnets
def feature_forward(sd, x, net_arch_fea, cell_arch_fea):
    """newFeature.forward, retrain/new_model_2d.py:140-165."""
    space = network_layer_to_space(net_arch_fea)
    levels = cell_levels(space)
    prims = _primitives(cell_arch_fea, ["skip", "conv"])  # genotypes_2d.py:5-8
    stem0 = conv_br(x, sd, "feature.stem0")
    stem1 = conv_br(stem0, sd, "feature.stem1", stride=3)
    stem2 = conv_br(stem1, sd, "feature.stem2")
    out = (stem1, stem2)
    for i, (_, downup) in enumerate(levels):
        out = cell_forward(sd, f"feature.cells.{i}", out[0], out[1], downup, cell_arch_fea, prims)
    last = out[-1]
    y = _head(sd, "feature", last, stem2.shape[2:], 2)
    return conv_br(y, sd, "feature.last_3", bn=False, relu=False)


def matching_forward(sd, x, net_arch_mat, cell_arch_mat, tap=None):
    """newMatching.forward, retrain/skip_model_3d.py:140-174.  ``tap(name, tensor)``, when
    given, sees each stage's output (stem0, stem1, conv1, conv2, cell{i}, matching): the
    per-stage parity checks compare the HIP executors' stages against these."""
    tap = tap or (lambda name, t: None)
    space = network_layer_to_space(net_arch_mat)
    levels = cell_levels(space)
    prims = _primitives(cell_arch_mat, ["skip", "conv"])  # genotypes_3d.py:5-8
    stem0 = conv_br(x, sd, "matching.stem0")
    tap("stem0", stem0)
    stem1 = conv_br(stem0, sd, "matching.stem1")
    tap("stem1", stem1)
    outs = []
    prev = (stem0, stem1)
    for i, (_, downup) in enumerate(levels):
        if i == 5:   # :150-151
            fused = conv_br(torch.cat((outs[1][-1], outs[4][-1]), 1), sd, "matching.conv1")
            tap("conv1", fused)
            prev = (outs[4][0], fused)
        elif i == 9:  # :155-156
            fused = conv_br(torch.cat((outs[4][-1], outs[8][-1]), 1), sd, "matching.conv2")
            tap("conv2", fused)
            prev = (outs[8][0], fused)
        o = cell_forward(sd, f"matching.cells.{i}", prev[0], prev[1], downup, cell_arch_mat, prims)
        tap(f"cell{i}", o[-1])
        outs.append(o)
        prev = o
    last = outs[-1][-1]
    y = _head(sd, "matching", last, x.shape[2:], 3)
    out = conv_br(y, sd, "matching.last_3", bn=False, relu=False)
    tap("matching", out)
    return out


def build_cost_volume(fl, fr, maxdisp):
    """Cost-volume concat, retrain/LEAStereo.py:34-48.

    cost[b, :C, i, :, i:] = L[..., i:]; cost[b, C:, i, :, i:] = R[..., :W-i];
    columns w < i stay zero in both halves.
    """
    b, c, h, w = fl.shape
    d3 = int(maxdisp / 3)
    cost = fl.new_zeros((b, 2 * c, d3, h, w))
    for i in range(d3):
        if i >= w:
            continue
        cost[:, :c, i, :, i:] = fl[:, :, :, i:]
        cost[:, c:, i, :, i:] = fr[:, :, :, :w - i]
    return cost


def disp_forward(cost, maxdisp):
    """Disp + DisparityRegression, models/build_model_2d.py:27-57.

    trilinear (align_corners=False) to [maxdisp, 3H, 3W] -> softmin over D ->
    sum_d d * p_d with d an fp32 arange (cast to the working dtype).
    """
    x = F.interpolate(cost, [maxdisp, cost.shape[3] * 3, cost.shape[4] * 3], mode="trilinear",
                      align_corners=False)
    x = torch.squeeze(x, 1)
    p = torch.softmax(-x, dim=1)
    d = torch.arange(0, maxdisp, dtype=torch.float32, device=p.device).to(p.dtype).reshape(
        1, maxdisp, 1, 1)
    return torch.sum(p * d, 1)


def leastereo_forward(sd, left, right, maxdisp, arch, return_stages=False, tap=None):
    """LEAStereo.forward, retrain/LEAStereo.py:30-52.

    ``arch`` = dict with net_arch_fea, cell_arch_fea, net_arch_mat, cell_arch_mat
    (the four .npy arrays, LEAStereo.py:16-17).  ``tap``: see matching_forward (plus
    fea_l / fea_r, the feature maps).
    """
    fl = feature_forward(sd, left, arch["net_arch_fea"], arch["cell_arch_fea"])
    fr = feature_forward(sd, right, arch["net_arch_fea"], arch["cell_arch_fea"])
    if tap is not None:
        tap("fea_l", fl)
        tap("fea_r", fr)
    cost = build_cost_volume(fl, fr, maxdisp)
    mat = matching_forward(sd, cost, arch["net_arch_mat"], arch["cell_arch_mat"], tap)
    disp = disp_forward(mat, maxdisp)
    if return_stages:
        return {"fea_l": fl, "fea_r": fr, "cost": cost, "matching": mat, "disp": disp}
    return disp


def epe(a, b):
    """Mean absolute disparity difference (the parity metric of BASELINE.json)."""
    return float((a.double() - b.double()).abs().mean())
