"""Drop-in ``LEAStereo(args, device)`` whose hot path runs on hand-written HIP kernels.

Mirrors retrain/LEAStereo.py:12-52: same constructor arguments, same
state_dict keys (918 tensors; ``load_state_dict(strict=True)`` of a reference
checkpoint works), same ``forward(left, right) -> [B, H, W]`` disparity.

Split (BASELINE.json north_star):
  * 2D feature net (retrain/new_model_2d.py) -> PyTorch-ROCm modules (MIOpen);
  * cost volume, matching net, disparity regression -> libleastereo_hip.so
    (``kernels.py``), driven by ``MatchingExecutor``.
There is no CPU path for the matching net: forward on a non-ROCm device raises.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels
from .arch import (PRIMITIVES_2D, PRIMITIVES_3D, cell_specs, check_matching_shape,
                   network_layer_to_space, ops_in_iteration_order, scale_dimension)


# ----------------------------------------------------------------- parameter modules
class ConvBR(nn.Module):
    """Conv (no bias) + BN + ReLU, key-compatible with models/operations_{2d,3d}.py:31."""

    def __init__(self, c_in, c_out, kernel_size, stride=1, padding=0, bn=True, relu=True, dims=3):
        super().__init__()
        conv = nn.Conv3d if dims == 3 else nn.Conv2d
        norm = nn.BatchNorm3d if dims == 3 else nn.BatchNorm2d
        self.relu = relu
        self.use_bn = bn
        self.stride = stride
        self.padding = padding
        self.conv = conv(c_in, c_out, kernel_size, stride=stride, padding=padding, bias=False)
        self.bn = norm(c_out)
        for m in self.modules():  # operations_3d.py:49-55
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm3d)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward(self, x):  # torch path: used by the 2D feature net only
        x = self.conv(x)
        if self.use_bn:
            x = self.bn(x)
        if self.relu:
            x = F.relu(x, inplace=True)
        return x

    @torch.no_grad()
    def folded_bn(self):
        """scale = gamma/sqrt(var+eps), shift = beta - mean*scale, in fp32 as aten's
        batch_norm inference transform folds them."""
        if not self.use_bn:
            return None, None
        bn = self.bn
        invstd = 1.0 / torch.sqrt(bn.running_var.float() + bn.eps)
        scale = invstd * bn.weight.float()
        shift = bn.bias.float() - bn.running_mean.float() * scale
        return scale.contiguous(), shift.contiguous()


class Cell(nn.Module):
    """Parameter container + 2D forward of a searched cell (skip_model_3d.py:12-75)."""

    def __init__(self, spec, cell_arch, steps, block_multiplier, dims):
        super().__init__()
        prims = PRIMITIVES_3D if dims == 3 else PRIMITIVES_2D
        self.spec = spec
        self.dims = dims
        self.c_out = spec.c_out
        self.steps = steps
        self.block_multiplier = block_multiplier
        self.downup_sample = spec.downup
        self.pre_preprocess = ConvBR(spec.c_prev_prev, spec.c_out, 1, 1, 0, dims=dims)
        self.preprocess = ConvBR(spec.c_prev, spec.c_out, 1, 1, 0, dims=dims)
        self._ops = nn.ModuleList()
        self.op_kinds = []
        for row in cell_arch:
            if prims[int(row[1])] == "skip_connect":
                self._ops.append(nn.Identity())
                self.op_kinds.append("skip")
            else:
                self._ops.append(ConvBR(spec.c_out, spec.c_out, 3, 1, 1, dims=dims))
                self.op_kinds.append("conv")
        self.plan = ops_in_iteration_order(np.asarray(cell_arch), steps)

    def forward(self, s0, s1):
        """2D (feature-net) forward in torch, new_model_2d.py:41-75."""
        prev_input = s1
        if self.downup_sample != 0:
            sc = 0.5 if self.downup_sample < 0 else 2
            s1 = F.interpolate(s1, [scale_dimension(n, sc) for n in s1.shape[2:]],
                               mode="bilinear", align_corners=True)
        if s0.shape[2:] != s1.shape[2:]:
            s0 = F.interpolate(s0, s1.shape[2:], mode="bilinear", align_corners=True)
        if s0.shape[1] != self.c_out:
            s0 = self.pre_preprocess(s0)
        s1 = self.preprocess(s1)
        states = [s0, s1]
        for terms in self.plan:
            s = None
            for k, j in terms:
                t = self._ops[k](states[j])
                s = t if s is None else s + t
            states.append(s)
        return prev_input, torch.cat(states[-self.block_multiplier:], dim=1)


def _head_modules(mod, initial_fm, dims, last3_bn_relu):
    mod.last_3 = ConvBR(initial_fm, 1 if dims == 3 else initial_fm, 3 if dims == 3 else 1, 1,
                        1 if dims == 3 else 0, bn=False, relu=False, dims=dims)
    mod.last_6 = ConvBR(initial_fm * 2, initial_fm, 1, 1, 0, dims=dims)
    mod.last_12 = ConvBR(initial_fm * 4, initial_fm * 2, 1, 1, 0, dims=dims)
    mod.last_24 = ConvBR(initial_fm * 8, initial_fm * 4, 1, 1, 0, dims=dims)


class NewFeature(nn.Module):
    """2D feature net, retrain/new_model_2d.py:78-165 (stays on PyTorch-ROCm)."""

    def __init__(self, network_arch, cell_arch, args):
        super().__init__()
        fm, bm, steps = args.fea_filter_multiplier, args.fea_block_multiplier, args.fea_step
        initial_fm = fm * bm
        self.cells = nn.ModuleList()  # registered first, as new_model_2d.py:82
        self.stem0 = ConvBR(3, initial_fm // 2, 3, stride=1, padding=1, dims=2)
        self.stem1 = ConvBR(initial_fm // 2, initial_fm, 3, stride=3, padding=1, dims=2)
        self.stem2 = ConvBR(initial_fm, initial_fm, 3, stride=1, padding=1, dims=2)
        specs = cell_specs(network_arch[: args.fea_num_layers], fm, bm)
        self.cells.extend(Cell(s, cell_arch, steps, bm, 2) for s in specs)
        _head_modules(self, initial_fm, 2, False)

    def forward(self, x):
        stem1 = self.stem1(self.stem0(x))
        stem2 = self.stem2(stem1)
        out = (stem1, stem2)
        for cell in self.cells:
            out = cell(out[0], out[1])
        last = out[-1]
        h, w = stem2.shape[2:]
        up = lambda t, size: F.interpolate(t, size, mode="bilinear", align_corners=True)  # noqa: E731
        if last.shape[2] == h:
            fea = last
        elif last.shape[2] == h // 2:
            fea = up(self.last_6(last), [h, w])
        elif last.shape[2] == h // 4:
            fea = up(self.last_6(up(self.last_12(last), [h // 2, w // 2])), [h, w])
        elif last.shape[2] == h // 8:
            fea = up(self.last_6(up(self.last_12(up(self.last_24(last), [h // 4, w // 4])),
                                    [h // 2, w // 2])), [h, w])
        else:
            # the reference raises UnboundLocalError here (new_model_2d.py:156-165)
            raise ValueError(f"feature size {tuple(x.shape[2:])} is not legal for the feature net")
        return self.last_3(fea)


class NewMatching(nn.Module):
    """Matching net parameters (retrain/skip_model_3d.py:78-138); forward on HIP."""

    def __init__(self, network_arch, cell_arch, args):
        super().__init__()
        fm, bm, steps = args.mat_filter_multiplier, args.mat_block_multiplier, args.mat_step
        initial_fm = fm * bm
        self.cells = nn.ModuleList()  # registered first, as skip_model_3d.py:82
        self.stem0 = ConvBR(initial_fm * 2, initial_fm, 3, stride=1, padding=1)
        self.stem1 = ConvBR(initial_fm, initial_fm, 3, stride=1, padding=1)
        self.specs = cell_specs(network_arch[: args.mat_num_layers], fm, bm)
        self.cells.extend(Cell(s, cell_arch, steps, bm, 3) for s in self.specs)
        _head_modules(self, initial_fm, 3, False)
        self.conv1 = ConvBR(initial_fm * 4, initial_fm * 2, 3, 1, 1)
        self.conv2 = ConvBR(initial_fm * 4, initial_fm * 2, 3, 1, 1)
        self._executor = None

    # parameter caches for the kernels are rebuilt whenever weights may have changed
    def invalidate(self):
        self._executor = None

    def _apply(self, fn, *a, **kw):
        self.invalidate()
        return super()._apply(fn, *a, **kw)

    def _load_from_state_dict(self, *a, **kw):
        self.invalidate()
        return super()._load_from_state_dict(*a, **kw)

    def executor(self):
        if self._executor is None:
            from .executor import MatchingExecutor
            self._executor = MatchingExecutor(self)
        return self._executor

    def forward(self, cost):
        return self.executor().run(cost)


class Disp(nn.Module):
    """models/build_model_2d.py:45-57, fused into one HIP kernel."""

    def __init__(self, device, maxdisp=192):
        super().__init__()
        self.maxdisp = maxdisp
        self.device = device

    def forward(self, x):
        return kernels.disparity_regression(x, self.maxdisp)


class LEAStereo(nn.Module):
    """retrain/LEAStereo.py:12-52 with the hot path on MI355X kernels."""

    def __init__(self, args, device):
        super().__init__()
        network_path_fea = np.load(args.net_arch_fea)
        cell_arch_fea = np.load(args.cell_arch_fea)
        network_path_mat = np.load(args.net_arch_mat)
        cell_arch_mat = np.load(args.cell_arch_mat)
        self.maxdisp = args.maxdisp
        self.feature = NewFeature(network_layer_to_space(network_path_fea), cell_arch_fea, args)
        self.matching = NewMatching(network_layer_to_space(network_path_mat), cell_arch_mat, args)
        self.disp = Disp(device, self.maxdisp)
        self.use_cuda = getattr(args, "cuda", True)
        self.device = device

    def check_shape(self, height: int, width: int):
        """Reject input sizes the reference cannot run."""
        # stem1 is k3/s3/p1 (new_model_2d.py:94): H3 = (H - 1) // 3 + 1
        check_matching_shape(int(self.maxdisp / 3), (height - 1) // 3 + 1, (width - 1) // 3 + 1,
                             self.matching.specs)

    def forward(self, x, y):
        if not x.is_cuda:
            raise RuntimeError("leastereo_amd.LEAStereo runs the matching net on a ROCm device only")
        self.check_shape(x.shape[2], x.shape[3])
        # LEAStereo.py:31-32 runs the feature net twice; in eval mode every layer is
        # per-sample, so one call on the stacked pair halves the (launch-bound)
        # torch/MIOpen kernel count.
        f = self.feature(torch.cat((x, y), 0))
        fx, fy = f[: x.shape[0]], f[x.shape[0]:]
        cost = kernels.build_cost_volume(fx, fy, self.maxdisp)
        cost = self.matching(cost)
        return self.disp(cost)
