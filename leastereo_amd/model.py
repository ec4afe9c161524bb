"""Drop-in ``LEAStereo(args, device)`` whose hot path runs on hand-written HIP kernels.

Mirrors retrain/LEAStereo.py:12-52: same constructor arguments, same
state_dict keys (918 tensors; ``load_state_dict(strict=True)`` of a reference
checkpoint works), same ``forward(left, right) -> [B, H, W]`` disparity.

Everything runs on libleastereo_hip.so (``kernels.py``): the 2D feature net
(retrain/new_model_2d.py, ``FeatureExecutor``; north_star allowed it to stay on
PyTorch -- moved to HIP as SURVEY.md §8f rank 2), the cost volume, the matching net
(``MatchingExecutor``) and the disparity regression.  The nn.Modules here are
parameter containers with the reference's names; there is no torch/CPU compute
path: forward on a non-ROCm device raises.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

# the fused feature stem reads left and right directly (two launches, no concatenated
# copy); LEASTEREO_STEM_PAIR=0 stacks the images first (one launch + a torch copy)
STEM_PAIR = os.environ.get("LEASTEREO_STEM_PAIR", "1") != "0"

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


def _head_modules(mod, initial_fm, dims, last3_bn_relu):
    mod.last_3 = ConvBR(initial_fm, 1 if dims == 3 else initial_fm, 3 if dims == 3 else 1, 1,
                        1 if dims == 3 else 0, bn=False, relu=False, dims=dims)
    mod.last_6 = ConvBR(initial_fm * 2, initial_fm, 1, 1, 0, dims=dims)
    mod.last_12 = ConvBR(initial_fm * 4, initial_fm * 2, 1, 1, 0, dims=dims)
    mod.last_24 = ConvBR(initial_fm * 8, initial_fm * 4, 1, 1, 0, dims=dims)


class _ExecutorCache:
    """Kernel-side parameters (packed weights, folded BN) built on first use and
    dropped whenever the weights may have changed: load_state_dict, .to(), and any
    in-place update of a parameter or buffer (an optimizer step, train-mode running
    statistics -- train.py alternates training with evaluation), seen through the
    tensors' version counters."""

    _executor_cls = None

    def invalidate(self):
        self._executor = None
        self._versioned = None

    def _weights_version(self):
        if getattr(self, "_versioned", None) is None:
            self._versioned = list(self.parameters()) + list(self.buffers())
        return sum(t._version for t in self._versioned)

    def _apply(self, fn, *a, **kw):
        self.invalidate()
        return super()._apply(fn, *a, **kw)

    def _load_from_state_dict(self, *a, **kw):
        self.invalidate()
        return super()._load_from_state_dict(*a, **kw)

    def executor(self):
        if self._executor is not None and self._executor_version != self._weights_version():
            self.invalidate()
        if self._executor is None:
            from . import executor
            self._executor = getattr(executor, self._executor_cls)(self)
            self._executor_version = self._weights_version()
        return self._executor


class NewFeature(_ExecutorCache, nn.Module):
    """2D feature net, retrain/new_model_2d.py:78-165, on the HIP kernels
    (``executor.FeatureExecutor``; ``FeatureExecutorBF16`` at precision bf16)."""

    _executor_cls = "FeatureExecutor"

    def set_precision(self, precision: str):
        cls = "FeatureExecutorBF16" if precision == "bf16" else "FeatureExecutor"
        if cls != self._executor_cls:
            self._executor_cls = cls
            self.invalidate()

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
        self._executor = None

    def forward(self, x, y=None):
        """newFeature.forward(x); with y, the features of x then y as one batch."""
        if not x.is_cuda:
            raise RuntimeError("leastereo_amd feature net runs on a ROCm device only")
        return self.executor().run(x, y)


class NewMatching(_ExecutorCache, nn.Module):
    """Matching net parameters (retrain/skip_model_3d.py:78-138); forward on HIP,
    in f32 (MatchingExecutor) or, with precision "bf16", on the bf16 engine
    (MatchingExecutorBF16, configs 3/4)."""

    _executor_cls = "MatchingExecutor"

    def set_precision(self, precision: str):
        """"f32", "bf16", or "f32_direct" (f32 on the direct-conv engine over the
        in-place cost volume: an independent algorithm, bench.py's per-pair check)."""
        cls = {"f32": "MatchingExecutor", "bf16": "MatchingExecutorBF16",
               "f32_direct": "MatchingExecutorDirect"}.get(precision)
        if cls is None:
            raise ValueError(f"precision must be 'f32', 'bf16' or 'f32_direct', got {precision!r}")
        if cls != self._executor_cls:
            self._executor_cls = cls
            self.invalidate()

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

    def forward(self, cost):
        return self.executor().run(cost)


class Disp(nn.Module):
    """models/build_model_2d.py:45-57, fused into one HIP kernel."""

    def __init__(self, device, maxdisp=192):
        super().__init__()
        self.maxdisp = maxdisp
        self.device = device

    def forward(self, x, fast_exp=False):
        return kernels.disparity_regression(x, self.maxdisp, fast_exp)


class LEAStereo(nn.Module):
    """retrain/LEAStereo.py:12-52 with the hot path on MI355X kernels."""

    def __init__(self, args, device, precision=None):
        """``precision``: "f32" (default; the reference's arithmetic) or "bf16"
        (configs 3/4: matching net on bf16 activations with f32 accumulation; the
        feature net and the disparity regression stay f32).  Also read from
        ``args.precision`` when present."""
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
        self.precision = precision or getattr(args, "precision", None) or "f32"
        self.matching.set_precision(self.precision)
        self.feature.set_precision(self.precision)

    def check_shape(self, height: int, width: int):
        """Reject input sizes the reference cannot run."""
        # stem1 is k3/s3/p1 (new_model_2d.py:94): H3 = (H - 1) // 3 + 1
        check_matching_shape(int(self.maxdisp / 3), (height - 1) // 3 + 1, (width - 1) // 3 + 1,
                             self.matching.specs)

    def forward(self, x, y):
        if not x.is_cuda:
            raise RuntimeError("leastereo_amd.LEAStereo runs the matching net on a ROCm device only")
        self.check_shape(x.shape[2], x.shape[3])
        if self.training or (torch.is_grad_enabled() and (x.requires_grad or y.requires_grad)):
            # train.py:150-158: model.train(); model(input1, input2); loss.backward() -- the
            # differentiable path (train-mode BN, unfused op order, autograd through the
            # library's backward kernels); eval-mode inference takes the executors below
            from .training import leastereo_forward_train
            return leastereo_forward_train(self, x, y)
        # LEAStereo.py:31-32 runs the feature net twice; every layer is per-sample
        # (eval-mode BN), so one call on the stacked pair halves the launch count (the
        # fused stem reads x and y directly into the stacked stem1 maps)
        f = self.feature(x, y) if STEM_PAIR else self.feature(torch.cat((x, y), 0))
        fx, fy = f[: x.shape[0]], f[x.shape[0]:]
        # cost volume (:34-48) + matching (:50): stem0 reads the volume in place
        cost = self.matching.executor().run_features(fx, fy, self.maxdisp)
        return self.disp(cost, fast_exp=self.precision == "bf16")

    def set_precision(self, precision: str):
        """Switch the arithmetic ("f32" / "bf16" / "f32_direct"); weights are re-packed
        on the next forward."""
        self.matching.set_precision(precision)
        self.feature.set_precision(precision)
        self.precision = precision

    def graphed(self, batch: int, height: int, width: int):
        """``forward`` for one input shape captured into a HIP graph (SURVEY.md §7:
        one host call per batch instead of ~140 launches, for serving and for ranks
        that share a node's host CPUs).  The forward issues only library kernels on
        the current stream and never synchronises, so it captures as is."""
        return GraphedForward(self, batch, height, width)


class GraphedForward:
    """``forward`` captured once into a torch.cuda.CUDAGraph (a hipGraph on ROCm)
    with static input/output buffers; ``__call__(x, y)`` copies the inputs in,
    replays, and returns the static output (overwritten by the next call)."""

    def __init__(self, model: LEAStereo, batch: int, height: int, width: int):
        if not torch.cuda.is_available():
            raise RuntimeError("HIP graphs need a ROCm device")
        if model.training:
            # a train-mode forward is the differentiable path (batch-statistics BN, running
            # statistics updated per call, autograd buffers): capture inference only
            raise RuntimeError("graphed() captures the eval-mode forward: call model.eval() first")
        model.check_shape(height, width)
        dev = next(model.parameters()).device
        self.model = model
        self.x = torch.zeros(batch, 3, height, width, device=dev)
        self.y = torch.zeros_like(self.x)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(2):  # packs the weights and warms the allocator outside the capture
                model(self.x, self.y)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = model(self.x, self.y)

    def __call__(self, x, y):
        self.x.copy_(x, non_blocking=True)
        self.y.copy_(y, non_blocking=True)
        self.graph.replay()
        return self.out
