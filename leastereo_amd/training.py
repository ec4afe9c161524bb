"""Training backward of the matching net's hot op on the HIP library (SURVEY.md
§8f rank 4): ``ConvBR3d`` is a drop-in for ``models/operations_3d.py:31-47``'s
``ConvBR`` (same constructor, same state_dict keys ``conv.weight``,
``bn.{weight,bias,running_mean,running_var,num_batches_tracked}``) whose forward and
backward run on ``csrc/conv3d_grad.hip`` plus the forward conv engine, so
``train.py:130-178``'s step (``model.train()``, ``loss.backward()``,
``optimizer.step()``) differentiates through it with torch autograd.

Forward (train mode: batch statistics, running-stat update with ``bn.momentum``;
eval mode: running statistics):
    z = conv3d(x, w)                  lea_conv3d_bnrelu[_wino] (stride 1, pad k // 2, no BN;
                                      the inference planner's engine choice)
    y = relu(bn(z))                   lea_bn_forward_f32
Backward:
    dz, dgamma, dbeta                 lea_bn_backward_f32 (ReLU mask from y)
    dx = conv3d(dz, flip(w)^T)        lea_conv3d_flip_weights + lea_conv3d_bnrelu[_wino]
    dw = sum dz (x) x                 lea_conv3d_wgrad (deterministic MFMA reduction)

Only the hot path's ConvBR shapes are supported (stride 1, padding k // 2, k in
{1, 3}, bias-free as the reference's); anything else raises.  There is no CPU
fallback: CPU tensors raise like every other wrapper in ``kernels``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, kernels
from ._lib import LEA_RELU, check


def _stream():
    return torch.cuda.current_stream().cuda_stream


def flip_weights(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, k, k, k] -> [cin, cout, k, k, k] spatially flipped (the input
    gradient's conv weight)."""
    kernels._require_cuda(w)
    w = w.detach().contiguous()
    cout, cin, k = w.shape[0], w.shape[1], w.shape[-1]
    wt = torch.empty((cin, cout, k, k, k), device=w.device, dtype=torch.float32)
    check(_lib.load().lea_conv3d_flip_weights(w.data_ptr(), wt.data_ptr(), cout, cin, k, _stream()),
          "lea_conv3d_flip_weights")
    return wt


def conv3d_wgrad(x: torch.Tensor, dz: torch.Tensor, k: int) -> torch.Tensor:
    """Weight gradient of a stride-1, pad k // 2 Conv3d: x [B, cin, D, H, W],
    dz [B, cout, D, H, W] -> dw [cout, cin, k, k, k]."""
    kernels._require_cuda(x, dz)
    x, dz = x.contiguous(), dz.contiguous()
    b, cin, d, h, w = x.shape
    cout = dz.shape[1]
    if dz.shape[0] != b or tuple(dz.shape[2:]) != (d, h, w):
        raise ValueError(f"conv3d_wgrad: dz {tuple(dz.shape)} does not match x {tuple(x.shape)}")
    lib = _lib.load()
    nws = lib.lea_conv3d_wgrad_workspace_bytes(b, cin, cout, d, h, w, k)
    if nws == 0:
        raise ValueError(f"conv3d_wgrad: unsupported shape {tuple(x.shape)} -> {cout}, k={k}")
    ws = torch.empty(nws // 4, device=x.device, dtype=torch.float32)
    dw = torch.empty((cout, cin, k, k, k), device=x.device, dtype=torch.float32)
    check(lib.lea_conv3d_wgrad(x.data_ptr(), dz.data_ptr(), dw.data_ptr(), ws.data_ptr(), nws, b, cin, cout,
                               d, h, w, k, _stream()), "lea_conv3d_wgrad")
    return dw


def _bn_workspace(c, device):
    n = _lib.load().lea_bn_workspace_bytes(c)
    return torch.empty((n + 7) // 8, device=device, dtype=torch.float64)


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _conv(x: torch.Tensor, w: torch.Tensor, relu: bool = False) -> torch.Tensor:
    """Bias-free stride-1, pad k // 2 conv (optionally ReLU) on the engine the inference
    planner would pick for this shape (Winograd where eligible and measured faster)."""
    cout, cin, k = w.shape[0], w.shape[1], w.shape[-1]
    b, _, d, h, wd = x.shape
    if kernels.wino_eligible(cout, cin, k) and kernels.wino_preferred(b, cout, cin, d, h, wd):
        with kernels.wino_depth_f2():  # the training bars' numerics (kernels.wino_depth_f2)
            return kernels.conv3d_bnrelu_wino(x, kernels.pack_conv_weight_wino(w), cout, None, None, relu=relu)
    return kernels.conv3d_bnrelu(x, kernels.pack_conv_weight(w), cout, k, None, None, relu=relu)


def conv2d_wgrad(x: torch.Tensor, dz: torch.Tensor) -> torch.Tensor:
    """Weight gradient of a Conv2d 3x3 / stride 1 / pad 1 on [B, C, 1, H, W] views:
    x [B, cin, 1, H, W], dz [B, cout, 1, H, W] -> dw [cout, cin, 3, 3]."""
    kernels._require_cuda(x, dz)
    x, dz = x.contiguous(), dz.contiguous()
    b, cin, _, h, w = x.shape
    cout = dz.shape[1]
    lib = _lib.load()
    nws = lib.lea_conv2d_wgrad_workspace_bytes(b, cin, cout, h, w)
    if nws == 0:
        raise ValueError(f"conv2d_wgrad: unsupported shape {tuple(x.shape)} -> {cout}")
    ws = torch.empty(nws // 4, device=x.device, dtype=torch.float32)
    dw = torch.empty((cout, cin, 3, 3), device=x.device, dtype=torch.float32)
    check(lib.lea_conv2d_wgrad(x.data_ptr(), dz.data_ptr(), dw.data_ptr(), ws.data_ptr(), nws, b, cin, cout, h, w,
                               _stream()), "lea_conv2d_wgrad")
    return dw


def conv2d_s3_backward(x: torch.Tensor, dz: torch.Tensor, w: torch.Tensor, need_dx: bool, need_dw: bool):
    """Gradients of the stride-3 stem conv (new_model_2d.py:94): x [B, cin, 1, Hi, Wi],
    dz [B, cout, 1, Ho, Wo], w [cout, cin, 3, 3] -> (dx, dw)."""
    kernels._require_cuda(x, dz, w)
    x, dz, w = x.contiguous(), dz.contiguous(), w.detach().contiguous()
    b, cin, _, hi, wi = x.shape
    cout = w.shape[0]
    lib = _lib.load()
    dx = dw = None
    if need_dx:
        dx = torch.empty_like(x)
        check(lib.lea_conv2d_s3_backward_data(dz.data_ptr(), w.data_ptr(), dx.data_ptr(), b, cin, cout, hi, wi,
                                              _stream()), "lea_conv2d_s3_backward_data")
    if need_dw:
        nws = lib.lea_conv2d_s3_wgrad_workspace_bytes(b, cin, cout, hi, wi)
        ws = torch.empty(nws // 4, device=x.device, dtype=torch.float32)
        dw = torch.empty((cout, cin, 3, 3), device=x.device, dtype=torch.float32)
        check(lib.lea_conv2d_s3_wgrad(x.data_ptr(), dz.data_ptr(), dw.data_ptr(), ws.data_ptr(), nws, b, cin, cout,
                                      hi, wi, _stream()), "lea_conv2d_s3_wgrad")
    return dx, dw


# conv kinds of the ConvBR autograd function: "3d" (Conv3d k in {1, 3}, stride 1),
# "2d" (Conv2d 3x3 / s1 / p1 on [B, C, 1, H, W] views), "s3" (Conv2d 3x3 / s3 / p1)
def _conv_forward(kind, x, w, relu=False):
    if kind == "3d":
        return _conv(x, w, relu=relu)
    if kind == "2d":
        return kernels.conv2d_bnrelu(x, kernels.pack_conv2d_weight(w), w.shape[0], None, None, relu=relu)
    return kernels.conv2d_s3_bnrelu(x, w, None, None, relu=relu)


def _conv_backward(kind, x, w, dz, need_dx, need_dw):
    if kind == "s3":
        return conv2d_s3_backward(x, dz, w, need_dx, need_dw)
    dx = dw = None
    if kind == "3d":
        if need_dx:
            dx = _conv(dz, flip_weights(w))
        if need_dw:
            dw = conv3d_wgrad(x, dz, w.shape[-1])
        return dx, dw
    if need_dx:  # flipped along (kh, kw), [cin, cout, 3, 3]: the transposed conv's weight
        wt = w.detach().flip(2, 3).transpose(0, 1).contiguous()
        dx = kernels.conv2d_bnrelu(dz, kernels.pack_conv2d_weight(wt), w.shape[1], None, None, relu=False)
    if need_dw:
        dw = conv2d_wgrad(x, dz)
    return dx, dw


class _ConvBRFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, training, momentum, eps, use_bn,
                relu, kind="3d"):
        kernels._require_cuda(x, weight)
        x = x.contiguous()
        b, cin = x.shape[:2]
        cout = weight.shape[0]
        if weight.shape[1] != cin:
            raise ValueError(f"ConvBR: weight {tuple(weight.shape)} does not take {cin} channels")
        z = _conv_forward(kind, x, weight, relu=not use_bn and relu)
        v = z.shape[2] * z.shape[3] * z.shape[4]
        lib = _lib.load()
        if use_bn:
            y = torch.empty_like(z)
            mean = torch.empty(cout, device=x.device, dtype=torch.float32)
            invstd = torch.empty_like(mean)
            ws = _bn_workspace(cout, x.device)
            check(lib.lea_bn_forward_f32(z.data_ptr(), y.data_ptr(), b, cout, v, _ptr(gamma), _ptr(beta),
                                         _ptr(running_mean), _ptr(running_var), float(momentum), float(eps),
                                         1 if training else 0, LEA_RELU if relu else 0, mean.data_ptr(),
                                         invstd.data_ptr(), ws.data_ptr(), _stream()), "lea_bn_forward_f32")
        else:
            y = z
            mean = torch.zeros(cout, device=x.device, dtype=torch.float32)
            invstd = torch.ones_like(mean)
        ctx.save_for_backward(x, weight, gamma, z, y, mean, invstd)
        ctx.cfg = (bool(training) and use_bn, use_bn, relu, kind)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, gamma, z, y, mean, invstd = ctx.saved_tensors
        train, use_bn, relu, kind = ctx.cfg
        dy = dy.contiguous()
        b, cout = dy.shape[:2]
        v = dy.shape[2] * dy.shape[3] * dy.shape[4]
        need_g = use_bn and gamma is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        dgamma = torch.empty(cout, device=dy.device, dtype=torch.float32) if need_g else None
        dbeta = torch.empty_like(dgamma) if need_g else None
        dz = torch.empty_like(dy)
        ws = _bn_workspace(cout, dy.device)
        check(_lib.load().lea_bn_backward_f32(
            dy.data_ptr(), y.data_ptr(), z.data_ptr(), dz.data_ptr(), b, cout, v,
            _ptr(gamma) if use_bn else None, mean.data_ptr(), invstd.data_ptr(), 1 if train else 0,
            LEA_RELU if relu else 0, _ptr(dgamma), _ptr(dbeta), ws.data_ptr(), _stream()),
            "lea_bn_backward_f32")
        dx, dw = _conv_backward(kind, x, weight, dz, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return (dx, dw, dgamma if ctx.needs_input_grad[2] else None,
                dbeta if ctx.needs_input_grad[3] else None) + (None,) * 8


_ConvBR3dFn = _ConvBRFn  # the round-3 name (tests, tools)


def resample3d_backward(dy: torch.Tensor, in_size, align_corners: bool = True) -> torch.Tensor:
    """Transpose of ``kernels.resample_trilinear``: dy [B, C, Do, Ho, Wo] -> dx
    [B, C, *in_size]."""
    kernels._require_cuda(dy)
    dy = dy.contiguous()
    b, c, do, ho, wo = dy.shape
    di, hi, wi = (int(s) for s in in_size)
    lib = _lib.load()
    nws = lib.lea_resample3d_backward_workspace_bytes(b, c, di, hi, wi, do, ho, wo)
    if nws == 0:
        raise ValueError(f"resample3d_backward: bad shape {tuple(dy.shape)} <- {tuple(in_size)}")
    ws = torch.empty(nws // 4, device=dy.device, dtype=torch.float32)
    dx = torch.empty((b, c, di, hi, wi), device=dy.device, dtype=torch.float32)
    check(lib.lea_resample3d_trilinear_backward(dy.data_ptr(), dx.data_ptr(), ws.data_ptr(), nws, b, c, di, hi,
                                                wi, do, ho, wo, 1 if align_corners else 0, _stream()),
          "lea_resample3d_trilinear_backward")
    return dx


class _Resample3dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, align_corners):
        ctx.cfg = (tuple(x.shape[2:]), bool(align_corners))
        return kernels.resample_trilinear(x.contiguous(), size, align_corners=align_corners)

    @staticmethod
    def backward(ctx, dy):
        in_size, ac = ctx.cfg
        return resample3d_backward(dy, in_size, ac), None, None


def interpolate3d(x: torch.Tensor, size, align_corners: bool = True) -> torch.Tensor:
    """``F.interpolate(x, size, mode='trilinear', align_corners=...)`` on the HIP
    library, differentiable (skip_model_3d.py:48,50,162; build_model_2d.py:53)."""
    return _Resample3dFn.apply(x, tuple(int(s) for s in size), align_corners)


class _DisparityFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cost, maxdisp):
        disp = kernels.disparity_regression(cost, maxdisp)
        ctx.save_for_backward(cost.contiguous(), disp)
        ctx.maxdisp = maxdisp
        return disp

    @staticmethod
    def backward(ctx, dout):
        cost, disp = ctx.saved_tensors
        b, _, d3, h3, w3 = cost.shape
        # dU transposed along D in the kernel (never materialised over maxdisp planes)
        dv = torch.empty((b, 1, d3, 3 * h3, 3 * w3), device=cost.device, dtype=torch.float32)
        check(_lib.load().lea_disparity_regression_backward(
            cost.data_ptr(), disp.data_ptr(), dout.contiguous().data_ptr(), dv.data_ptr(), b, d3, h3, w3,
            ctx.maxdisp, _stream()), "lea_disparity_regression_backward")
        return resample3d_backward(dv, (d3, h3, w3), align_corners=False), None


def disparity_regression(cost: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """Disp + DisparityRegression (build_model_2d.py:33-42,52-57), differentiable:
    [B, 1, D3, H3, W3] -> [B, 3 H3, 3 W3]."""
    return _DisparityFn.apply(cost, int(maxdisp))


class _CostVolumeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fl, fr, maxdisp):
        ctx.shape = tuple(fl.shape)
        return kernels.build_cost_volume(fl.contiguous(), fr.contiguous(), maxdisp)

    @staticmethod
    def backward(ctx, dcost):
        b, c, h, w = ctx.shape
        dcost = dcost.contiguous()
        dl = torch.empty(ctx.shape, device=dcost.device, dtype=torch.float32)
        dr = torch.empty_like(dl)
        check(_lib.load().lea_build_cost_volume_backward(dcost.data_ptr(), dl.data_ptr(), dr.data_ptr(), b, c, h,
                                                         w, dcost.shape[2], _stream()),
              "lea_build_cost_volume_backward")
        return dl, dr, None


def build_cost_volume(fl: torch.Tensor, fr: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """retrain/LEAStereo.py:34-48's cost volume, differentiable."""
    return _CostVolumeFn.apply(fl, fr, int(maxdisp))


def convbr3d(x, weight, bn: nn.Module | None, relu: bool = True, training: bool = False, kind: str = "3d"):
    """Functional form: ConvBR of x with ``weight`` and (optionally) ``bn``; ``kind``
    "2d" / "s3" for the feature net's Conv2d 3x3 (stride 1 / 3) on [B, C, 1, H, W] views."""
    if bn is None:
        return _ConvBRFn.apply(x, weight, None, None, None, None, False, 0.0, 1e-5, False, relu, kind)
    track = bn.track_running_stats and bn.running_mean is not None
    use_batch = training or not track
    if use_batch and x.shape[0] * x.shape[2] * x.shape[3] * x.shape[4] == 1:
        raise ValueError(f"Expected more than 1 value per channel when training, got input size {tuple(x.shape)}")
    momentum = bn.momentum if bn.momentum is not None else 0.0
    if training and track:
        bn.num_batches_tracked.add_(1)
        if bn.momentum is None:  # cumulative moving average (torch's momentum=None)
            momentum = 1.0 / float(bn.num_batches_tracked.item())
    return _ConvBRFn.apply(x, weight, bn.weight, bn.bias, bn.running_mean if (track and training) or not use_batch
                           else None, bn.running_var if (track and training) or not use_batch else None,
                           use_batch, momentum, bn.eps, True, relu, kind)


class ConvBR3d(nn.Module):
    """``models/operations_3d.py:31-47`` ConvBR on the HIP library, with gradients."""

    def __init__(self, C_in, C_out, kernel_size, stride=1, padding=None, bn=True, relu=True):
        super().__init__()
        padding = kernel_size // 2 if padding is None else padding
        if kernel_size not in (1, 3) or stride != 1 or padding != kernel_size // 2:
            raise NotImplementedError(f"ConvBR3d: k={kernel_size} stride={stride} padding={padding} "
                                      "(the hot path's convs are k in {1, 3}, stride 1, pad k // 2)")
        self.relu = relu
        self.use_bn = bn
        self.conv = nn.Conv3d(C_in, C_out, kernel_size, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm3d(C_out)
        # operations_3d.py:49-56's init
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")
        nn.init.constant_(self.bn.weight, 1)
        nn.init.constant_(self.bn.bias, 0)

    def forward(self, x):
        return convbr3d(x, self.conv.weight, self.bn if self.use_bn else None, self.relu, self.training)


# ------------------------------------------------- the matching net's training forward
def _convbr(m, x, training):
    """A ``model.ConvBR`` parameter container (operations_3d.py:31-47, or
    operations_2d.py:31-47 on a [B, C, 1, H, W] view) through the differentiable HIP op."""
    w, bn = m.conv.weight, (m.bn if m.use_bn else None)
    if w.dim() == 5:
        return convbr3d(x, w, bn, m.relu, training)
    if w.shape[-1] == 1:  # Conv2d 1x1 = Conv3d 1x1x1 on the one-plane view
        return convbr3d(x, w.view(w.shape[0], w.shape[1], 1, 1, 1), bn, m.relu, training)
    if (m.stride, m.padding) not in ((1, 1), (3, 1)):
        raise NotImplementedError(f"Conv2d 3x3 stride={m.stride} padding={m.padding}")
    return convbr3d(x, w, bn, m.relu, training, kind="s3" if m.stride == 3 else "2d")


def _cell(cell, s0, s1, training):
    """Cell.forward, retrain/skip_model_3d.py:41-75 and new_model_2d.py:41-75 (a 2D cell's
    maps are [B, C, 1, H, W] views: its bilinear resize is the trilinear one with an
    identity D axis, scale_dimension(1, s) = 1).  Pairwise sums and the cat stay torch
    autograd glue; every conv, BN, ReLU and resample runs on the HIP library."""
    from .arch import scale_dimension
    prev_input = s1
    if cell.downup_sample != 0:
        sc = 0.5 if cell.downup_sample < 0 else 2
        s1 = interpolate3d(s1, [scale_dimension(n, sc) for n in s1.shape[2:]])
    if tuple(s0.shape[2:]) != tuple(s1.shape[2:]):
        s0 = interpolate3d(s0, s1.shape[2:])
    if s0.shape[1] != cell.c_out:
        s0 = _convbr(cell.pre_preprocess, s0, training)
    s1 = _convbr(cell.preprocess, s1, training)
    states = [s0, s1]
    for terms in cell.plan:
        new = [(_convbr(cell._ops[k], states[j], training) if cell.op_kinds[k] == "conv" else states[j])
               for k, j in terms]
        s = new[0]
        for t in new[1:]:
            s = s + t
        states.append(s)
    return prev_input, torch.cat(states[-cell.block_multiplier:], dim=1)


def matching_forward(net, cost: torch.Tensor, training: bool = True) -> torch.Tensor:
    """newMatching.forward (retrain/skip_model_3d.py:140-174) on ``net``
    (``model.NewMatching``'s parameters) with gradients: the op order of the
    reference (no fused or commuted forms), BN in train mode when ``training``."""
    if cost.dim() != 5:
        raise ValueError("cost must be [B, C, D3, H3, W3]")
    d, h, w = cost.shape[2:]
    stem0 = _convbr(net.stem0, cost, training)
    stem1 = _convbr(net.stem1, stem0, training)
    outs, prev = [], (stem0, stem1)
    n = len(net.cells)
    for i in range(n):
        if i == 5 and n == 12:
            prev = (outs[4][0], _convbr(net.conv1, torch.cat((outs[1][1], outs[4][1]), 1), training))
        elif i == 9 and n == 12:
            prev = (outs[8][0], _convbr(net.conv2, torch.cat((outs[4][1], outs[8][1]), 1), training))
        outs.append(_cell(net.cells[i], prev[0], prev[1], training))
        prev = outs[-1]
    last = outs[-1][1]
    lh = last.shape[3]
    full, half, quarter = (d, h, w), (d // 2, h // 2, w // 2), (d // 4, h // 4, w // 4)
    if lh == h:
        y = last
    elif lh == h // 2:
        y = interpolate3d(_convbr(net.last_6, last, training), full)
    elif lh == h // 4:
        y = interpolate3d(_convbr(net.last_6, interpolate3d(_convbr(net.last_12, last, training), half),
                                  training), full)
    elif lh == h // 8:
        y = interpolate3d(_convbr(net.last_24, last, training), quarter)
        y = interpolate3d(_convbr(net.last_12, y, training), half)
        y = interpolate3d(_convbr(net.last_6, y, training), full)
    else:
        raise ValueError(f"matching-net output size {tuple(last.shape[2:])} has no head")
    return _convbr(net.last_3, y, training)


def cost_to_disparity_train(model, fl: torch.Tensor, fr: torch.Tensor) -> torch.Tensor:
    """retrain/LEAStereo.py:34-51 from the two feature maps, differentiable: cost
    volume -> matching net (BN in the model's train/eval mode) -> Disp."""
    cost = build_cost_volume(fl, fr, model.maxdisp)
    return disparity_regression(matching_forward(model.matching, cost, model.training), model.maxdisp)


# ------------------------------------------------- the feature net and the whole model
def feature_forward(net, x: torch.Tensor, training: bool = True) -> torch.Tensor:
    """newFeature.forward (retrain/new_model_2d.py:140-165) on ``net`` (``model.NewFeature``'s
    parameters) with gradients: x [B, 3, H, W] -> [B, 32, H3, W3], the reference's op order,
    BN in train mode when ``training``."""
    if x.dim() != 4:
        raise ValueError("x must be [B, 3, H, W]")
    stem0 = _convbr(net.stem0, x.unsqueeze(2), training)
    stem1 = _convbr(net.stem1, stem0, training)
    stem2 = _convbr(net.stem2, stem1, training)
    out = (stem1, stem2)
    for cell in net.cells:
        out = _cell(cell, out[0], out[1], training)
    last = out[-1]
    h, w = stem2.shape[3:]
    full, half, quarter = (1, h, w), (1, h // 2, w // 2), (1, h // 4, w // 4)
    lh = last.shape[3]
    if lh == h:
        y = last
    elif lh == h // 2:
        y = interpolate3d(_convbr(net.last_6, last, training), full)
    elif lh == h // 4:
        y = interpolate3d(_convbr(net.last_6, interpolate3d(_convbr(net.last_12, last, training), half),
                                  training), full)
    elif lh == h // 8:
        y = interpolate3d(_convbr(net.last_24, last, training), quarter)
        y = interpolate3d(_convbr(net.last_12, y, training), half)
        y = interpolate3d(_convbr(net.last_6, y, training), full)
    else:
        # the reference raises UnboundLocalError here (new_model_2d.py:156-165)
        raise ValueError(f"feature size {tuple(x.shape[2:])} is not legal for the feature net")
    return _convbr(net.last_3, y, training).squeeze(2)


def leastereo_forward_train(model, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """LEAStereo.forward (retrain/LEAStereo.py:30-52) with gradients, as train.py:150-158
    runs it (``model.train()``, ``model(input1, input2)``, ``loss.backward()``): the feature
    net once per image (train-mode BN normalises each image batch by its own statistics and
    updates the running stats twice, as the reference's two calls do), the cost volume,
    the matching net and Disp, every op on the HIP library."""
    if model.precision != "f32":
        raise NotImplementedError("training runs in f32 (the reference's arithmetic)")
    training = model.training
    fx = feature_forward(model.feature, x, training)
    fy = feature_forward(model.feature, y, training)
    cost = build_cost_volume(fx, fy, model.maxdisp)
    return disparity_regression(matching_forward(model.matching, cost, training), model.maxdisp)
