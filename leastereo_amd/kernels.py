"""Tensor-level wrappers over the C ABI: device tensors in, device tensors out.

Each wrapper checks shapes/strides on the host, then launches on the current
HIP stream (``torch.cuda.current_stream()``), so it composes with torch ops
and is capturable by ``torch.cuda.graph``.  There is no fallback: a non-CUDA
tensor or a missing library raises.
"""
from __future__ import annotations

import contextlib
import os

import torch

from . import _lib
from ._lib import LEA_F32, LEA_PAIR_SUM, LEA_RELU, LEA_RESIDUAL, check


def _stream():
    return torch.cuda.current_stream().cuda_stream


class KernelProbe:
    """Times launches of conv kernel instantiations with HIP events recorded on
    the stream the kernel is launched on (torch's current stream).

    ``names=None`` records every conv launch.  Each record carries the launch's
    algorithmic FLOPs and bytes (input + output + weights [+ residual read]).
    """

    def __init__(self, names=None):
        self.names = None if names is None else set(names)
        self.records = []  # (name, flops, bytes, start_event, end_event, mfma_flops, shape)

    def __enter__(self):
        global _probe
        _probe = self
        return self

    def __exit__(self, *exc):
        global _probe
        _probe = None

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, flops, nbytes, e0, e1, mfma, _ in self.records:
            d = out.setdefault(name, {"launches": 0, "flops": 0.0, "bytes": 0.0, "ms": 0.0,
                                      "mfma_flops": 0.0})
            d["launches"] += 1
            d["flops"] += flops
            d["bytes"] += nbytes
            d["ms"] += e0.elapsed_time(e1)
            d["mfma_flops"] += mfma
        return out

    def by_shape(self, name):
        """Launches of kernel ``name`` grouped by layer shape (B, cin, cout, D, H, W, k)."""
        torch.cuda.synchronize()
        out = {}
        for n, flops, nbytes, e0, e1, mfma, shape in self.records:
            if n != name:
                continue
            d = out.setdefault(shape, {"launches": 0, "flops": 0.0, "bytes": 0.0, "ms": 0.0, "mfma_flops": 0.0})
            d["launches"] += 1
            d["flops"] += flops
            d["bytes"] += nbytes
            d["ms"] += e0.elapsed_time(e1)
            d["mfma_flops"] += mfma
        return out


_probe = None


def conv_kernel_name(b, cout, d, h, w, k, resampled=False):
    name = _lib.load().lea_conv3d_kernel_name(b, cout, d, h, w, k, 1 if resampled else 0)
    return name.decode() if name else None


def _require_cuda(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise _lib.HipKernelError(
                f"HIP path needs float32 tensors on a ROCm device, got {t.dtype} on {t.device}")


def _check_volume_view(t: torch.Tensor, name: str):
    """NCDHW tensor whose (C, D, H, W) block is contiguous per batch (a channel
    slice of a contiguous tensor qualifies); returns the batch stride."""
    b, c, d, h, w = t.shape
    if t.stride()[1:] != (d * h * w, h * w, w, 1):
        raise ValueError(f"{name}: NCDHW slice with contiguous C,D,H,W required, strides {t.stride()}")
    return t.stride(0)


def build_cost_volume(fl: torch.Tensor, fr: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """retrain/LEAStereo.py:34-48 -> [B, 2C, int(maxdisp/3), H, W]."""
    _require_cuda(fl, fr)
    fl, fr = fl.contiguous(), fr.contiguous()
    if fl.shape != fr.shape or fl.dim() != 4:
        raise ValueError("left/right features must both be [B, C, H, W]")
    b, c, h, w = fl.shape
    d3 = int(maxdisp / 3)
    cost = torch.empty((b, 2 * c, d3, h, w), device=fl.device, dtype=fl.dtype)
    check(_lib.load().lea_build_cost_volume(fl.data_ptr(), fr.data_ptr(), cost.data_ptr(), b, c, h,
                                            w, d3, LEA_F32, _stream()), "lea_build_cost_volume")
    return cost


def packed_floats(cout: int, cin: int, k: int) -> int:
    n = _lib.load().lea_conv3d_packed_floats(cout, cin, k)
    if n == 0:
        raise ValueError(f"unsupported conv shape cout={cout} cin={cin} k={k}")
    return n


def pack_conv_weight(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, k, k, k] fp32 device weight -> the kernel's packed layout."""
    _require_cuda(w)
    w = w.detach().contiguous()
    cout, cin, k = w.shape[0], w.shape[1], w.shape[-1]
    packed = torch.empty(packed_floats(cout, cin, k), device=w.device, dtype=torch.float32)
    check(_lib.load().lea_conv3d_pack_weights(w.data_ptr(), packed.data_ptr(), cout, cin, k,
                                              _stream()), "lea_conv3d_pack_weights")
    return packed


def _probe_begin(b, cin, cout, d, h, w, k, accumulate, in_vox, resampled, name=None, mfma_scale=1.0,
                 esz=4):
    """Start HIP-event timing of this launch if the active probe wants its kernel.
    ``flops`` is the direct convolution's (the reference algorithm's) count;
    ``mfma_scale`` converts it to the products the kernel actually issues (2/3 for
    Winograd F(2,3), times its cout padding); ``esz`` is the activation element size."""
    probe = _probe
    if probe is None:
        return None
    if name is None:
        name = conv_kernel_name(b, cout, d, h, w, k, resampled)
    if probe.names is not None and name not in probe.names:
        return None
    vox = b * d * h * w
    flops = 2.0 * vox * cout * cin * k ** 3
    nbytes = esz * (in_vox * cin + vox * cout * (2 if accumulate else 1)) + 4.0 * cout * cin * k ** 3
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return probe, name, flops, nbytes, e0, flops * mfma_scale, (b, cin, cout, d, h, w, k)


def _probe_launch(name, flops, nbytes, mfma=None):
    """Start HIP-event timing of a launch that is not a 3D conv (2D convs, resamples,
    the head, the disparity regression, layout conversions): ``flops`` / ``nbytes`` are
    its algorithmic work, ``mfma`` the matrix-core products it issues (default: flops)."""
    probe = _probe
    if probe is None or (probe.names is not None and name not in probe.names):
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return probe, name, float(flops), float(nbytes), e0, float(flops if mfma is None else mfma), None


def _probe_end(rec):
    if rec is not None:
        probe, name, flops, nbytes, e0, mfma, shape = rec
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        probe.records.append((name, flops, nbytes, e0, e1, mfma, shape))


def _conv_out(x_shape5, cout, spatial, out, accumulate, device, dtype):
    b = x_shape5[0]
    shape = (b, cout) + tuple(int(s) for s in spatial)
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(shape, device=device, dtype=dtype)
    if tuple(out.shape) != shape:
        raise ValueError(f"out shape {tuple(out.shape)} != {shape}")
    return out, _check_volume_view(out, "out")


def _residual(out, accumulate, residual, ybs):
    """(pointer, batch stride) of the epilogue's residual: ``out`` itself under
    ``accumulate``, else an explicit tensor of out's shape (or none)."""
    if accumulate:
        if residual is not None:
            raise ValueError("accumulate and residual are exclusive")
        return out.data_ptr(), ybs
    if residual is None:
        return None, 0
    _require_cuda(residual)
    if tuple(residual.shape) != tuple(out.shape):
        raise ValueError(f"residual shape {tuple(residual.shape)} != {tuple(out.shape)}")
    return residual.data_ptr(), _check_volume_view(residual, "residual")


def conv3d_bnrelu(x: torch.Tensor, packed: torch.Tensor, cout: int, k: int,
                  scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool = True,
                  out: torch.Tensor | None = None, accumulate: bool = False,
                  x2: torch.Tensor | None = None,
                  residual: torch.Tensor | None = None) -> torch.Tensor:
    """ConvBR3d (operations_3d.py:41-47) of ``torch.cat((x, x2), 1)`` (x2 optional,
    never materialised).  ``out`` may be a channel slice of a larger (cat) buffer;
    ``accumulate`` adds the activation to what ``out`` holds (the cell's pairwise
    sum, skip_model_3d.py:69)."""
    _require_cuda(x, x2, packed, scale, shift, out)
    b, cin, d, h, w = x.shape
    xbs = _check_volume_view(x, "x")
    cin2, x2bs = 0, 0
    if x2 is not None:
        if x2.shape[0] != b or tuple(x2.shape[2:]) != (d, h, w):
            raise ValueError("x2 must match x in batch and volume")
        cin2 = x2.shape[1]
        x2bs = _check_volume_view(x2, "x2")
    out, ybs = _conv_out(x.shape, cout, (d, h, w), out, accumulate, x.device, x.dtype)
    rptr, rbs = _residual(out, accumulate, residual, ybs)
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0)
    rec = _probe_begin(b, cin + cin2, cout, d, h, w, k, rptr is not None, b * d * h * w, False)
    check(_lib.load().lea_conv3d_bnrelu(
        x.data_ptr(), xbs, x2.data_ptr() if x2 is not None else None, x2bs, cin2,
        packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None,
        rptr, rbs, out.data_ptr(), ybs, b, cin + cin2, cout, d, h, w, k, flags, LEA_F32, _stream()),
        "lea_conv3d_bnrelu")
    _probe_end(rec)
    return out


def costvolume_kernel_name(b, cout, d3, h, w):
    name = _lib.load().lea_conv3d_costvolume_kernel_name(b, cout, d3, h, w)
    return name.decode() if name else None


def conv3d_bnrelu_costvolume(fl: torch.Tensor, fr: torch.Tensor, maxdisp: int, packed: torch.Tensor,
                             cout: int, scale: torch.Tensor | None, shift: torch.Tensor | None,
                             relu: bool = True) -> torch.Tensor:
    """ConvBR3d 3x3x3 of the cost volume of (fl, fr) (LEAStereo.py:34-48 then
    skip_model_3d.py:141) without materialising the volume; bit-identical to
    ``conv3d_bnrelu(build_cost_volume(fl, fr, maxdisp), ...)``."""
    _require_cuda(fl, fr, packed, scale, shift)
    if fl.shape != fr.shape or fl.dim() != 4:
        raise ValueError("left/right features must both be [B, C, H, W]")
    if fl.stride() != fr.stride() or fl.stride()[1:] != (fl.shape[2] * fl.shape[3], fl.shape[3], 1):
        raise ValueError("left/right features need contiguous C,H,W and equal strides")
    b, c, h, w = fl.shape
    d3 = int(maxdisp / 3)
    out = torch.empty((b, cout, d3, h, w), device=fl.device, dtype=fl.dtype)
    rec = None if _probe is None else _probe_begin(b, 2 * c, cout, d3, h, w, 3, False, 0, False,
                                                   name=costvolume_kernel_name(b, cout, d3, h, w))
    check(_lib.load().lea_conv3d_bnrelu_costvolume(
        fl.data_ptr(), fr.data_ptr(), fl.stride(0), packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), out.stride(0), b, c, cout,
        d3, h, w, LEA_RELU if relu else 0, LEA_F32, _stream()), "lea_conv3d_bnrelu_costvolume")
    _probe_end(rec)
    return out


def conv3d_bnrelu_resampled(x: torch.Tensor, size, packed: torch.Tensor, cout: int, k: int,
                            scale: torch.Tensor | None, shift: torch.Tensor | None,
                            relu: bool = True, out: torch.Tensor | None = None,
                            accumulate: bool = False) -> torch.Tensor:
    """ConvBR3d(F.interpolate(x, size, mode='trilinear', align_corners=True)) with
    the interpolation fused into the conv's input staging (skip_model_3d.py:44-53)."""
    _require_cuda(x, packed, scale, shift, out)
    b, cin, di, hi, wi = x.shape
    d, h, w = (int(s) for s in size)
    xbs = _check_volume_view(x, "x")
    out, ybs = _conv_out(x.shape, cout, (d, h, w), out, accumulate, x.device, x.dtype)
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if accumulate else 0)
    rec = _probe_begin(b, cin, cout, d, h, w, k, accumulate, b * di * hi * wi, True)
    check(_lib.load().lea_conv3d_bnrelu_resampled(
        x.data_ptr(), xbs, di, hi, wi, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None,
        out.data_ptr() if accumulate else None, ybs if accumulate else 0,
        out.data_ptr(), ybs, b, cin, cout, d, h, w, k, flags, LEA_F32, _stream()),
        "lea_conv3d_bnrelu_resampled")
    _probe_end(rec)
    return out


# ------------------------------------------------------------------- 2D feature net
# Feature-net activations travel as NCDHW views with D = 1 ([B, C, 1, H, W]), so the
# 1x1 convs and bilinear resizes are the 3D entry points on a single plane.

def conv2d_kernel_name(b, cout, h, w, cin=None):
    lib = _lib.load()
    name = (lib.lea_conv2d_kernel_name(b, cout, h, w) if cin is None
            else lib.lea_conv2d_kernel_name_cin(b, cin, cout, h, w))
    return name.decode() if name else None


def pack_conv2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, 3, 3] fp32 device weight -> packed layout of lea_conv2d_bnrelu."""
    _require_cuda(w)
    w = w.detach().contiguous()
    if w.dim() != 4 or tuple(w.shape[2:]) != (3, 3):
        raise ValueError(f"expected a [cout, cin, 3, 3] weight, got {tuple(w.shape)}")
    cout, cin = w.shape[:2]
    n = _lib.load().lea_conv2d_packed_floats(cout, cin)
    packed = torch.empty(n, device=w.device, dtype=torch.float32)
    check(_lib.load().lea_conv2d_pack_weights(w.data_ptr(), packed.data_ptr(), cout, cin, _stream()),
          "lea_conv2d_pack_weights")
    return packed


def conv2d_bnrelu(x: torch.Tensor, packed: torch.Tensor, cout: int,
                  scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool = True,
                  out: torch.Tensor | None = None, accumulate: bool = False,
                  residual: torch.Tensor | None = None) -> torch.Tensor:
    """ConvBR2d 3x3/s1/p1 (operations_2d.py:31-47) on x [B, cin, 1, H, W]; ``residual``
    (or ``accumulate`` into out) adds a cell-sum operand in the epilogue."""
    _require_cuda(x, packed, scale, shift, out)
    b, cin, d, h, w = x.shape
    if d != 1:
        raise ValueError("conv2d_bnrelu takes [B, C, 1, H, W] views")
    xbs = _check_volume_view(x, "x")
    out, ybs = _conv_out(x.shape, cout, (1, h, w), out, accumulate, x.device, x.dtype)
    rptr, rbs = _residual(out, accumulate, residual, ybs)
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0)
    rec = None if _probe is None else _probe_launch(
        conv2d_kernel_name(b, cout, h, w, cin), 2.0 * b * h * w * cout * cin * 9,
        4.0 * b * h * w * (cin + cout * (2 if rptr is not None else 1)) + 36.0 * cout * cin)
    check(_lib.load().lea_conv2d_bnrelu(
        x.data_ptr(), xbs, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None,
        rptr, rbs, out.data_ptr(), ybs, b, cin, cout, h, w, flags, LEA_F32, _stream()),
        "lea_conv2d_bnrelu")
    _probe_end(rec)
    return out


def conv2d_bnrelu_pair(x: torch.Tensor, packed: torch.Tensor, c1: int, cout: int,
                       scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool,
                       out1: torch.Tensor, out2: torch.Tensor,
                       residual: torch.Tensor | None = None) -> None:
    """Two ConvBR2d 3x3/s1/p1 of x [B, cin, 1, H, W] in one launch (lea_conv2d_bnrelu_pair):
    ``packed`` holds both weight stacks along cout; couts [0, c1) go to ``out1`` (plus the
    ``residual``, the cell's skip term), [c1, cout) to ``out2`` ([B, cout - c1, 1, H, W] views,
    e.g. two non-adjacent slots of a cell's cat buffer)."""
    _require_cuda(x, packed, scale, shift, out1, out2, residual)
    b, cin, d, h, w = x.shape
    if d != 1:
        raise ValueError("conv2d_bnrelu_pair takes [B, C, 1, H, W] views")
    xbs = _check_volume_view(x, "x")
    if tuple(out1.shape) != (b, c1, 1, h, w) or tuple(out2.shape) != (b, cout - c1, 1, h, w):
        raise ValueError(f"conv2d_bnrelu_pair: outputs {tuple(out1.shape)} / {tuple(out2.shape)}")
    y1bs, y2bs = _check_volume_view(out1, "out1"), _check_volume_view(out2, "out2")
    rptr, rbs = None, 0
    if residual is not None:
        if tuple(residual.shape) != tuple(out1.shape):
            raise ValueError(f"conv2d_bnrelu_pair: residual {tuple(residual.shape)}")
        rbs = _check_volume_view(residual, "residual")
        rptr = residual.data_ptr()
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0)
    rec = None if _probe is None else _probe_launch(
        conv2d_kernel_name(b, cout, h, w, cin), 2.0 * b * h * w * cout * cin * 9,
        4.0 * b * h * w * (cin + cout + (c1 if rptr is not None else 0)) + 36.0 * cout * cin)
    check(_lib.load().lea_conv2d_bnrelu_pair(
        x.data_ptr(), xbs, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None,
        rptr, rbs, out1.data_ptr(), y1bs, out2.data_ptr(), y2bs, b, cin, cout, c1, h, w, flags, _stream()),
        "lea_conv2d_bnrelu_pair")
    _probe_end(rec)


def feature_stem(x: torch.Tensor, w0: torch.Tensor, scale0, shift0, w1: torch.Tensor, scale1, shift1,
                 c8: bool = False, x2: torch.Tensor | None = None) -> torch.Tensor:
    """new_model_2d.py:93-94 fused (ConvBR 3x3 s1 then ConvBR 3x3 s3, BN + ReLU each):
    x [B, cin, H, W] f32 -> [B, c1, 1, Ho, Wo] f32, or c8 [B, c1/8, 1, Ho, Wo, 8] bf16.
    With ``x2`` (same shape) the output stacks both, [x; x2] along the batch, without
    a concatenated copy of the images: one launch per source, or for one image each a
    single launch whose batch stride is the distance between the two images."""
    _require_cuda(x, x2, scale0, shift0, scale1, shift1)
    w0, w1 = w0.detach().contiguous(), w1.detach().contiguous()
    _require_cuda(w0, w1)
    x = x.contiguous()
    srcs = [x]
    if x2 is not None:
        if tuple(x2.shape) != tuple(x.shape):
            raise ValueError(f"feature_stem: x2 {tuple(x2.shape)} differs from x {tuple(x.shape)}")
        x2 = x2.contiguous()  # both branches below read this tensor (pointer difference too)
        srcs.append(x2)
    b, cin, hi, wi = x.shape
    c0, c1 = w0.shape[0], w1.shape[0]
    if tuple(w0.shape) != (c0, cin, 3, 3) or tuple(w1.shape) != (c1, c0, 3, 3):
        raise ValueError(f"feature_stem: weights {tuple(w0.shape)} / {tuple(w1.shape)} do not chain")
    ho, wo = (hi - 1) // 3 + 1, (wi - 1) // 3 + 1
    nb = b * len(srcs)
    if c8:
        out = torch.empty((nb, c1 // 8, 1, ho, wo, 8), device=x.device, dtype=torch.bfloat16)
    else:
        out = torch.empty((nb, c1, 1, ho, wo), device=x.device, dtype=torch.float32)
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    if len(srcs) == 2 and b == 1:
        # one image per source: one launch whose batch stride is the distance between them
        srcs, b, xbs = [x], 2, (x2.data_ptr() - x.data_ptr()) // x.element_size()
    else:
        xbs = x.stride(0)
    rec = None if _probe is None else _probe_launch(
        "feature_stem_kernel", 2.0 * nb * ho * wo * (9 * 9 * cin * c0 + 9 * c0 * c1),
        4.0 * nb * cin * hi * wi + out.numel() * out.element_size(), 0.0)
    for i, src in enumerate(srcs):
        check(_lib.load().lea_feature_stem_bnrelu(
            src.data_ptr(), xbs, w0.data_ptr(), ptr(scale0), ptr(shift0), w1.data_ptr(),
            ptr(scale1), ptr(shift1), out[i * b:].data_ptr(), out.stride(0), b, cin, c0, c1, hi, wi,
            _lib.LEA_BF16 if c8 else LEA_F32, _stream()), "lea_feature_stem_bnrelu")
    _probe_end(rec)
    return out


def conv2d_s3_bnrelu(x: torch.Tensor, w: torch.Tensor, scale: torch.Tensor | None,
                     shift: torch.Tensor | None, relu: bool = True) -> torch.Tensor:
    """ConvBR2d 3x3, stride 3, pad 1 (new_model_2d.py:94) on x [B, cin, 1, H, W]."""
    _require_cuda(x, w, scale, shift)
    b, cin, d, hi, wi = x.shape
    if d != 1:
        raise ValueError("conv2d_s3_bnrelu takes [B, C, 1, H, W] views")
    w = w.detach().contiguous()
    cout = w.shape[0]
    if tuple(w.shape) != (cout, cin, 3, 3):
        raise ValueError(f"weight {tuple(w.shape)} does not match cin={cin}")
    xbs = _check_volume_view(x, "x")
    out = torch.empty((b, cout, 1, (hi - 1) // 3 + 1, (wi - 1) // 3 + 1), device=x.device,
                      dtype=x.dtype)
    rec = None if _probe is None else _probe_launch(
        "conv2d_s3_kernel", 2.0 * out.numel() * cin * 9, 4.0 * (x.numel() + out.numel()), 0.0)
    check(_lib.load().lea_conv2d_s3_bnrelu(
        x.data_ptr(), xbs, w.data_ptr(), scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), out.stride(0), b, cin,
        cout, hi, wi, LEA_RELU if relu else 0, LEA_F32, _stream()), "lea_conv2d_s3_bnrelu")
    _probe_end(rec)
    return out


def resample_trilinear(x: torch.Tensor, size, align_corners: bool = True,
                       out: torch.Tensor | None = None, scale: torch.Tensor | None = None,
                       shift: torch.Tensor | None = None, relu: bool = False) -> torch.Tensor:
    """F.interpolate(x, size, mode='trilinear', align_corners=...) for NCDHW, with
    an optional per-channel ``relu(scale * . + shift)`` epilogue; ``out`` may be a
    channel slice of a larger tensor."""
    _require_cuda(x, out, scale, shift)
    b, c, di, hi, wi = x.shape
    do, ho, wo = (int(s) for s in size)
    xbs = _check_volume_view(x, "x")
    if out is None:
        out = torch.empty((b, c, do, ho, wo), device=x.device, dtype=x.dtype)
    if tuple(out.shape) != (b, c, do, ho, wo):
        raise ValueError(f"out shape {tuple(out.shape)} != {(b, c, do, ho, wo)}")
    ybs = _check_volume_view(out, "out")
    rec = None if _probe is None else _probe_launch(
        "resample3d_f32", 0.0, 4.0 * b * c * (di * hi * wi + do * ho * wo))
    check(_lib.load().lea_resample3d_trilinear(
        x.data_ptr(), xbs, out.data_ptr(), ybs, b, c, di, hi, wi, do, ho, wo,
        1 if align_corners else 0, scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, LEA_RELU if relu else 0, LEA_F32,
        _stream()), "lea_resample3d_trilinear")
    _probe_end(rec)
    return out


def tapsum_upsample(q: torch.Tensor, cout: int, size, scale: torch.Tensor | None = None,
                    shift: torch.Tensor | None = None, relu: bool = False) -> torch.Tensor:
    """conv3x3x3(upsample(y)) from q = per-tap partial sums of y (27*cout channels at
    the low resolution): see include/leastereo_hip.h lea_tapsum_upsample."""
    _require_cuda(q, scale, shift)
    b, c27, di, hi, wi = q.shape
    if c27 != 27 * cout:
        raise ValueError(f"q has {c27} channels, expected 27*{cout}")
    qbs = _check_volume_view(q, "q")
    do, ho, wo = (int(s) for s in size)
    out = torch.empty((b, cout, do, ho, wo), device=q.device, dtype=q.dtype)
    lib = _lib.load()
    ws = torch.empty(lib.lea_tapsum_workspace_bytes(b, cout, hi, wi, do) // 4, device=q.device,
                     dtype=torch.float32)
    rec = None if _probe is None else _probe_launch(
        "tapsum_f32", 0.0, 4.0 * (q.shape[0] * q.shape[1] * di * hi * wi + out.numel()))
    check(lib.lea_tapsum_upsample(
        q.data_ptr(), qbs, out.data_ptr(), out.stride(0), b, cout, di, hi, wi, do, ho, wo,
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, LEA_RELU if relu else 0,
        ws.data_ptr(), LEA_F32, _stream()), "lea_tapsum_upsample")
    _probe_end(rec)
    return out


def disparity_regression(cost: torch.Tensor, maxdisp: int, fast_exp: bool = False) -> torch.Tensor:
    """Disp + DisparityRegression (build_model_2d.py:52-57, 33-42): [B,1,D3,H3,W3] -> [B,3H3,3W3].
    ``fast_exp``: hardware exp (the bf16 path)."""
    _require_cuda(cost)
    if cost.dim() != 5 or cost.shape[1] != 1:
        raise ValueError("cost must be [B, 1, D3, H3, W3]")
    cost = cost.contiguous()
    b, _, d3, h3, w3 = cost.shape
    disp = torch.empty((b, 3 * h3, 3 * w3), device=cost.device, dtype=torch.float32)
    rec = None if _probe is None else _probe_launch(
        "disparity_regression", 0.0, 4.0 * (cost.numel() + disp.numel()))
    check(_lib.load().lea_disparity_regression(cost.data_ptr(), disp.data_ptr(), b, d3, h3, w3,
                                               maxdisp, _lib.LEA_BF16 if fast_exp else LEA_F32,
                                               _stream()),
          "lea_disparity_regression")
    _probe_end(rec)
    return disp


# ------------------------------------------------------------------ bf16 path (c8)
# Activations: torch.bfloat16 [B, C/8, D, H, W, 8] ("c8": 8 channels per voxel word).

def _require_c8(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.bfloat16 or t.dim() != 6
                              or t.shape[-1] != 8):
            raise _lib.HipKernelError(
                f"bf16 path needs [B, C/8, D, H, W, 8] bfloat16 ROCm tensors, got {t.dtype} "
                f"{tuple(t.shape)} on {t.device}")


def _check_c8_view(t: torch.Tensor, name: str):
    b, cb, d, h, w, _ = t.shape
    if t.stride()[1:] != (d * h * w * 8, h * w * 8, w * 8, 8, 1):
        raise ValueError(f"{name}: c8 block slice with contiguous blocks required, strides {t.stride()}")
    return t.stride(0)


def c8_channels(t: torch.Tensor) -> int:
    return t.shape[1] * 8


def to_c8(x: torch.Tensor) -> torch.Tensor:
    """f32 [B, C, D, H, W] (or [B, C, H, W] as D = 1) -> bf16 c8."""
    _require_cuda(x)
    x5 = x.unsqueeze(2) if x.dim() == 4 else x
    b, c, d, h, w = x5.shape
    xbs = _check_volume_view(x5, "x")
    out = torch.empty((b, c // 8, d, h, w, 8), device=x.device, dtype=torch.bfloat16)
    rec = None if _probe is None else _probe_launch("to_c8_bf16", 0.0, 6.0 * out.numel())
    check(_lib.load().lea_to_c8_bf16(x5.data_ptr(), xbs, out.data_ptr(), out.stride(0), b, c,
                                     d * h * w, _stream()), "lea_to_c8_bf16")
    _probe_end(rec)
    return out


def from_c8(x: torch.Tensor) -> torch.Tensor:
    """bf16 c8 -> f32 [B, C, D, H, W]."""
    _require_c8(x)
    b, cb, d, h, w, _ = x.shape
    xbs = _check_c8_view(x, "x")
    out = torch.empty((b, cb * 8, d, h, w), device=x.device, dtype=torch.float32)
    check(_lib.load().lea_from_c8_bf16(x.data_ptr(), xbs, out.data_ptr(), out.stride(0), b, cb * 8,
                                       d * h * w, _stream()), "lea_from_c8_bf16")
    return out


def pack_conv_weight_bf16(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, k, k, k] f32 device weight -> packed bf16 fragments (bf16 engine)."""
    _require_cuda(w)
    w = w.detach().contiguous()
    cout, cin, k = w.shape[0], w.shape[1], w.shape[-1]
    lib = _lib.load()
    n = lib.lea_conv3d_packed_elems_bf16(cout, cin, k)
    if n == 0:
        raise ValueError(f"unsupported bf16 conv shape cout={cout} cin={cin} k={k}")
    packed = torch.empty(n, device=w.device, dtype=torch.bfloat16)
    check(lib.lea_conv3d_pack_weights_bf16(w.data_ptr(), packed.data_ptr(), cout, cin, k, _stream()),
          "lea_conv3d_pack_weights_bf16")
    return packed


def conv_kernel_name_bf16(b, cout, cin, d, h, w, k, costvolume=False):
    name = _lib.load().lea_conv3d_kernel_name_bf16(b, cout, cin, d, h, w, k, 1 if costvolume else 0)
    return name.decode() if name else None


def _pair_kernel_name_bf16(cb: int) -> str:
    """The LEA_PAIR_SUM launch's kernel (conv3d_bf16.hip run(): the split-wave kernel unless
    LEASTEREO_PAIR_SPLIT=0, the two-source D-streaming kernel otherwise) for the probe."""
    th = 8 if cb == 1 else 4
    split = os.environ.get("LEASTEREO_PAIR_SPLIT", "3")
    if split in ("1", "2") or (split == "3" and cb == 1):
        return f"conv_bf16_pair_kernel<{th}, {cb}, {'true' if split != '1' and cb == 1 else 'false'}>"
    return f"conv_bf16_stream_kernel<1, 1, {th}, {cb}, 2>"


def conv3d_bnrelu_bf16(x: torch.Tensor, packed: torch.Tensor, cout: int, k: int,
                       scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool = True,
                       out: torch.Tensor | None = None, accumulate: bool = False,
                       x2: torch.Tensor | None = None,
                       residual: torch.Tensor | None = None, pair_sum: bool = False) -> torch.Tensor:
    """conv3d_bnrelu at dtype bf16 on c8 tensors (out may be a block slice).  ``pair_sum``
    (LEA_PAIR_SUM, the D-streaming kernel): x's and x2's channels feed two ConvBRs whose
    activations are summed; ``packed`` = pack_conv_weight_bf16(W_a) then (W_b) (one K chunk
    each), scale / shift 2 * cout values."""
    _require_c8(x, x2, out, residual)
    _require_cuda(scale, shift)
    if pair_sum and (x2 is None or accumulate or residual is not None):
        raise ValueError("pair_sum takes two sources and no residual")
    b, cb, d, h, w, _ = x.shape
    xbs = _check_c8_view(x, "x")
    cin2, x2bs = 0, 0
    if x2 is not None:
        if x2.shape[0] != b or tuple(x2.shape[2:5]) != (d, h, w):
            raise ValueError("x2 must match x in batch and volume")
        cin2 = x2.shape[1] * 8
        x2bs = _check_c8_view(x2, "x2")
    shape = (b, cout // 8, d, h, w, 8)
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(shape, device=x.device, dtype=torch.bfloat16)
    if tuple(out.shape) != shape:
        raise ValueError(f"out shape {tuple(out.shape)} != {shape}")
    ybs = _check_c8_view(out, "out")
    if accumulate:
        rptr, rbs = out.data_ptr(), ybs
    elif residual is not None:
        if tuple(residual.shape) != shape:
            raise ValueError("residual shape mismatch")
        rptr, rbs = residual.data_ptr(), _check_c8_view(residual, "residual")
    else:
        rptr, rbs = None, 0
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0) | (LEA_PAIR_SUM if pair_sum else 0)
    rec = None if _probe is None else _probe_begin(
        b, cb * 8 + cin2, cout, d, h, w, k, rptr is not None, b * d * h * w, False,
        name=(_pair_kernel_name_bf16(cb) if pair_sum else
              conv_kernel_name_bf16(b, cout, cb * 8 + cin2, d, h, w, k)), esz=2)
    check(_lib.load().lea_conv3d_bnrelu_bf16(
        x.data_ptr(), xbs, x2.data_ptr() if x2 is not None else None, x2bs, cin2, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, rptr, rbs, out.data_ptr(), ybs, b,
        cb * 8 + cin2, cout, d, h, w, k, flags, _stream()), "lea_conv3d_bnrelu_bf16")
    _probe_end(rec)
    return out


def pair_sum_supported_bf16(x: torch.Tensor, x2: torch.Tensor, out: torch.Tensor) -> bool:
    """Whether conv3d_bnrelu_bf16(..., pair_sum=True) takes these c8 operands: two equal sources
    of one K chunk each (8 or 16 channels), cout <= 16, D >= 4 (the D-streaming kernel)."""
    if not (x.shape[1] == x2.shape[1] and x.shape[1] in (1, 2) and out.shape[1] * 8 <= 16
            and x.shape[2] >= 4 and tuple(x.shape[2:5]) == tuple(x2.shape[2:5])):
        return False
    # the library's own plan decides (a tuning override can take the shape off the
    # D-streaming kernel): ask it rather than fail mid-forward
    b, cb, d, h, w = (int(s) for s in x.shape[:5])
    return bool(_lib.load().lea_conv3d_bf16_pair_supported(b, cb * 8, int(out.shape[1]) * 8, d, h, w))


def conv1x1_resampled_bf16(x: torch.Tensor, size, packed: torch.Tensor, cout: int, scale, shift,
                           relu: bool = True, out: torch.Tensor | None = None) -> torch.Tensor:
    """ConvBR 1x1 of interp(x, size, align_corners=True) on c8 tensors, the resampled
    input never materialised (lea_conv1x1_resampled_bf16)."""
    _require_c8(x, out)
    _require_cuda(scale, shift)
    b, cb, di, hi, wi, _ = x.shape
    d, h, w = (int(t) for t in size)
    xbs = _check_c8_view(x, "x")
    shape = (b, cout // 8, d, h, w, 8)
    if out is None:
        out = torch.empty(shape, device=x.device, dtype=torch.bfloat16)
    if tuple(out.shape) != shape:
        raise ValueError(f"out shape {tuple(out.shape)} != {shape}")
    ybs = _check_c8_view(out, "out")
    name = "conv1x1_rs_c8_kernel"
    rec = _probe_begin(b, cb * 8, cout, d, h, w, 1, False, b * di * hi * wi, True, name=name, esz=2)
    check(_lib.load().lea_conv1x1_resampled_bf16(
        x.data_ptr(), xbs, di, hi, wi, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), ybs, b, cb * 8, cout, d, h,
        w, LEA_RELU if relu else 0, _stream()), "lea_conv1x1_resampled_bf16")
    _probe_end(rec)
    return out


def conv3d_bnrelu_costvolume_bf16(fl: torch.Tensor, fr: torch.Tensor, maxdisp: int,
                                  packed: torch.Tensor, cout: int, scale, shift,
                                  relu: bool = True) -> torch.Tensor:
    """conv3d_bnrelu_costvolume at bf16: fl/fr c8 feature maps [B, C/8, 1, H, W, 8]."""
    _require_c8(fl, fr)
    if fl.shape != fr.shape or fl.shape[2] != 1:
        raise ValueError("left/right c8 features must match and have D = 1")
    fbs = _check_c8_view(fl, "left")
    if _check_c8_view(fr, "right") != fbs:
        raise ValueError("left/right batch strides differ")
    b, cb, _, h, w, _ = fl.shape
    d3 = int(maxdisp / 3)
    out = torch.empty((b, cout // 8, d3, h, w, 8), device=fl.device, dtype=torch.bfloat16)
    rec = None if _probe is None else _probe_begin(
        b, 2 * cb * 8, cout, d3, h, w, 3, False, 0, False,
        name=conv_kernel_name_bf16(b, cout, 2 * cb * 8, d3, h, w, 3, True), esz=2)
    check(_lib.load().lea_conv3d_bnrelu_costvolume_bf16(
        fl.data_ptr(), fr.data_ptr(), fbs, packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), out.stride(0), b, cb * 8,
        cout, d3, h, w, LEA_RELU if relu else 0, _stream()), "lea_conv3d_bnrelu_costvolume_bf16")
    _probe_end(rec)
    return out


def resample_trilinear_bf16(x: torch.Tensor, size, align_corners: bool = True,
                            out: torch.Tensor | None = None, scale=None, shift=None,
                            relu: bool = False) -> torch.Tensor:
    """resample_trilinear on c8 tensors."""
    _require_c8(x, out)
    b, cb, di, hi, wi, _ = x.shape
    do, ho, wo = (int(s) for s in size)
    xbs = _check_c8_view(x, "x")
    if out is None:
        out = torch.empty((b, cb, do, ho, wo, 8), device=x.device, dtype=torch.bfloat16)
    if tuple(out.shape) != (b, cb, do, ho, wo, 8):
        raise ValueError("out shape mismatch")
    ybs = _check_c8_view(out, "out")
    rec = None if _probe is None else _probe_launch(
        "resample3d_c8", 0.0, 2.0 * b * cb * 8 * (di * hi * wi + do * ho * wo))
    check(_lib.load().lea_resample3d_trilinear_bf16(
        x.data_ptr(), xbs, out.data_ptr(), ybs, b, cb * 8, di, hi, wi, do, ho, wo,
        1 if align_corners else 0, scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, LEA_RELU if relu else 0, _stream()),
        "lea_resample3d_trilinear_bf16")
    _probe_end(rec)
    return out


def tapsum_upsample_bf16(q: torch.Tensor, cout: int, size, scale=None, shift=None,
                         relu: bool = False) -> torch.Tensor:
    """tapsum_upsample with q in c8 (27*cout channels padded to a multiple of 8) -> f32."""
    _require_c8(q)
    b, cb, di, hi, wi, _ = q.shape
    if cb * 8 < 27 * cout:
        raise ValueError(f"q has {cb * 8} channels, need 27*{cout}")
    qbs = _check_c8_view(q, "q")
    do, ho, wo = (int(s) for s in size)
    out = torch.empty((b, cout, do, ho, wo), device=q.device, dtype=torch.float32)
    lib = _lib.load()
    ws = torch.empty(lib.lea_tapsum_workspace_bytes(b, cout, hi, wi, do) // 4, device=q.device,
                     dtype=torch.float32)
    rec = None if _probe is None else _probe_launch(
        "tapsum_c8", 0.0, 2.0 * q.numel() + 4.0 * out.numel())
    check(lib.lea_tapsum_upsample(
        q.data_ptr(), qbs, out.data_ptr(), out.stride(0), b, cout, di, hi, wi, do, ho, wo,
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, LEA_RELU if relu else 0, ws.data_ptr(),
        _lib.LEA_BF16, _stream()), "lea_tapsum_upsample(bf16)")
    _probe_end(rec)
    return out


def pack_conv2d_weight_bf16(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, 3, 3] f32 device weight -> packed bf16 fragments (2D engine)."""
    _require_cuda(w)
    w = w.detach().contiguous()
    if w.dim() != 4 or tuple(w.shape[2:]) != (3, 3):
        raise ValueError(f"expected a [cout, cin, 3, 3] weight, got {tuple(w.shape)}")
    cout, cin = w.shape[:2]
    lib = _lib.load()
    n = lib.lea_conv2d_packed_elems_bf16(cout, cin)
    if n == 0:
        raise ValueError(f"unsupported bf16 conv2d shape cout={cout} cin={cin}")
    packed = torch.empty(n, device=w.device, dtype=torch.bfloat16)
    check(lib.lea_conv2d_pack_weights_bf16(w.data_ptr(), packed.data_ptr(), cout, cin, _stream()),
          "lea_conv2d_pack_weights_bf16")
    return packed


def conv2d_bnrelu_bf16(x: torch.Tensor, packed: torch.Tensor, cout: int, scale, shift,
                       relu: bool = True, out: torch.Tensor | None = None, accumulate: bool = False,
                       residual: torch.Tensor | None = None) -> torch.Tensor:
    """conv2d_bnrelu on c8 maps [B, C/8, 1, H, W, 8]."""
    _require_c8(x, out, residual)
    _require_cuda(scale, shift)
    b, cb, d, h, w, _ = x.shape
    if d != 1:
        raise ValueError("conv2d_bnrelu_bf16 takes D = 1 maps")
    xbs = _check_c8_view(x, "x")
    shape = (b, cout // 8, 1, h, w, 8)
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(shape, device=x.device, dtype=torch.bfloat16)
    if tuple(out.shape) != shape:
        raise ValueError(f"out shape {tuple(out.shape)} != {shape}")
    ybs = _check_c8_view(out, "out")
    if accumulate:
        rptr, rbs = out.data_ptr(), ybs
    elif residual is not None:
        if tuple(residual.shape) != shape:
            raise ValueError("residual shape mismatch")
        rptr, rbs = residual.data_ptr(), _check_c8_view(residual, "residual")
    else:
        rptr, rbs = None, 0
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0)
    rec = None if _probe is None else _probe_launch(
        "conv2d_bf16", 2.0 * b * h * w * cout * cb * 8 * 9,
        2.0 * b * h * w * (cb * 8 + cout * (2 if rptr is not None else 1)) + 18.0 * cout * cb * 8)
    check(_lib.load().lea_conv2d_bnrelu_bf16(
        x.data_ptr(), xbs, packed.data_ptr(), scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, rptr, rbs, out.data_ptr(), ybs, b, cb * 8,
        cout, h, w, flags, _stream()), "lea_conv2d_bnrelu_bf16")
    _probe_end(rec)
    return out


# ---- stem0 over the cost volume, factored through 2D maps (csrc/cv_stem.hip) ----

def cv_stem_split_weights(w: torch.Tensor):
    """stem0's [cout, 2C, 3, 3, 3] weight -> (wl [9 cout, C, 3, 3], wr [6 cout, C, 3, 3]),
    the 2D map weights of lea_cv_stem_split_weights."""
    _require_cuda(w)
    w = w.detach().contiguous()
    if w.dim() != 5 or tuple(w.shape[2:]) != (3, 3, 3) or w.shape[1] % 2:
        raise ValueError(f"expected a [cout, 2C, 3, 3, 3] weight, got {tuple(w.shape)}")
    cout, c = w.shape[0], w.shape[1] // 2
    wl = torch.empty((9 * cout, c, 3, 3), device=w.device, dtype=torch.float32)
    wr = torch.empty((6 * cout, c, 3, 3), device=w.device, dtype=torch.float32)
    check(_lib.load().lea_cv_stem_split_weights(w.data_ptr(), wl.data_ptr(), wr.data_ptr(), cout, c,
                                                _stream()), "lea_cv_stem_split_weights")
    return wl, wr


def cv_stem_supported(cout: int, d3: int, w: int, bf16: bool) -> bool:
    """Shapes lea_cv_stem_combine takes (f32 stores float4 rows; one plane has no
    interior to factor around)."""
    return d3 >= 2 and (cout % 8 == 0 if bf16 else w % 4 == 0)


def cv_stem_combine(lmaps: torch.Tensor, rmaps: torch.Tensor, cout: int, d3: int,
                    scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool = True,
                    name: str = "cv_stem_f32_kernel") -> torch.Tensor:
    """stem0's output from the 2D maps: lmaps [B, 9 cout, 1, H, W] / rmaps [B, 6 cout, 1, H, W]
    f32 -> [B, cout, D3, H, W] f32, or c8 maps -> c8 [B, cout/8, D3, H, W, 8] bf16."""
    c8 = lmaps.dtype == torch.bfloat16
    if c8:
        _require_c8(lmaps, rmaps)
        b, _, _, h, w, _ = lmaps.shape
        lbs, rbs = _check_c8_view(lmaps, "lmaps"), _check_c8_view(rmaps, "rmaps")
        if lmaps.shape[1] * 8 != 9 * cout or rmaps.shape[1] * 8 != 6 * cout:
            raise ValueError("cv_stem_combine: map channels must be 9 / 6 x cout")
        out = torch.empty((b, cout // 8, d3, h, w, 8), device=lmaps.device, dtype=torch.bfloat16)
        ybs = out.stride(0)
    else:
        _require_cuda(lmaps, rmaps)
        b, _, _, h, w = lmaps.shape
        lbs, rbs = _check_volume_view(lmaps, "lmaps"), _check_volume_view(rmaps, "rmaps")
        if lmaps.shape[1] != 9 * cout or rmaps.shape[1] != 6 * cout:
            raise ValueError("cv_stem_combine: map channels must be 9 / 6 x cout")
        out = torch.empty((b, cout, d3, h, w), device=lmaps.device, dtype=torch.float32)
        ybs = out.stride(0)
    _require_cuda(scale, shift)
    if tuple(rmaps.shape[0:1]) != (b,) or tuple(rmaps.shape[3:5]) != (h, w):
        raise ValueError("cv_stem_combine: left/right maps differ in batch or size")
    rec = None
    if _probe is not None and (_probe.names is None or name in _probe.names):
        # algorithmic bytes: the output write (the maps are L2/MALL-resident reads)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rec = (name, 0.0, float(out.numel() * out.element_size()), e0, e1, 0.0, (b, 0, cout, d3, h, w, 0))
    check(_lib.load().lea_cv_stem_combine(
        lmaps.data_ptr(), lbs, rmaps.data_ptr(), rbs,
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), ybs, b, cout, d3, h, w,
        LEA_RELU if relu else 0, _lib.LEA_BF16 if c8 else LEA_F32, _stream()), "lea_cv_stem_combine")
    if rec is not None:
        rec[4].record()
        _probe.records.append(rec)
    return out


# ---- host steps either side of forward ----

def standardize_crop_u8(left: torch.Tensor, right: torch.Tensor, crop_height: int, crop_width: int):
    """predict.py:162-184 (load_data) fused with :144-159 (test_transform) on the device.

    ``left``/``right``: uint8 [B, H, W, 3|4] (or [H, W, 3|4]) decoded images on the
    ROCm device.  Returns (left, right) float32 [B, 3, crop_height, crop_width]."""
    for t in (left, right):
        if not t.is_cuda or t.dtype != torch.uint8:
            raise _lib.HipKernelError(f"standardize_crop_u8 needs uint8 device images, got "
                                      f"{t.dtype} on {t.device}")
    if left.dim() == 3:
        left, right = left.unsqueeze(0), right.unsqueeze(0)
    if left.shape != right.shape or left.dim() != 4 or left.shape[-1] not in (3, 4):
        raise ValueError(f"left/right must both be [B, H, W, 3|4] uint8, got {tuple(left.shape)} "
                         f"and {tuple(right.shape)}")
    left, right = left.contiguous(), right.contiguous()
    b, h, w, ps = left.shape
    lib = _lib.load()
    ws = torch.empty(lib.lea_standardize_workspace_bytes(b), device=left.device, dtype=torch.uint8)
    out_l = torch.empty((b, 3, crop_height, crop_width), device=left.device, dtype=torch.float32)
    out_r = torch.empty_like(out_l)
    rc = lib.lea_standardize_crop_u8(left.data_ptr(), right.data_ptr(), b, h, w, ps,
                                     out_l.data_ptr(), out_r.data_ptr(), crop_height, crop_width,
                                     ws.data_ptr(), _stream())
    if rc == _lib.LEA_E_INVALID and b"test_transform" in lib.lea_last_error():
        raise ValueError(lib.lea_last_error().decode())
    check(rc, "lea_standardize_crop_u8")
    return out_l, out_r


METRIC_FIELDS = ("n_epe", "sum_abs", "n_valid", "n_correct3", "n_le_thr1", "n_le_thr2", "n_le_thr3")


def disparity_metrics(pred: torch.Tensor, gt: torch.Tensor, maxdisp: float, round_pred: bool = False,
                      z_shift: int = 0, thresholds=(1, 2, 3), correct_mask: bool = False):
    """Per-pair metric counts of evaluation.py:287-307 / utils/metrics.py:6-46 in
    one device pass.  pred/gt: float32 [B, H, W] (or [H, W]) on the ROCm device.
    Returns (counts float64 [B, 8] on the device, laid out as
    ``include/leastereo_hip.h`` lea_disparity_metrics documents, and the uint8
    3-px correct mask [B, H, W] or None)."""
    _require_cuda(pred, gt)
    if pred.dim() == 2:
        pred, gt = pred.unsqueeze(0), gt.unsqueeze(0)
    if pred.shape != gt.shape or pred.dim() != 3:
        raise ValueError(f"pred/gt must both be [B, H, W], got {tuple(pred.shape)} and {tuple(gt.shape)}")
    if len(thresholds) != 3:
        raise ValueError("three bad-pixel thresholds")
    pred, gt = pred.contiguous(), gt.contiguous()
    b, h, w = pred.shape
    lib = _lib.load()
    ws = torch.empty(lib.lea_disparity_metrics_workspace_bytes(b, h, w), device=pred.device,
                     dtype=torch.uint8)
    out = torch.empty((b, 8), device=pred.device, dtype=torch.float64)
    mask = torch.empty((b, h, w), device=pred.device, dtype=torch.uint8) if correct_mask else None
    check(lib.lea_disparity_metrics(pred.data_ptr(), h * w, gt.data_ptr(), h * w, b, h, w,
                                    float(maxdisp), int(bool(round_pred)), int(z_shift),
                                    *(int(t) for t in thresholds),
                                    mask.data_ptr() if mask is not None else None, out.data_ptr(),
                                    ws.data_ptr(), _stream()), "lea_disparity_metrics")
    return out, mask


# ---- Winograd F(2,3)-along-W 3x3x3 convs (csrc/conv3d_wino.hip), fp32 ----

def wino_eligible(cout: int, cin: int, k: int) -> bool:
    """Layers the Winograd engine takes: k = 3 and input channels in chunks of 4
    (couts <= 8 run depth-paired: the couts of two output planes in one 16-row tile)."""
    return k == 3 and cin % 4 == 0


# below this the direct engine's smaller tiles fill the chip better (A/B override:
# LEASTEREO_WINO_MIN_VOXELS)
WINO_MIN_VOXELS = int(os.environ.get("LEASTEREO_WINO_MIN_VOXELS", "200000"))
# ... except for 32-cout blocks on the one-barrier W x D tile down to this volume (r04
# planner audit, profiles/r04_planner_sweep.txt: the C2 L2 32->32 cells, 61 K voxels, 34.6 us
# on conv3d_wino2p_kernel vs 38.2 us direct; A/B override: LEASTEREO_WINO_SMALL32_MIN)
WINO_SMALL32_MIN = int(os.environ.get("LEASTEREO_WINO_SMALL32_MIN", "32768"))


def wino_preferred(b, cout, cin, d, h, w) -> bool:
    """Per-call engine choice for an eligible layer (tools/wino_sweep.py at config 2):
    Winograd wins on the large volumes when the output channels fill its 16/32/48-row
    blocks (stem0, stem1, conv1/2, the L1 cells and sibling groups, the 8->24 L0
    group); on the small L2 volumes only the 96-channel sibling groups gain, the
    32-channel cells take the pipelined W x D tile down to WINO_SMALL32_MIN voxels (r04)."""
    if b * d * h * w < WINO_MIN_VOXELS:
        # small volumes: only wide blocks amortise the tile; 32-cout blocks run the one-barrier
        # pipelined tile (more than two 4-channel chunks per depth pair)
        return cout % 32 == 0 and (cout >= 64 or (b * d * h * w >= WINO_SMALL32_MIN and cin > 8))
    return cout <= 8 or cout == 16 or cout == 24 or cout % 32 == 0 or cout % 48 == 0


def wino_mfma_scale(cout: int, name: str) -> float:
    """MFMA products issued per direct-convolution product: (F + 2) per 3F for the
    kernel's F (first template argument of ``name``), times the padding of cout to
    the engine's 16/32/48-row block.  The W x D engine (conv3d_wino2_kernel<Q, WC, MTE,
    ...>) issues 24 products per 72: 1/3, with couts padded to 16 WC MTE; the F(2,3) x F(2,3)
    tile (conv3d_wino22_kernel) 16 per 36: 4/9, couts padded to 16."""
    if name.startswith("conv3d_wino22_kernel"):  # F(2,3) x F(2,3): 16 per (2 x 2 outputs x 9 taps)
        return (-(-cout // 16) * 16) / cout * 4.0 / 9.0
    if name.startswith("conv3d_wino2p_kernel"):  # the one-barrier W x D tile: 32-cout blocks
        return (-(-cout // 32) * 32) / cout / 3.0
    if name.startswith("conv3d_wino44_kernel"):  # F(4,3) x F(4,3): 36 per (4 x 4 outputs x 9 taps)
        return (-(-cout // 32) * 32) / cout / 4.0
    if name.startswith("conv3d_wino2_kernel<"):
        _, wc, mte = (int(t) for t in name.split("<", 1)[1].split(",")[:3])
        cop = 16 * wc * mte
        return (-(-cout // cop) * cop) / cout / 3.0
    f = int(name.split("<", 1)[1].split(",", 1)[0])  # conv3d_wino_kernel<F, Q, MT, ...>
    if cout <= 8:  # depth-paired: 12 (plane, kh) steps per 9 taps, 16 rows = 8 couts x 2 planes
        return (f + 2) / (3.0 * f) * 12 / 9 * 8 / cout
    cop = 16 if cout <= 16 else (48 if cout % 32 != 0 and cout % 48 == 0 else 32)
    return (f + 2) / (3.0 * f) * (-(-cout // cop) * cop) / cout


@contextlib.contextmanager
def wino_depth_f2():
    """Run the enclosed Winograd convs of the pipelined kernel's layers on the F(4,3) x F(2,3)
    tile (lea_conv3d_wino44_set(0)) instead of the F(4,3) x F(4,3) one, then restore the
    process setting (LEASTEREO_WINO44, default 2).  The training path uses it: its gradient
    bars (tests/test_gpu_training.py) were calibrated on the F(2,3)-along-D numerics, and
    F(4,3) along D adds fp32 roundings that the backward chain amplifies (r06: a feature-net
    BN-weight gradient at 2.9e-3 of its scale against the 2e-3 bar).  Process-wide, like
    every tuning setter: not for concurrent use from several threads."""
    lib = _lib.load()
    check(lib.lea_conv3d_wino44_set(0), "lea_conv3d_wino44_set")
    try:
        yield
    finally:
        check(lib.lea_conv3d_wino44_set(int(os.environ.get("LEASTEREO_WINO44") or 2)), "lea_conv3d_wino44_set")


def wino_kernel_name(b, cout, d, h, w, costvolume=False, cin=0):
    name = _lib.load().lea_conv3d_wino_kernel_name(b, cin, cout, d, h, w, 1 if costvolume else 0)
    return name.decode() if name else None


def pack_conv_weight_wino(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, 3, 3, 3] fp32 device weight -> U = G g per kw row, the layout of
    lea_conv3d_bnrelu_wino."""
    _require_cuda(w)
    w = w.detach().contiguous()
    if w.dim() != 5 or tuple(w.shape[2:]) != (3, 3, 3):
        raise ValueError(f"expected a [cout, cin, 3, 3, 3] weight, got {tuple(w.shape)}")
    cout, cin = w.shape[0], w.shape[1]
    n = _lib.load().lea_conv3d_wino_packed_floats(cout, cin)
    if n == 0:
        raise ValueError(f"unsupported Winograd conv shape cout={cout} cin={cin}")
    packed = torch.empty(n, device=w.device, dtype=torch.float32)
    check(_lib.load().lea_conv3d_wino_pack_weights(w.data_ptr(), packed.data_ptr(), cout, cin,
                                                   _stream()), "lea_conv3d_wino_pack_weights")
    return packed


def pair_sum_supported(x: torch.Tensor, x2: torch.Tensor, out: torch.Tensor) -> bool:
    """Whether conv3d_bnrelu_wino(..., pair_sum=True) takes these operands: the F(2,3) x F(2,3)
    tile's rule (csrc/conv3d_wino22.hip wino22_ok) -- cout <= 32, W % 4 == 0, 16-byte aligned
    sources with batch strides of whole 16-byte words, 8-byte aligned output."""
    b, c, d, h, w = x.shape
    ok = out.shape[1] <= 32 and w % 4 == 0 and x2.shape[2:] == x.shape[2:] and x.shape[1] % 4 == 0
    for t, al in ((x, 16), (x2, 16), (out, 8)):
        ok = ok and t.data_ptr() % al == 0 and t.stride(0) % (al // 4) == 0 and \
            t.stride()[1:] == (d * h * w, h * w, w, 1)
    return bool(ok and 16 * d * h * w * 4 < 0xFFFFFF00)


def conv3d_bnrelu_wino(x: torch.Tensor, packed: torch.Tensor, cout: int,
                       scale: torch.Tensor | None, shift: torch.Tensor | None, relu: bool = True,
                       out: torch.Tensor | None = None, accumulate: bool = False,
                       x2: torch.Tensor | None = None,
                       residual: torch.Tensor | None = None, pair_sum: bool = False) -> torch.Tensor:
    """``conv3d_bnrelu`` (k = 3) on the Winograd engine: same semantics, weights
    packed by ``pack_conv_weight_wino``.  ``pair_sum`` (LEA_PAIR_SUM): x's and x2's channels
    feed two separate ConvBRs (the packed weight is [W_a | W_b] along cin, scale / shift
    2 * cout values) whose activations are summed -- a matching-cell step."""
    _require_cuda(x, x2, packed, scale, shift, out)
    if pair_sum and (x2 is None or accumulate or residual is not None):
        raise ValueError("pair_sum takes two sources and no residual")
    b, cin, d, h, w = x.shape
    xbs = _check_volume_view(x, "x")
    cin2, x2bs = 0, 0
    if x2 is not None:
        if x2.shape[0] != b or tuple(x2.shape[2:]) != (d, h, w):
            raise ValueError("x2 must match x in batch and volume")
        cin2 = x2.shape[1]
        x2bs = _check_volume_view(x2, "x2")
    out, ybs = _conv_out(x.shape, cout, (d, h, w), out, accumulate, x.device, x.dtype)
    rptr, rbs = _residual(out, accumulate, residual, ybs)
    flags = (LEA_RELU if relu else 0) | (LEA_RESIDUAL if rptr is not None else 0) | (LEA_PAIR_SUM if pair_sum else 0)
    rec = None
    if _probe is not None:  # (the kernel-name query only when a probe listens)
        name = "conv3d_wino22_kernel" if pair_sum else wino_kernel_name(b, cout, d, h, w, cin=cin + cin2)
        rec = _probe_begin(b, cin + cin2, cout, d, h, w, 3, rptr is not None, b * d * h * w, False,
                           name=name, mfma_scale=wino_mfma_scale(cout, name))
    check(_lib.load().lea_conv3d_bnrelu_wino(
        x.data_ptr(), xbs, x2.data_ptr() if x2 is not None else None, x2bs, cin2,
        packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None,
        rptr, rbs, out.data_ptr(), ybs, b, cin + cin2, cout, d, h, w, flags, LEA_F32, _stream()),
        "lea_conv3d_bnrelu_wino")
    _probe_end(rec)
    return out


def conv3d_bnrelu_costvolume_wino(fl: torch.Tensor, fr: torch.Tensor, maxdisp: int,
                                  packed: torch.Tensor, cout: int, scale: torch.Tensor | None,
                                  shift: torch.Tensor | None, relu: bool = True) -> torch.Tensor:
    """``conv3d_bnrelu_costvolume`` on the Winograd engine (the cost volume of
    LEAStereo.py:34-48 read in place, never materialised)."""
    _require_cuda(fl, fr, packed, scale, shift)
    if fl.shape != fr.shape or fl.dim() != 4:
        raise ValueError("left/right features must both be [B, C, H, W]")
    if fl.stride() != fr.stride() or fl.stride()[1:] != (fl.shape[2] * fl.shape[3], fl.shape[3], 1):
        raise ValueError("left/right features need contiguous C,H,W and equal strides")
    b, c, h, w = fl.shape
    d3 = int(maxdisp / 3)
    out = torch.empty((b, cout, d3, h, w), device=fl.device, dtype=fl.dtype)
    rec = None
    if _probe is not None:
        name = wino_kernel_name(b, cout, d3, h, w, True, cin=2 * c)
        rec = _probe_begin(b, 2 * c, cout, d3, h, w, 3, False, 0, False,
                           name=name, mfma_scale=wino_mfma_scale(cout, name))
    check(_lib.load().lea_conv3d_bnrelu_costvolume_wino(
        fl.data_ptr(), fr.data_ptr(), fl.stride(0), packed.data_ptr(),
        scale.data_ptr() if scale is not None else None,
        shift.data_ptr() if shift is not None else None, out.data_ptr(), out.stride(0), b, c, cout,
        d3, h, w, LEA_RELU if relu else 0, LEA_F32, _stream()), "lea_conv3d_bnrelu_costvolume_wino")
    _probe_end(rec)
    return out
