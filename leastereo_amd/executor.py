"""Cell-graph executors: run the searched networks on the HIP kernels.

``MatchingExecutor`` runs newMatching.forward (retrain/skip_model_3d.py:140-174),
``FeatureExecutor`` runs newFeature.forward (retrain/new_model_2d.py:140-165).
Both are prepared once per weight load (``NewMatching.executor()`` /
``NewFeature.executor()``): every ConvBR's weight is re-laid out for its kernel
and its BN folded into fp32 scale/shift.  ``run`` then issues only C-ABI launches
on the current stream (no host syncs), so a whole forward can be captured in a
HIP graph.

Memory plan per cell (skip_model_3d.py:41-75, new_model_2d.py:41-75): the cell
output ``cat([s1, s2, s3, s4])`` is allocated once and every producer writes its
channel slice directly (preprocess -> s1 slot, first DAG op -> s_k slot, second
DAG op accumulates into the same slot through the conv epilogue; a skip_connect
term enters as the epilogue's residual), so neither the ``cat`` nor the ``sum``
moves data.  Feature-net activations are [B, C, 1, H, W] views: a 2D map is the
one-plane case of the 3D kernels (1x1 convs, bilinear = trilinear on one plane),
and the 3x3 convs run on the 2D entry of the same MFMA engine.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import kernels
from .arch import scale_dimension


def _stacked(fl: torch.Tensor, fr: torch.Tensor) -> torch.Tensor:
    """[fl; fr] along the batch: a view when fr directly follows fl in one buffer (the
    forward's stacked feature batch, LEAStereo.forward), else a copy (torch.cat) -- the
    r05 C4 forward's two copyBuffer launches were this cat of adjacent views."""
    if (fl.is_contiguous() and fr.is_contiguous() and fl.shape == fr.shape and fl.dtype == fr.dtype
            and fl.device == fr.device
            and fr.data_ptr() == fl.data_ptr() + fl.numel() * fl.element_size()):
        return fl.as_strided((2 * fl.shape[0],) + tuple(fl.shape[1:]), fl.stride())
    return torch.cat((fl, fr), 0)


@dataclass
class ConvParams:
    packed: torch.Tensor      # packed weights ("s3": the raw [cout, cin, 3, 3] weight)
    scale: torch.Tensor | None
    shift: torch.Tensor | None
    cin: int
    cout: int
    k: int
    relu: bool
    kind: str = "3d"          # "3d" (k 1/3), "2d" (3x3 s1), "s3" (3x3 stride 3)
    wino: torch.Tensor | None = None  # Winograd-packed weight (f32 3D k=3 layers)


# f32 3x3x3 layers run on the Winograd F(2,3)-along-W engine (2/3 of the direct
# engine's MFMA work); LEASTEREO_WINOGRAD=0 keeps them on the direct engine.
WINOGRAD = os.environ.get("LEASTEREO_WINOGRAD", "1") != "0"
# stem0 over the cost volume through 2D maps (csrc/cv_stem.hip); LEASTEREO_CV_STEM=0
# runs the 3D conv on the in-place cost volume instead.
CV_STEM = os.environ.get("LEASTEREO_CV_STEM", "1") != "0"


def _conv_params(mod, w=None, folded=None):
    """ConvParams of a ConvBR (weights/BN may be overridden by stacked ones)."""
    w = mod.conv.weight if w is None else w
    scale, shift = mod.folded_bn() if folded is None else folded
    cout, cin, k = w.shape[0], w.shape[1], w.shape[-1]
    if w.dim() == 5:
        return ConvParams(kernels.pack_conv_weight(w), scale, shift, cin, cout, k, mod.relu)
    if k == 1:  # 1x1 Conv2d = 1x1x1 Conv3d on one plane
        return ConvParams(kernels.pack_conv_weight(w.reshape(cout, cin, 1, 1, 1)), scale, shift,
                          cin, cout, 1, mod.relu)
    if mod.stride == 3:
        return ConvParams(w.detach().contiguous(), scale, shift, cin, cout, 3, mod.relu, "s3")
    if mod.stride != 1 or mod.padding != 1:
        raise ValueError(f"unsupported Conv2d stride={mod.stride} padding={mod.padding}")
    return ConvParams(kernels.pack_conv2d_weight(w), scale, shift, cin, cout, 3, mod.relu, "2d")


class CellGraphExecutor:
    """Shared machinery: parameter packing, ConvBR dispatch, the searched cell."""

    # stage capture for the per-stage parity checks (tests): tap(name, f32 NCDHW copy) at
    # the stages oracle/torch_ref.matching_forward names; None (the default) costs nothing
    tap = None

    def _emit(self, name, t):
        if self.tap is not None:
            self.tap(name, self._as_f32(t))

    @staticmethod
    def _as_f32(t):
        return t.detach().clone()

    # fp32: a down-sampled s1 that the next cell reads again as its s0 (same tensor, same
    # size) feeds one stacked 1x1 conv for both cells (the bf16 executors memoise every
    # resample instead); LEASTEREO_SHARE_DOWNSAMPLE=0 keeps two passes
    SHARE_DOWNSAMPLE = os.environ.get("LEASTEREO_SHARE_DOWNSAMPLE", "1") != "0"
    # a three-op sibling group of 16-channel 3D ops (the L1 cells: 16 -> 48) as a 32-cout
    # launch on the pipelined W x D kernel plus a 16-cout one (r03: 66 + 43 us vs 124 us on
    # the 1-D 48-row engine); the f32 Winograd matching executor only.  Split as step 0's op
    # (head, 16 couts) + steps 1, 2 (the 32-cout group).  (r04: running op0 (s0 -> step 0)
    # on a side stream beside s1's preprocess and this group, the head accumulating after
    # the join, measured 140.6 -> 138.1 pairs/s at C2 in graph replay: not kept)
    SPLIT_S1_GROUP48 = False
    # the feature net's 2D cells: their two conv ops on s0 (op0 -> step 0 with the skip term as
    # its residual, op4 -> step 2 before op5 accumulates) as one launch writing two slots
    # (lea_conv2d_bnrelu_pair; r04).  The f32 feature executor only; LEASTEREO_PAIR_S0=0: two launches
    PAIR_S0 = False
    # a 3D cell whose every step sums two conv ops (the shipped matching genotype): each step
    # as ONE LEA_PAIR_SUM launch, y = relu(BN_a(conv_a(s_ja))) + relu(BN_b(conv_b(s_jb))),
    # reading the two states and writing the step's slot once (r05) -- instead of the s1
    # sibling group plus an accumulating launch per remaining op (a read-modify-write of the
    # slot each).  Executors whose engine takes LEA_PAIR_SUM set it
    PAIR_STEPS = False
    # the cells' channel counts that take the pair launches (A/B: LEASTEREO_PAIR_C=16,32 ...)
    PAIR_C = tuple(int(c) for c in os.environ.get("LEASTEREO_PAIR_C", "8,16,32").split(",") if c)

    def __init__(self, net):
        from .model import ConvBR
        self.m = net
        self.p = {}
        with torch.no_grad():
            for name, mod in net.named_modules():
                if isinstance(mod, ConvBR):
                    self.p[name] = _conv_params(mod)
            # Sibling ops: the DAG ops that read s1 (one per step: ops 1, 2, 4 of the
            # matching genotype) write consecutive cat slots, so they run as ONE conv
            # with cout = n*C over channels [.., ..) of the cell output (their weights
            # and folded BN stacked along cout).  The remaining ops accumulate.
            self.s1_group = {}
            self.s1_split = set()
            for i, cell in enumerate(net.cells):
                group = []
                for k, terms in enumerate(cell.plan):
                    for op, j in terms:
                        if j == 1 and cell.op_kinds[op] == "conv":
                            group.append((k, op))
                            break
                first_cat_state = 2 + cell.steps - cell.block_multiplier
                steps = [k for k, _ in group]
                if (len(group) < 2 or steps != list(range(steps[0], steps[0] + len(steps)))
                        or 2 + steps[0] < first_cat_state):
                    continue
                mods = [cell._ops[op] for _, op in group]
                split = (self.SPLIT_S1_GROUP48 and WINOGRAD and len(mods) == 3 and cell.c_out == 16
                         and mods[0].conv.weight.dim() == 5 and mods[0].conv.weight.shape[2] == 3)
                for key, part in ((("s1_group_head", mods[:1]), ("s1_group", mods[1:])) if split
                                  else (("s1_group", mods),)):
                    w = torch.cat([m.conv.weight for m in part], 0)
                    folded = [m.folded_bn() for m in part]
                    scale = torch.cat([f[0] for f in folded]).contiguous()
                    shift = torch.cat([f[1] for f in folded]).contiguous()
                    self.p[f"cells.{i}.{key}"] = _conv_params(part[0], w, (scale, shift))
                self.s1_group[i] = group
                if split:
                    self.s1_split.add(i)
            self.s0_pair = {}
            for i, cell in enumerate(net.cells) if self.PAIR_S0 else ():
                pair = [(k, op) for k, terms in enumerate(cell.plan) for op, j in terms
                        if j == 0 and cell.op_kinds[op] == "conv"]
                first_cat_state = 2 + cell.steps - cell.block_multiplier
                if (len(pair) != 2 or getattr(cell, "dims", 3) != 2 or 2 + pair[0][0] < first_cat_state
                        or cell.c_out % 8 or 2 * cell.c_out > 32):
                    continue
                (k0, op0), (k1, op1) = pair
                m0, m1 = cell._ops[op0], cell._ops[op1]
                other = [(o, j) for o, j in cell.plan[k1] if o != op1]
                # the s1 sibling group writes its steps' slots without accumulating, after
                # the pair: a step both of them write would lose the pair's term
                if {k for k, _ in self.s1_group.get(i, [])} & {k0, k1}:
                    continue
                # op1 writes its step first (the other term a conv that accumulates after it)
                if (m0.relu != m1.relu or m0.conv.weight.dim() != 4 or m0.conv.weight.shape[-1] != 3
                        or m0.stride != 1 or m1.stride != 1 or cell.plan[k1][0][0] != op1
                        or not other or cell.op_kinds[other[0][0]] != "conv"):
                    continue
                w = torch.cat([m0.conv.weight, m1.conv.weight], 0)
                folded = [m0.folded_bn(), m1.folded_bn()]
                self.p[f"cells.{i}.s0_pair"] = _conv_params(
                    m0, w, (torch.cat([f[0] for f in folded]).contiguous(),
                            torch.cat([f[1] for f in folded]).contiguous()))
                self.s0_pair[i] = pair
            self.pair_steps = {}
            for i, cell in enumerate(net.cells) if self.PAIR_STEPS else ():
                terms = [[(op, j) for op, j in t] for t in cell.plan]
                if (getattr(cell, "dims", 3) != 3 or not terms or cell.c_out not in self.PAIR_C
                        or any(len(t) != 2 or any(cell.op_kinds[op] != "conv" for op, _ in t) for t in terms)):
                    continue
                mods = [[cell._ops[op] for op, _ in t] for t in terms]
                if any(m.conv.weight.shape[-1] != 3 or not m.relu for ms in mods for m in ms):
                    continue
                for k, (ma, mb) in enumerate(mods):
                    folded = [ma.folded_bn(), mb.folded_bn()]
                    self.p[f"cells.{i}.pair{k}"] = self._pair_params(
                        ma, torch.cat([ma.conv.weight, mb.conv.weight], 1),
                        (torch.cat([f[0] for f in folded]).contiguous(),
                         torch.cat([f[1] for f in folded]).contiguous()))
                self.pair_steps[i] = terms
            # a cell that resamples s1, followed by a same-level cell: the next cell's s0
            # is this s1 (Cell.forward returns prev_input, skip_model_3d.py:75) at the same
            # size, so both 1x1 convs run as one stacked conv over one read of it (down:
            # interpolation in the conv's staging; up: one low-resolution conv and one
            # up-sampling with the stacked BN)
            cells = list(net.cells)
            for i, (cell, nxt) in enumerate(zip(cells, cells[1:])):
                if (self.SHARE_DOWNSAMPLE and cell.downup_sample != 0 and nxt.downup_sample == 0
                        and nxt.c_out == cell.c_out and 2 + cell.steps - cell.block_multiplier == 1
                        and cell.preprocess.conv.weight.shape[1] == nxt.pre_preprocess.conv.weight.shape[1]
                        # the next cell applies pre_preprocess only when s0's channels differ
                        # from its C_out (skip_model_3d.py:52); the memo path assumes it does
                        and cell.preprocess.conv.weight.shape[1] != nxt.c_out):
                    mods = [nxt.pre_preprocess, cell.preprocess]
                    folded = [m.folded_bn() for m in mods]
                    self.p[f"cells.{i}.share"] = _conv_params(
                        mods[0], torch.cat([m.conv.weight for m in mods], 0),
                        (torch.cat([f[0] for f in folded]).contiguous(),
                         torch.cat([f[1] for f in folded]).contiguous()))

    def conv(self, name, x, out=None, accumulate=False, x2=None, size=None, residual=None):
        """ConvBR ``name`` on x (or cat(x, x2)); with ``size`` != x's volume the input
        is trilinearly resampled (align_corners=True) inside the conv."""
        p = self.p[name]
        cin = x.shape[1] + (x2.shape[1] if x2 is not None else 0)
        if cin != p.cin:
            raise ValueError(f"{name}: expected {p.cin} input channels, got {cin}")
        resized = size is not None and tuple(size) != tuple(x.shape[2:5])
        if p.kind == "s3":
            return kernels.conv2d_s3_bnrelu(x, p.packed, p.scale, p.shift, p.relu)
        if p.kind == "2d":
            if resized or x2 is not None:
                raise ValueError(f"{name}: 2D 3x3 conv takes one input at its own size")
            return kernels.conv2d_bnrelu(x, p.packed, p.cout, p.scale, p.shift, p.relu, out,
                                         accumulate, residual)
        if resized:
            if x2 is not None or residual is not None:
                raise ValueError("resampled conv takes one input and no residual")
            up = all(int(o) >= int(i) for o, i in zip(size, x.shape[2:]))
            if p.k == 1 and up and not accumulate:
                # interp and the 1x1 conv commute: conv at the low resolution, then
                # resample the narrow result with the BN/ReLU epilogue into `out`
                z = kernels.conv3d_bnrelu(x, p.packed, p.cout, 1, None, None, relu=False)
                return kernels.resample_trilinear(z, size, True, out, p.scale, p.shift, p.relu)
            return kernels.conv3d_bnrelu_resampled(x, size, p.packed, p.cout, p.k, p.scale,
                                                   p.shift, p.relu, out, accumulate)
        if p.wino is not None and kernels.wino_preferred(x.shape[0], p.cout, p.cin, *x.shape[2:5]):
            return kernels.conv3d_bnrelu_wino(x, p.wino, p.cout, p.scale, p.shift, p.relu, out,
                                              accumulate, x2, residual)
        return kernels.conv3d_bnrelu(x, p.packed, p.cout, p.k, p.scale, p.shift, p.relu, out,
                                     accumulate, x2, residual)

    def _pair_params(self, mod, w, folded):
        """ConvParams of a LEA_PAIR_SUM step: [W_a | W_b] along cin, BN (a's, then b's)."""
        p = _conv_params(mod, w, folded)
        p.cout = w.shape[0]
        return p

    def _pair_ok(self, x, x2, out):
        """The f32 pair launch's shape / alignment rule (lea_conv3d_bnrelu_wino, LEA_PAIR_SUM:
        the F(2,3) x F(2,3) tile, conv3d_wino22.hip)."""
        return kernels.pair_sum_supported(x, x2, out)

    def pair_conv(self, name, x, x2, out):
        p = self.p[name]
        return kernels.conv3d_bnrelu_wino(x, p.wino, p.cout, p.scale, p.shift, True, out, x2=x2, pair_sum=True)

    def _use_winograd(self):
        """Pack the eligible 3x3x3 layers for the Winograd engine (f32 executors)."""
        if not WINOGRAD:
            return
        with torch.no_grad():
            for name, p in self.p.items():
                if p.kind != "3d" or not kernels.wino_eligible(p.cout, p.cin, p.k):
                    continue
                if ".pair" in name:
                    i, k = int(name.split(".")[1]), int(name.rsplit("pair", 1)[1])
                    cell = self.m.cells[i]
                    w = torch.cat([cell._ops[op].conv.weight for op, _ in self.pair_steps[i][k]], 1)
                elif name.endswith("s1_group") or name.endswith("s1_group_head"):
                    i = int(name.split(".")[1])
                    mods = [self.m.cells[i]._ops[op] for _, op in self.s1_group[i]]
                    if i in self.s1_split:
                        mods = mods[:1] if name.endswith("_head") else mods[1:]
                    w = torch.cat([m.conv.weight for m in mods], 0)
                else:
                    w = self.m.get_submodule(name).conv.weight
                p.wino = kernels.pack_conv_weight_wino(w)

    # activation layout hooks (f32 NCDHW here; the bf16 executor overrides them)
    def _empty(self, b, c, size, like):
        return torch.empty((b, c) + tuple(size), device=like.device, dtype=like.dtype)

    @staticmethod
    def _channels(t, c0, c1):
        return t[:, c0:c1]

    @staticmethod
    def _nchannels(t):
        return t.shape[1]

    @staticmethod
    def _volume(t):
        return tuple(t.shape[2:5])

    @staticmethod
    def _resample(x, size):
        return kernels.resample_trilinear(x, size)

    def cell(self, i, s0, s1):
        """Cell.forward (skip_model_3d.py:41-75 / new_model_2d.py:41-75).  The level
        change of s1 (:44-48) and the size match of s0 (:49-51) are fused into the
        1x1 preprocess convs (:52-53) that consume them."""
        cell = self.m.cells[i]
        c = cell.c_out
        prev_input = s1
        size = self._volume(s1)
        if cell.downup_sample != 0:
            sc = 0.5 if cell.downup_sample < 0 else 2
            # the D axis of a 2D map stays 1 (bilinear on H, W only)
            size = tuple(n if (cell.dims == 2 and ax == 0) else scale_dimension(n, sc)
                         for ax, n in enumerate(size))
        b = s1.shape[0]
        bm = cell.block_multiplier
        n_states = 2 + cell.steps
        memo, self._share_memo = getattr(self, "_share_memo", None), None
        share = f"cells.{i}.share" in self.p
        if share:
            # this cell's s1 preprocess and the next cell's s0 pre_preprocess read the
            # same down-sampled tensor: one stacked 1x1 conv writes [next s0 | this s1]
            # into the channels just before and at the start of this cell's output
            big = self._empty(b, c + bm * c, size, s1)
            out = self._channels(big, c, c + bm * c)
        else:
            out = self._empty(b, bm * c, size, s1)
        slot = {idx: self._channels(out, k * c, (k + 1) * c)
                for k, idx in enumerate(range(n_states - bm, n_states))}
        group = self.s1_group.get(i, [])
        if memo is not None and memo[0] is s0 and memo[1] == size:
            s0 = memo[2]  # computed by the previous cell's stacked conv
            if 0 in slot:
                slot[0].copy_(s0)
        elif self._nchannels(s0) != c:
            s0 = self.conv(f"cells.{i}.pre_preprocess", s0, out=slot.get(0), size=size)
        else:
            if self._volume(s0) != size:
                s0 = self._resample(s0, size)
            if 0 in slot:
                slot[0].copy_(s0)
        if share:
            self.conv(f"cells.{i}.share", s1, out=self._channels(big, 0, 2 * c), size=size)
            self._share_memo = (prev_input, size, self._channels(big, 0, c))
            s1 = self._channels(big, c, 2 * c)
        else:
            s1 = self.conv(f"cells.{i}.preprocess", s1, out=slot.get(1), size=size)
        states = [s0, s1]
        pairs = self.pair_steps.get(i)
        if pairs is not None:
            dsts = [slot.get(2 + k) for k in range(len(pairs))]
            if all(d is not None for d in dsts) and all(
                    self._pair_ok(states[t[0][1]] if t[0][1] < 2 else dsts[t[0][1] - 2],
                                  states[t[1][1]] if t[1][1] < 2 else dsts[t[1][1] - 2], dsts[k])
                    for k, t in enumerate(pairs)):
                for k, ((_, ja), (_, jb)) in enumerate(pairs):
                    self.pair_conv(f"cells.{i}.pair{k}", states[ja], states[jb], dsts[k])
                    states.append(dsts[k])
                return prev_input, out
        written = set()
        done = set(group)
        consumed = set()  # steps whose skip term went in as an epilogue residual already
        pair = self.s0_pair.get(i)
        if pair is not None and self._nchannels(s0) == c and self._volume(s0) == size:
            (k0, op0), (k1, op1) = pair
            skips0 = [states[j] for o, j in cell.plan[k0] if cell.op_kinds[o] != "conv"]
            p = self.p[f"cells.{i}.s0_pair"]
            kernels.conv2d_bnrelu_pair(s0, p.packed, c, 2 * c, p.scale, p.shift, p.relu,
                                       slot[2 + k0], slot[2 + k1], skips0[-1] if skips0 else None)
            done |= {(k0, op0), (k1, op1)}
            written |= {k0, k1}
            if skips0:
                consumed.add(k0)
        if group:  # ops on s1 of every step, one launch, straight into their slots
            k0 = 2 + group[0][0] - (n_states - bm)
            if i in self.s1_split:
                self.conv(f"cells.{i}.s1_group", s1, out=self._channels(out, (k0 + 1) * c, (k0 + 3) * c))
                self.conv(f"cells.{i}.s1_group_head", s1, out=self._channels(out, k0 * c, (k0 + 1) * c))
            else:
                self.conv(f"cells.{i}.s1_group", s1, out=self._channels(out, k0 * c, (k0 + len(group)) * c))
            written |= {k for k, _ in group}
        for step, terms in enumerate(cell.plan):
            dst = slot.get(len(states))
            if dst is None:
                dst = self._empty(b, c, size, s1)
            skips = [states[j] for k, j in terms if cell.op_kinds[k] != "conv"]
            if step in consumed:
                skips.pop()
            for k, j in terms:
                if (step, k) in done or cell.op_kinds[k] != "conv":
                    continue
                residual = None
                if step not in written and skips:  # skip_connect term -> epilogue residual
                    residual = skips.pop()
                self.conv(f"cells.{i}._ops.{k}", states[j], out=dst, accumulate=step in written,
                          residual=residual)
                written.add(step)
            for t in skips:
                if step in written:
                    dst.add_(t)
                else:
                    dst.copy_(t)
                written.add(step)
            states.append(dst)
        return prev_input, out


class MatchingExecutor(CellGraphExecutor):
    SPLIT_S1_GROUP48 = os.environ.get("LEASTEREO_SPLIT_GROUP48", "1") != "0"
    # the matching cells' steps as LEA_PAIR_SUM launches (LEASTEREO_PAIR_STEPS=0: the s1 group
    # + accumulating launches); the f32 pair runs on the Winograd F(2,3) x F(2,3) tile
    PAIR_STEPS = WINOGRAD and os.environ.get("LEASTEREO_PAIR_STEPS", "0") != "0"

    def run(self, x):
        """newMatching.forward (skip_model_3d.py:140-174): [B,64,D3,H3,W3] -> [B,1,D3,H3,W3]."""
        return self._from_stem0(self.conv("stem0", x))

    def run_features(self, fl, fr, maxdisp):
        """build_cost_volume + newMatching.forward (LEAStereo.py:34-50) with the cost
        volume read in place by stem0's conv (never materialised)."""
        p = self.p["stem0"]
        if fl.shape[1] * 2 != p.cin:
            raise ValueError(f"stem0 expects {p.cin} cost-volume channels, got 2*{fl.shape[1]}")
        d3 = int(maxdisp / 3)
        if self.cv is not None and kernels.cv_stem_supported(p.cout, d3, fl.shape[3], False):
            return self._from_stem0(self._cv_stem(fl.unsqueeze(2), fr.unsqueeze(2), d3))
        if p.wino is not None and kernels.wino_preferred(fl.shape[0], p.cout, p.cin, int(maxdisp / 3),
                                                         *fl.shape[2:4]):
            stem0 = kernels.conv3d_bnrelu_costvolume_wino(fl, fr, maxdisp, p.wino, p.cout, p.scale,
                                                          p.shift, p.relu)
        else:
            stem0 = kernels.conv3d_bnrelu_costvolume(fl, fr, maxdisp, p.packed, p.cout, p.scale,
                                                     p.shift, p.relu)
        return self._from_stem0(stem0)

    def _cv_stem(self, fl5, fr5, d3):
        """stem0 = ConvBR3d(cost volume) (LEAStereo.py:34-48, skip_model_3d.py:141) as
        2D maps of each feature map + lea_cv_stem_combine (csrc/cv_stem.hip)."""
        p, (wl, wr) = self.p["stem0"], self.cv
        lm = kernels.conv2d_bnrelu(fl5, wl, 9 * p.cout, None, None, relu=False)
        rm = kernels.conv2d_bnrelu(fr5, wr, 6 * p.cout, None, None, relu=False)
        return kernels.cv_stem_combine(lm, rm, p.cout, d3, p.scale, p.shift, p.relu)

    def _cv_stem_pack(self, wl, wr):
        return kernels.pack_conv2d_weight(wl), kernels.pack_conv2d_weight(wr)

    def _from_stem0(self, stem0):
        out = self._matching_body(stem0)
        if self.tap is not None:  # the head's output is f32 NCDHW in every executor
            self.tap("matching", out.detach().clone())
        return out

    def _matching_body(self, stem0):
        d, h, w = self._volume(stem0)
        self._emit("stem0", stem0)
        stem1 = self.conv("stem1", stem0)
        self._emit("stem1", stem1)
        outs = []
        prev = (stem0, stem1)
        n = len(self.m.cells)
        for i in range(n):
            if i == 5 and n == 12:   # :150-151, cat read in place by the conv
                fused = self.conv("conv1", outs[1][1], x2=outs[4][1])
                self._emit("conv1", fused)
                prev = (outs[4][0], fused)
            elif i == 9 and n == 12:  # :155-156
                fused = self.conv("conv2", outs[4][1], x2=outs[8][1])
                self._emit("conv2", fused)
                prev = (outs[8][0], fused)
            o = self.cell(i, prev[0], prev[1])
            self._emit(f"cell{i}", o[1])
            outs.append(o)
            prev = o
        last = outs[-1][1]
        lh = self._volume(last)[1]
        full, half, quarter = (d, h, w), (d // 2, h // 2, w // 2), (d // 4, h // 4, w // 4)
        # head (:161-173): the 1x1 Upsample pairs run commuted (see conv()); the final
        # Upsample + last_3 run as per-tap partial sums at the low resolution, then one
        # 27-sample interpolating sum per output voxel (no full-resolution 32-ch tensor)
        if lh == h:
            return self._last3_same_size(last)
        if lh == h // 2:
            y = self.conv("last_6", last)
        elif lh == h // 4:
            y = self.conv("last_6", self.conv("last_12", last), size=half)
        elif lh == h // 8:
            y = self.conv("last_12", self.conv("last_24", last), size=quarter)
            y = self.conv("last_6", y, size=half)
        else:
            raise ValueError(f"matching-net output size {tuple(last.shape[2:])} has no head")
        p3 = self.p["last_3"]
        q = self.conv("last_3.taps", y)
        return self._tapsum(q, p3, full)

    @staticmethod
    def _tapsum(q, p3, full):
        return kernels.tapsum_upsample(q, p3.cout, full, p3.scale, p3.shift, p3.relu)

    def _last3_same_size(self, last):
        return self.conv("last_3", last)

    def __init__(self, matching):
        super().__init__(matching)
        with torch.no_grad():
            # Head: last_3(Upsample(y)) = sum over taps of upsampled per-tap partial
            # sums (lea_tapsum_upsample); the taps run as a 1x1 conv with 27*cout outputs.
            last3 = matching.last_3.conv.weight
            co, ci = last3.shape[:2]
            taps = last3.permute(0, 2, 3, 4, 1).reshape(co * 27, ci, 1, 1, 1)
            self.p["last_3.taps"] = ConvParams(kernels.pack_conv_weight(taps), None, None,
                                               ci, co * 27, 1, False)
            self.cv = None
            if CV_STEM:
                self.cv = self._cv_stem_pack(*kernels.cv_stem_split_weights(matching.stem0.conv.weight))
        self._use_winograd()


class MatchingExecutorDirect(MatchingExecutor):
    """newMatching.forward on the direct implicit-GEMM engine only: stem0 reads the
    cost volume in place (no factored 2D maps) and no layer runs Winograd.  An
    independent algorithm for the same f32 arithmetic, used by bench.py as the
    per-pair cross-check of every rank's shard (precision "f32_direct")."""

    SPLIT_S1_GROUP48 = False
    PAIR_STEPS = False

    def __init__(self, matching):
        super().__init__(matching)
        self.cv = None

    def _use_winograd(self):
        """Direct engine only."""


class FeatureExecutor(CellGraphExecutor):
    # stems 0 and 1 as one kernel (csrc/feature_stem.hip); LEASTEREO_FEATURE_STEM=0 runs
    # them as two convs
    FUSED_STEM = os.environ.get("LEASTEREO_FEATURE_STEM", "1") != "0"
    PAIR_S0 = os.environ.get("LEASTEREO_PAIR_S0", "1") != "0"

    def _stems(self, x, c8=False, x2=None):
        """new_model_2d.py:93-94 (stem1(stem0(x))), fused where the kernel is instantiated;
        with x2 the images of x then x2 as one batch (the fused stem reads both sources,
        no concatenated copy)."""
        p0, p1 = self.p["stem0"], self.p["stem1"]
        if (self.FUSED_STEM and p0.relu and p1.relu and (p0.cin, p0.cout, p1.cout) == (3, 16, 32)
                and p1.kind == "s3"):
            return kernels.feature_stem(x, self.m.stem0.conv.weight, p0.scale, p0.shift, p1.packed,
                                        p1.scale, p1.shift, c8, x2)
        if x2 is not None:
            x = torch.cat((x, x2), 0)
        stem1 = self.conv("stem1", self.conv("stem0", x.unsqueeze(2)))
        return kernels.to_c8(stem1) if c8 else stem1

    def run(self, x, x2=None):
        """newFeature.forward (new_model_2d.py:140-165): [N,3,H,W] -> [N,32,H/3,W/3]
        (with x2: the stacked features of x then x2)."""
        stem1 = self._stems(x, x2=x2)
        stem2 = self.conv("stem2", stem1)
        out = (stem1, stem2)
        for i in range(len(self.m.cells)):
            out = self.cell(i, out[0], out[1])
        last = out[-1]
        h, w = stem2.shape[3:]
        lh = last.shape[3]
        full, half, quarter = (1, h, w), (1, h // 2, w // 2), (1, h // 4, w // 4)
        # head (:156-163): ConvBR at the low level, then nn.Upsample; a ConvBR after an
        # Upsample reads it through conv(size=...) (interpolation fused/commuted)
        if lh == h:
            y = last
        elif lh == h // 2:
            y = kernels.resample_trilinear(self.conv("last_6", last), full)
        elif lh == h // 4:
            y = self.conv("last_6", self.conv("last_12", last), size=half)
            y = kernels.resample_trilinear(y, full)
        elif lh == h // 8:
            y = self.conv("last_12", self.conv("last_24", last), size=quarter)
            y = kernels.resample_trilinear(self.conv("last_6", y, size=half), full)
        else:
            # the reference raises UnboundLocalError here (new_model_2d.py:156-165)
            raise ValueError(f"feature size {tuple(x.shape[2:])} is not legal for the feature net")
        return self.conv("last_3", y).squeeze(2)


class _C8Layout:
    """Activation-layout hooks of the bf16 executors: c8 tensors
    ([B, C/8, D, H, W, 8] bfloat16), channel slices on block boundaries."""

    # down-sampling 1x1 convs read their input through the interpolating gather-GEMM
    # (lea_conv1x1_resampled_bf16), so the shared-preprocess stacking applies as in fp32
    # (LEASTEREO_BF16_FUSED_RS=0: materialise + memoise the resampled tensor instead)
    FUSED_RS = os.environ.get("LEASTEREO_BF16_FUSED_RS", "1") != "0"
    SHARE_DOWNSAMPLE = FUSED_RS and CellGraphExecutor.SHARE_DOWNSAMPLE

    def _empty(self, b, c, size, like):
        return torch.empty((b, c // 8) + tuple(size) + (8,), device=like.device, dtype=torch.bfloat16)

    @staticmethod
    def _as_f32(t):
        return kernels.from_c8(t)

    @staticmethod
    def _channels(t, c0, c1):
        return t[:, c0 // 8:c1 // 8]

    @staticmethod
    def _nchannels(t):
        return t.shape[1] * 8

    @staticmethod
    def _resample(x, size):
        return kernels.resample_trilinear_bf16(x, size)

    @staticmethod
    def _share_weight(net, name):
        """The stacked 1x1 weight of cells.{i}.share: [next cell's pre_preprocess ; this
        cell's preprocess] (CellGraphExecutor.__init__)."""
        i = int(name.split(".")[1])
        return torch.cat([net.cells[i + 1].pre_preprocess.conv.weight, net.cells[i].preprocess.conv.weight], 0)

    def _downsampled(self, x, size):
        """Materialised trilinear resample of a c8 tensor, memoised for one reuse: cell i
        resizes its s1 (skip_model_3d.py:44-48) and cell i+1 resizes the same raw tensor
        as its s0 to the same size (:49-51) -- stem1 L0->L1, cell1's output and conv1's
        L1->L2.  The memo holds the source itself (no address reuse while cached) and
        is dropped at the end of every forward (_fresh)."""
        memo = getattr(self, "_rs_memo", None)
        if memo is not None and memo[0] is x and memo[1] == tuple(size):
            return memo[2]
        y = kernels.resample_trilinear_bf16(x, size)
        self._rs_memo = (x, tuple(size), y)
        return y

    def _fresh(self):
        self._rs_memo = None

    def _conv_c8(self, name, x, out=None, accumulate=False, x2=None, size=None, residual=None):
        p = self.p[name]
        cin = (x.shape[1] + (x2.shape[1] if x2 is not None else 0)) * 8
        if cin != p.cin:
            raise ValueError(f"{name}: expected {p.cin} input channels, got {cin}")
        if size is not None and tuple(size) != tuple(x.shape[2:5]):
            if x2 is not None or residual is not None or accumulate:
                raise ValueError("resampled conv takes one input and no residual")
            up = all(int(o) >= int(i) for o, i in zip(size, x.shape[2:5]))
            if p.k == 1 and up:  # commuted: 1x1 at the low resolution, resample + BN/ReLU
                z = kernels.conv3d_bnrelu_bf16(x, p.packed, p.cout, 1, None, None, relu=False)
                return kernels.resample_trilinear_bf16(z, size, True, out, p.scale, p.shift, p.relu)
            if (self.FUSED_RS and p.k == 1 and p.kind == "bf16" and p.cin % 32 == 0 and p.cin <= 128
                    and p.cout in (16, 32, 64)):
                return kernels.conv1x1_resampled_bf16(x, size, p.packed, p.cout, p.scale, p.shift,
                                                      p.relu, out)
            x = self._downsampled(x, size)
        if p.kind == "bf16_2d":
            if x2 is not None:
                raise ValueError(f"{name}: 2D conv takes one input")
            return kernels.conv2d_bnrelu_bf16(x, p.packed, p.cout, p.scale, p.shift, p.relu, out,
                                              accumulate, residual)
        return kernels.conv3d_bnrelu_bf16(x, p.packed, p.cout, p.k, p.scale, p.shift, p.relu, out,
                                          accumulate, x2, residual)


class MatchingExecutorBF16(_C8Layout, MatchingExecutor):
    """newMatching.forward at bf16 (configs 3/4): activations in the c8 layout
    ([B, C/8, D, H, W, 8] bfloat16), convs on the bf16 matrix cores with f32
    accumulation and the f32 BN epilogue; the head's output (the matching cost)
    is f32 for the disparity regression.  Same graph as MatchingExecutor."""

    SPLIT_S1_GROUP48 = False
    # the L0 / L1 cells' steps (8 or 16 channels: one K chunk per conv) as LEA_PAIR_SUM
    # launches of the D-streaming kernel; the L2 cells keep the group + accumulating launches
    PAIR_STEPS = os.environ.get("LEASTEREO_PAIR_STEPS", "1") != "0"

    def __init__(self, matching):
        from .model import ConvBR
        super().__init__(matching)
        with torch.no_grad():
            # re-pack every f32 ConvParams into bf16 fragments (same scale/shift)
            for name, p in list(self.p.items()):
                if name == "last_3":
                    continue  # runs through last_3.taps + tap-sum
                if name == "last_3.taps":
                    w = matching.last_3.conv.weight
                    co, ci = w.shape[:2]
                    taps = w.permute(0, 2, 3, 4, 1).reshape(co * 27, ci, 1, 1, 1)
                    pad = (-taps.shape[0]) % 8  # c8: 27*cout channels padded to a block
                    taps = torch.cat([taps, taps.new_zeros((pad,) + tuple(taps.shape[1:]))], 0)
                    self.p[name] = ConvParams(kernels.pack_conv_weight_bf16(taps), None, None, ci,
                                              taps.shape[0], 1, False, "bf16")
                    continue
                if ".pair" in name:
                    i, k = int(name.split(".")[1]), int(name.rsplit("pair", 1)[1])
                    wa, wb = (matching.cells[i]._ops[op].conv.weight for op, _ in self.pair_steps[i][k])
                    packed = torch.cat([kernels.pack_conv_weight_bf16(wa), kernels.pack_conv_weight_bf16(wb)])
                    self.p[name] = ConvParams(packed, p.scale, p.shift, p.cin, p.cout, p.k, p.relu, "bf16")
                    continue
                if name.endswith(".s1_group"):
                    i = int(name.split(".")[1])
                    mods = [matching.cells[i]._ops[op] for _, op in self.s1_group[i]]
                    w = torch.cat([m.conv.weight for m in mods], 0)
                elif name.endswith(".share"):
                    w = self._share_weight(matching, name)
                else:
                    mod = matching.get_submodule(name)
                    assert isinstance(mod, ConvBR)
                    w = mod.conv.weight
                self.p[name] = ConvParams(kernels.pack_conv_weight_bf16(w), p.scale, p.shift, p.cin,
                                          p.cout, p.k, p.relu, "bf16")

    def _use_winograd(self):
        """bf16 layers stay on the bf16 engine."""

    def _pair_ok(self, x, x2, out):
        return kernels.pair_sum_supported_bf16(x, x2, out)

    def pair_conv(self, name, x, x2, out):
        p = self.p[name]
        return kernels.conv3d_bnrelu_bf16(x, p.packed, p.cout, 3, p.scale, p.shift, True, out, x2=x2,
                                          pair_sum=True)

    def _cv_stem_pack(self, wl, wr):
        return kernels.pack_conv2d_weight_bf16(wl), kernels.pack_conv2d_weight_bf16(wr)

    def _cv_stem(self, fl8, fr8, d3):
        p, (wl, wr) = self.p["stem0"], self.cv
        lm = kernels.conv2d_bnrelu_bf16(fl8, wl, 9 * p.cout, None, None, relu=False)
        rm = kernels.conv2d_bnrelu_bf16(fr8, wr, 6 * p.cout, None, None, relu=False)
        return kernels.cv_stem_combine(lm, rm, p.cout, d3, p.scale, p.shift, p.relu,
                                       name="cv_stem_c8_kernel")

    @staticmethod
    def _tapsum(q, p3, full):
        return kernels.tapsum_upsample_bf16(q, p3.cout, full, p3.scale, p3.shift, p3.relu)

    def _last3_same_size(self, last):
        # per-tap partial sums + a tap-sum at the same size (identity interpolation)
        return self._tapsum(self.conv("last_3.taps", last), self.p["last_3"], self._volume(last))

    def conv(self, *args, **kw):
        return self._conv_c8(*args, **kw)

    def run(self, x):
        """x: f32 cost volume [B, 64, D3, H3, W3] -> f32 matching cost [B, 1, D3, H3, W3]."""
        self._fresh()
        try:
            return self._from_stem0(self.conv("stem0", kernels.to_c8(x)))
        finally:
            self._fresh()

    def run_features(self, fl, fr, maxdisp):
        self._fresh()
        try:
            return self._run_features(fl, fr, maxdisp)
        finally:
            self._fresh()

    def _run_features(self, fl, fr, maxdisp):
        p = self.p["stem0"]
        cf = fl.shape[1] * (8 if fl.dtype == torch.bfloat16 else 1)
        if cf * 2 != p.cin:
            raise ValueError(f"stem0 expects {p.cin} cost-volume channels, got 2*{cf}")
        if fl.dtype == torch.bfloat16:  # the bf16 feature net already hands over c8 maps
            f8, b = _stacked(fl, fr), fl.shape[0]
        else:
            f8 = kernels.to_c8(_stacked(fl, fr))  # [2B, C/8, 1, H, W, 8]
            b = fl.shape[0]
        d3 = int(maxdisp / 3)
        if self.cv is not None and kernels.cv_stem_supported(p.cout, d3, f8.shape[4], True):
            return self._from_stem0(self._cv_stem(f8[:b], f8[b:], d3))
        stem0 = kernels.conv3d_bnrelu_costvolume_bf16(f8[:b], f8[b:], maxdisp, p.packed, p.cout,
                                                      p.scale, p.shift, p.relu)
        return self._from_stem0(stem0)


class FeatureExecutorBF16(_C8Layout, FeatureExecutor):
    """newFeature.forward at bf16 (configs 3/4): stem0 (3 input channels) and the
    stride-3 stem1 stay f32; from stem2 on the maps are c8 and the 3x3 convs run on
    the bf16 engine's 2D tiles.  Returns c8 feature maps [N, 32/8, 1, H3, W3, 8],
    which the bf16 matching net reads directly."""
    PAIR_S0 = False  # (the pair launch is the f32 few-channel tile's)

    def __init__(self, feature):
        super().__init__(feature)
        with torch.no_grad():
            for name, p in list(self.p.items()):
                if name in ("stem0", "stem1"):
                    continue
                if name.endswith(".s1_group"):
                    i = int(name.split(".")[1])
                    w = torch.cat([feature.cells[i]._ops[op].conv.weight for _, op in self.s1_group[i]], 0)
                elif name.endswith(".share"):
                    w = self._share_weight(feature, name)
                else:
                    w = feature.get_submodule(name).conv.weight
                if p.kind == "2d":
                    self.p[name] = ConvParams(kernels.pack_conv2d_weight_bf16(w), p.scale, p.shift,
                                              p.cin, p.cout, 3, p.relu, "bf16_2d")
                else:  # 1x1
                    self.p[name] = ConvParams(
                        kernels.pack_conv_weight_bf16(w.reshape(p.cout, p.cin, 1, 1, 1)), p.scale,
                        p.shift, p.cin, p.cout, 1, p.relu, "bf16")

    def conv(self, name, x, *args, **kw):
        if name in ("stem0", "stem1"):
            return CellGraphExecutor.conv(self, name, x, *args, **kw)
        return self._conv_c8(name, x, *args, **kw)

    def run(self, x, x2=None):
        self._fresh()
        try:
            return self._run(x, x2)
        finally:
            self._fresh()

    def _run(self, x, x2=None):
        stem1 = self._stems(x, c8=True, x2=x2)
        stem2 = self.conv("stem2", stem1)
        out = (stem1, stem2)
        for i in range(len(self.m.cells)):
            out = self.cell(i, out[0], out[1])
        last = out[-1]
        h, w = self._volume(stem2)[1:]
        lh = self._volume(last)[1]
        full, half, quarter = (1, h, w), (1, h // 2, w // 2), (1, h // 4, w // 4)
        if lh == h:
            y = last
        elif lh == h // 2:
            y = self._resample(self.conv("last_6", last), full)
        elif lh == h // 4:
            y = self._resample(self.conv("last_6", self.conv("last_12", last), size=half), full)
        elif lh == h // 8:
            # new_model_2d.py:163: last_12(up_24(last_24(x))), then last_6(up_12(.)), up_6
            y = self.conv("last_12", self.conv("last_24", last), size=quarter)
            y = self._resample(self.conv("last_6", y, size=half), full)
        else:
            raise ValueError(f"feature size {tuple(x.shape[2:])} is not legal for the feature net")
        return self.conv("last_3", y)
