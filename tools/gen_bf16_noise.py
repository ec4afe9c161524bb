#!/usr/bin/env python3
"""Noise figure of the reference network computed in bf16 (tests/golden/bf16_noise.json).

No bf16 tolerance exists upstream (the reference is fp32), so the bf16 path's EPE
bar is taken from the reference network's own sensitivity to bf16 arithmetic: its
feature and matching nets with bf16 weights and activations (torch CPU bf16
convolutions accumulate in f32), the matching cost handed to the disparity regression
in f32 -- the precision split of the HIP bf16 path -- against the same network in f32,
on the inputs tests/test_gpu_bf16.py uses at configs 3 and 4 (8 pairs each), plus pair
0's relative L2 distance at every stage (feature maps, stem0/1, conv1/2, the 12 cells,
the matching cost).

--source oracle (the default since r06): oracle/torch_ref.py (the reference's
aten op sequence restated) in bf16 vs f32: tests/golden/bf16_noise_oracle.json.  It
reproduces the reference's figures bit for bit (``agreement_with_oracle`` in
bf16_noise.json), so regenerating the bar needs no reference code.

--source reference (explicit opt-in only; VERDICT r04 #5 made the committed
bf16_noise.json this way): the reference itself --
/root/reference/retrain/LEAStereo.py imported read-only (bytecode writing off, as
tools/gen_golden.py does), its ``feature`` and ``matching`` modules converted to
bfloat16, its own ``LEAStereo.forward`` (cost volume at LEAStereo.py:34-48 included)
with the ``Disp`` module wrapped to take the cost in f32 (LEAStereo.py:51); stage
values through forward hooks on the reference's modules.  Writes bf16_noise.json and
its agreement with the oracle's figures (bf16_noise_oracle.json).

Only our own deterministic weights (leastereo_amd.weights) are loaded into it; no
pickle or checkpoint from the reference tree is read.

    python tools/gen_bf16_noise.py                       # oracle
    PYTHONDONTWRITEBYTECODE=1 python tools/gen_bf16_noise.py --source reference
    (~10-20 min on 8 cores)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.dont_write_bytecode = True
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import torch_ref as ref  # noqa: E402
from tests.golden_util import GOLD, arch, normal, state_dict  # noqa: E402

# (name, height, width, maxdisp, seed base, pairs measured) -- the tests' inputs:
# pair i of a config is normal(seed + 2 i) / normal(seed + 2 i + 1), [1, 3, H, W]
CASES = [("c3", 384, 1248, 192, 7000, 8), ("c4", 576, 960, 192, 8000, 8)]
STAGES = ["fea_l", "fea_r", "stem0", "stem1"] + [f"cell{i}" for i in range(5)] + ["conv1"] + \
         [f"cell{i}" for i in range(5, 9)] + ["conv2"] + [f"cell{i}" for i in range(9, 12)] + ["matching"]


def pair_inputs(seed, i, h, w):
    return normal(seed + 2 * i, (1, 3, h, w)), normal(seed + 2 * i + 1, (1, 3, h, w))


def rel_l2(a, r):
    """||a - r|| / ||r|| in float64 (the per-stage parity metric)."""
    a, r = a.double(), r.double()
    return float(torch.linalg.vector_norm(a - r) / torch.linalg.vector_norm(r).clamp_min(1e-30))


# ------------------------------------------------------------------ the oracle restatement
def oracle_runner(sd, a):
    def f32(left, right, md, tap):
        return ref.leastereo_forward(sd, left, right, md, a, tap=tap)

    def bf16(left, right, md, tap):
        sdb = {k: (v.bfloat16() if v.is_floating_point() else v) for k, v in sd.items()}
        fl = ref.feature_forward(sdb, left.bfloat16(), a["net_arch_fea"], a["cell_arch_fea"])
        fr = ref.feature_forward(sdb, right.bfloat16(), a["net_arch_fea"], a["cell_arch_fea"])
        if tap is not None:
            tap("fea_l", fl)
            tap("fea_r", fr)
        mat = ref.matching_forward(sdb, ref.build_cost_volume(fl, fr, md), a["net_arch_mat"],
                                   a["cell_arch_mat"], tap)
        return ref.disp_forward(mat.float(), md)
    return f32, bf16


# ------------------------------------------------------------------ the reference itself
class _F32Disp(nn.Module):
    """The reference's Disp (build_model_2d.py:45-57) on the matching cost cast to f32."""

    def __init__(self, disp):
        super().__init__()
        self.inner = disp

    def forward(self, x):
        return self.inner(x.float())


def reference_runner(sd):
    sys.path.insert(0, REF)
    from config_utils.leastereo_args import LEAStereoArgs  # reference: config_utils/leastereo_args.py:16
    from retrain.LEAStereo import LEAStereo  # reference: retrain/LEAStereo.py:12
    arch_dir = os.path.join(REPO, "leastereo_amd", "data", "architecture")
    cache = {}

    def model(md, bf16):
        if (md, bf16) not in cache:
            args = LEAStereoArgs(net_arch_fea=os.path.join(arch_dir, "feature_network_path.npy"),
                                 cell_arch_fea=os.path.join(arch_dir, "feature_genotype.npy"),
                                 net_arch_mat=os.path.join(arch_dir, "matching_network_path.npy"),
                                 cell_arch_mat=os.path.join(arch_dir, "matching_genotype.npy"))
            args.maxdisp, args.cuda = md, False
            m = LEAStereo(args, "cpu")
            m.load_state_dict(sd, strict=True)
            m.eval()
            if bf16:
                m.feature.to(torch.bfloat16)
                m.matching.to(torch.bfloat16)
                m.disp = _F32Disp(m.disp)
            cache[(md, bf16)] = m
        return cache[(md, bf16)]

    def run(m, left, right, tap, bf16):
        hooks = []
        if tap is not None:
            calls = []

            def feature_hook(mod, i, o):  # LEAStereo.py:31-32: left, then right
                tap("fea_r" if calls else "fea_l", o)
                calls.append(1)
            hooks.append(m.feature.register_forward_hook(feature_hook))
            mm = m.matching
            for name in ("stem0", "stem1", "conv1", "conv2"):
                hooks.append(getattr(mm, name).register_forward_hook(
                    lambda mod, i, o, n=name: tap(n, o)))
            for k, cell in enumerate(mm.cells):  # Cell.forward returns (prev_input, concat_feature)
                hooks.append(cell.register_forward_hook(lambda mod, i, o, n=f"cell{k}": tap(n, o[1])))
            hooks.append(mm.register_forward_hook(lambda mod, i, o: tap("matching", o)))
        try:
            x, y = (left.bfloat16(), right.bfloat16()) if bf16 else (left, right)
            return m(x, y)
        finally:
            for h in hooks:
                h.remove()

    def f32(left, right, md, tap):
        return run(model(md, False), left, right, tap, False)

    def bf16(left, right, md, tap):
        return run(model(md, True), left, right, tap, True)
    return f32, bf16


def measure(f32_fn, bf16_fn):
    cases = {}
    with torch.no_grad():
        for name, h, w, md, seed, n in CASES:
            epes, stages = [], {}
            for i in range(n):
                left, right = pair_inputs(seed, i, h, w)
                f32 = {}
                want = f32_fn(left, right, md, (lambda k, t: f32.__setitem__(k, t)) if i == 0 else None)
                got = bf16_fn(left, right, md,
                              (lambda k, t: stages.__setitem__(k, rel_l2(t, f32.pop(k)))) if i == 0 else None)
                f32.clear()
                epes.append(ref.epe(got, want))
                print(name, i, epes[-1], flush=True)
            missing = [s for s in STAGES if s not in stages]
            assert not missing, f"stages not tapped: {missing}"
            cases[name] = {"height": h, "width": w, "maxdisp": md, "seed": seed, "epe_px": epes,
                           "stage_rel_l2_pair0": {s: stages[s] for s in STAGES}}
    return cases


def agreement(cases, other):
    """How closely two runs' figures agree: per config the largest |difference| of the pair
    EPEs, of their worst pairs, and the largest ratio of the stage distances."""
    out = {}
    for name, c in cases.items():
        o = other[name]
        ratios = [c["stage_rel_l2_pair0"][s] / o["stage_rel_l2_pair0"][s] for s in STAGES]
        out[name] = {"max_abs_diff_pair_epe_px": max(abs(x - y) for x, y in zip(c["epe_px"], o["epe_px"])),
                     "worst_pair_px": [max(c["epe_px"]), max(o["epe_px"])],
                     "stage_ratio_min_max": [min(ratios), max(ratios)]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", choices=("reference", "oracle"), default="oracle",
                    help="oracle (default): the restatement; reference: import /root/reference (opt-in)")
    opt = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    sd, a = state_dict(), arch()
    if opt.source == "oracle":
        cases = measure(*oracle_runner(sd, a))
        out = {"what": "EPE (px) of the oracle (oracle/torch_ref.py) with bf16 feature + matching nets and an "
                       "f32 disparity regression vs the oracle in f32, per pair; for pair 0 also each stage's "
                       "relative L2 distance", "source": "oracle", "script": "tools/gen_bf16_noise.py --source oracle",
               "cases": cases}
        path = os.path.join(GOLD, "bf16_noise_oracle.json")
    else:
        cases = measure(*reference_runner(sd))
        out = {"what": "EPE (px) of the reference network with bf16 feature + matching nets and an f32 "
                       "disparity regression vs the reference in f32, per pair; for pair 0 also each stage's "
                       "relative L2 distance (feature maps, stem0/1, conv1/2, every cell, the matching cost)",
               "source": "reference: /root/reference/retrain/LEAStereo.py imported read-only; feature and "
                         "matching modules in bfloat16, LEAStereo.forward unchanged, Disp on the f32 cost; "
                         "stages through forward hooks",
               "script": "tools/gen_bf16_noise.py", "cases": cases}
        op = os.path.join(GOLD, "bf16_noise_oracle.json")
        if os.path.exists(op):
            with open(op) as f:
                out["agreement_with_oracle"] = agreement(cases, json.load(f)["cases"])
        path = os.path.join(GOLD, "bf16_noise.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
