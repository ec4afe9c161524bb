#!/usr/bin/env python3
"""Noise figure of the reference network computed in bf16 (tests/golden/bf16_noise.json).

No bf16 tolerance exists upstream (the reference is fp32), so the bf16 path's EPE
bar is taken from the reference algorithm's own sensitivity to bf16 arithmetic: the
oracle (oracle/torch_ref.py, the reference's aten op sequence) run with bf16
weights and activations through the feature and matching nets (torch CPU bf16
convolutions accumulate in f32), its matching cost handed to the disparity
regression in f32 -- the precision split of the HIP bf16 path -- against the same
oracle in f32, on the inputs tests/test_gpu_bf16.py uses at configs 3 and 4.

    python tools/gen_bf16_noise.py      # ~10 min on 8 cores (8 pairs per config)
"""
from __future__ import annotations

import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import torch_ref as ref  # noqa: E402
from tests.golden_util import arch, normal, state_dict  # noqa: E402

# (name, height, width, maxdisp, seed base, pairs measured) -- the tests' inputs:
# pair i of a config is normal(seed + 2 i) / normal(seed + 2 i + 1), [1, 3, H, W]
CASES = [("c3", 384, 1248, 192, 7000, 8), ("c4", 576, 960, 192, 8000, 8)]


def pair_inputs(seed, i, h, w):
    return normal(seed + 2 * i, (1, 3, h, w)), normal(seed + 2 * i + 1, (1, 3, h, w))


def bf16_nets_f32_disp(sd, left, right, maxdisp, a, tap=None):
    sdb = {k: (v.bfloat16() if v.is_floating_point() else v) for k, v in sd.items()}
    fl = ref.feature_forward(sdb, left.bfloat16(), a["net_arch_fea"], a["cell_arch_fea"])
    fr = ref.feature_forward(sdb, right.bfloat16(), a["net_arch_fea"], a["cell_arch_fea"])
    if tap is not None:
        tap("fea_l", fl)
        tap("fea_r", fr)
    mat = ref.matching_forward(sdb, ref.build_cost_volume(fl, fr, maxdisp), a["net_arch_mat"],
                               a["cell_arch_mat"], tap)
    return ref.disp_forward(mat.float(), maxdisp)


def rel_l2(a, r):
    """||a - r|| / ||r|| in float64 (the per-stage parity metric)."""
    a, r = a.double(), r.double()
    return float(torch.linalg.vector_norm(a - r) / torch.linalg.vector_norm(r).clamp_min(1e-30))


def main():
    torch.set_num_threads(os.cpu_count() or 1)
    sd, a = state_dict(), arch()
    out = {"what": "EPE (px) of the oracle with bf16 feature + matching nets and an f32 disparity "
                   "regression vs the oracle in f32, per pair; for pair 0 also each stage's relative L2 "
                   "distance (feature maps, stem0/1, conv1/2, every cell, the matching cost)",
           "script": "tools/gen_bf16_noise.py",
           "cases": {}}
    with torch.no_grad():
        for name, h, w, md, seed, n in CASES:
            epes = []
            stages = {}
            for i in range(n):
                left, right = pair_inputs(seed, i, h, w)
                f32 = {}
                # pair 0: every stage's relative L2 distance too (the oracle in bf16 vs f32)
                want = ref.leastereo_forward(sd, left, right, md, a,
                                             tap=(lambda k, t: f32.__setitem__(k, t)) if i == 0 else None)
                got = bf16_nets_f32_disp(sd, left, right, md, a,
                                         tap=(lambda k, t: stages.__setitem__(k, rel_l2(t, f32.pop(k))))
                                         if i == 0 else None)
                f32.clear()
                epes.append(ref.epe(got, want))
                print(name, i, epes[-1], flush=True)
            out["cases"][name] = {"height": h, "width": w, "maxdisp": md, "seed": seed, "epe_px": epes,
                                  "stage_rel_l2_pair0": stages}
    with open(os.path.join(REPO, "tests", "golden", "bf16_noise.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
