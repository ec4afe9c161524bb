#!/usr/bin/env python3
"""Generate golden vectors by running the *reference* LEAStereo on CPU.

Runs only in the build container (it imports /root/reference, read-only, with
bytecode writing disabled).  Outputs (committed):
  leastereo_amd/data/synthetic_bn.npz  calibrated BN tensors of the weight recipe
  tests/golden/*.npz                   per-op and end-to-end fixtures
  tests/golden/meta.json               seeds, shapes, state_dict sha256, fp32-vs-fp64 noise floor

Inputs are regenerated from seeds (leastereo_amd.weights.seeded_normal) by the
tests, so only outputs are stored.  Nothing from the reference's source is
copied: the fixtures are numbers produced by calling its classes.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from leastereo_amd.weights import (BN_FILE, DEFAULT_SEED, seeded_normal,  # noqa: E402
                                   state_dict_sha256, synthetic_state_dict)

GOLD = os.path.join(REPO, "tests", "golden")
ARCH = os.path.join(REPO, "leastereo_amd", "data", "architecture")


def ref_model(maxdisp):
    sys.path.insert(0, REF)
    from config_utils.leastereo_args import LEAStereoArgs  # reference: config_utils/leastereo_args.py:16
    from retrain.LEAStereo import LEAStereo  # reference: retrain/LEAStereo.py:12
    args = LEAStereoArgs(
        net_arch_fea=os.path.join(ARCH, "feature_network_path.npy"),
        cell_arch_fea=os.path.join(ARCH, "feature_genotype.npy"),
        net_arch_mat=os.path.join(ARCH, "matching_network_path.npy"),
        cell_arch_mat=os.path.join(ARCH, "matching_genotype.npy"))
    args.maxdisp = maxdisp
    args.cuda = False
    return LEAStereo(args, "cpu")


def calibrate_bn(model, shapes):
    """One train-mode pass with momentum 1.0 -> running stats = batch stats."""
    sd0 = synthetic_state_dict(shapes, bn_file=None)
    model.load_state_dict(sd0, strict=True)
    for m in model.modules():
        if isinstance(m, (nn.BatchNorm2d, nn.BatchNorm3d)):
            m.momentum = 1.0
    model.train()
    left = torch.from_numpy(seeded_normal(101, (1, 3, 288, 576)))
    right = torch.from_numpy(seeded_normal(102, (1, 3, 288, 576)))
    with torch.no_grad():
        model(left, right)
    model.eval()
    out = {}
    for k, v in model.state_dict().items():
        if ".bn." in k:
            v = v.detach().clone()
            if k.endswith("running_var"):
                v = v.clamp(min=2.0)
            out[k] = v.numpy()
    np.savez(BN_FILE, **out)
    print(f"wrote {BN_FILE}: {len(out)} tensors")


def main():
    os.makedirs(GOLD, exist_ok=True)
    t0 = time.time()
    model = ref_model(96)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    calibrate_bn(model, shapes)
    sd = synthetic_state_dict(shapes)
    model.load_state_dict(sd, strict=True)
    model.eval()
    meta = {"seed": DEFAULT_SEED, "state_dict_sha256": state_dict_sha256(sd),
            "n_tensors": len(sd), "n_params": int(sum(v.numel() for k, v in sd.items()
                                                      if "running" not in k and "num_batches" not in k)),
            "state_dict_shapes": [[k, list(v)] for k, v in shapes.items()],
            "torch": torch.__version__, "numpy": np.__version__, "cases": {}}

    # ---- (1) cost volume through LEAStereo.forward with identity sub-nets (LEAStereo.py:34-48)
    cv = {}
    for name, (b, c, h, w, maxdisp, sa, sb) in {
            "c4_h8_w16_d24": (1, 4, 8, 16, 24, 11, 12),
            "c32_h8_w12_d24": (1, 32, 8, 12, 24, 13, 14),
            "b2_c4_h4_w6_d24": (2, 4, 4, 6, 24, 15, 16),   # W3 < D3: empty slices
            "c3_h5_w7_d9": (1, 3, 5, 7, 9, 17, 18)}.items():
        m = ref_model(maxdisp)
        m.feature = nn.Identity(); m.matching = nn.Identity(); m.disp = nn.Identity()
        fl = torch.from_numpy(seeded_normal(sa, (b, c, h, w)))
        fr = torch.from_numpy(seeded_normal(sb, (b, c, h, w)))
        with torch.no_grad():
            cv[name] = m(fl, fr).numpy()
        meta["cases"]["cost_volume/" + name] = {"shape": [b, c, h, w], "maxdisp": maxdisp,
                                                "seeds": [sa, sb]}
    np.savez_compressed(os.path.join(GOLD, "cost_volume.npz"), **cv)

    # ---- (2) ConvBR3d, one per distinct (Cin, Cout, k, bn, relu) (operations_3d.py:31-47)
    convs = {}
    seen = set()
    mods = dict(model.named_modules())
    seed = 200
    for name, mod in mods.items():
        if not name.startswith("matching.") or type(mod).__name__ != "ConvBR":
            continue
        w = mod.conv.weight
        sig = (w.shape[1], w.shape[0], w.shape[-1], mod.use_bn, mod.relu)
        if sig in seen:
            continue
        seen.add(sig)
        for tag, shape in (("", (1, w.shape[1], 4, 6, 10)), ("_ragged", (2, w.shape[1], 3, 5, 19))):
            seed += 1
            x = torch.from_numpy(seeded_normal(seed, shape))
            with torch.no_grad():
                y = mod(x)
            key = name.replace(".", "_") + tag
            convs[key] = y.numpy()
            meta["cases"]["convbr/" + key] = {"module": name, "input": list(shape), "seed": seed,
                                              "cin": sig[0], "cout": sig[1], "k": sig[2],
                                              "bn": bool(sig[3]), "relu": bool(sig[4])}
    np.savez_compressed(os.path.join(GOLD, "convbr.npz"), **convs)

    # ---- (3) trilinear align_corners=True with the reference's scale_dimension (skip_model_3d.py:38-50)
    cell = model.matching.cells[0]
    rs = {}
    cases = [("down_odd", (1, 3, 5, 7, 9), 0.5), ("down_even", (1, 2, 4, 6, 8), 0.5),
             ("up_mixed", (2, 3, 3, 4, 5), 2), ("down_mixed", (1, 4, 8, 5, 12), 0.5)]
    for name, shape, scale in cases:
        seed += 1
        x = torch.from_numpy(seeded_normal(seed, shape))
        size = [cell.scale_dimension(n, scale) for n in shape[2:]]
        rs[name] = F.interpolate(x, size, mode="trilinear", align_corners=True).numpy()
        meta["cases"]["resample/" + name] = {"input": list(shape), "seed": seed, "size": size}
    for name, shape, size in [("match", (1, 2, 8, 12, 16), [4, 6, 8]), ("generic", (1, 2, 5, 6, 7), [8, 9, 10])]:
        seed += 1
        x = torch.from_numpy(seeded_normal(seed, shape))
        rs[name] = F.interpolate(x, size, mode="trilinear", align_corners=True).numpy()
        meta["cases"]["resample/" + name] = {"input": list(shape), "seed": seed, "size": size}
    np.savez_compressed(os.path.join(GOLD, "resample.npz"), **rs)

    # ---- (4) Disp (build_model_2d.py:27-57)
    sys.path.insert(0, REF)
    from models.build_model_2d import Disp  # reference: models/build_model_2d.py:45
    ds = {}
    for name, shape, maxdisp, gain in [("d8_h12_w16_md24", (1, 1, 8, 12, 16), 24, 1.0),
                                       ("b2_d4_h5_w7_md12", (2, 1, 4, 5, 7), 12, 1.0),
                                       ("sharp_d8_h6_w10_md24", (1, 1, 8, 6, 10), 24, 8.0)]:
        seed += 1
        x = torch.from_numpy(seeded_normal(seed, shape)) * gain
        with torch.no_grad():
            ds[name] = Disp("cpu", maxdisp)(x.contiguous()).numpy()
        meta["cases"]["disp/" + name] = {"input": list(shape), "seed": seed, "maxdisp": maxdisp,
                                         "gain": gain}
    np.savez_compressed(os.path.join(GOLD, "disp.npz"), **ds)

    # ---- (5) end to end (LEAStereo.py:30-52), fp32 and fp64
    e2e = {}
    for name, (b, h, w, maxdisp, sa, sb) in {"b1_h96_w192_md48": (1, 96, 192, 48, 301, 302),
                                              "b2_h48_w96_md24": (2, 48, 96, 24, 303, 304)}.items():
        m = ref_model(maxdisp)
        m.load_state_dict(sd, strict=True)
        m.eval()
        left = torch.from_numpy(seeded_normal(sa, (b, 3, h, w)))
        right = torch.from_numpy(seeded_normal(sb, (b, 3, h, w)))
        with torch.no_grad():
            fl = m.feature(left)
            mat_in = None
            d32 = m(left, right)
            md = m.double()
            d64 = md(left.double(), right.double())
        e2e[name + "/disp32"] = d32.numpy()
        e2e[name + "/disp64"] = d64.numpy()
        if b == 1:
            e2e[name + "/fea_l"] = fl.numpy()
            # matching output of the fp32 model for stage-level checks
            mf = ref_model(maxdisp); mf.load_state_dict(sd, strict=True); mf.eval()
            captured = {}
            mf.disp.register_forward_hook(lambda mod, inp, out: captured.setdefault("mat", inp[0].detach().clone()))
            with torch.no_grad():
                mf(left, right)
            e2e[name + "/matching"] = captured["mat"].numpy()
        noise = float(np.abs(d32.numpy().astype(np.float64) - d64.numpy()).mean())
        noise_max = float(np.abs(d32.numpy().astype(np.float64) - d64.numpy()).max())
        meta["cases"]["e2e/" + name] = {"batch": b, "height": h, "width": w, "maxdisp": maxdisp,
                                        "seeds": [sa, sb], "epe_fp32_vs_fp64": noise,
                                        "max_abs_fp32_vs_fp64": noise_max,
                                        "disp_std": float(d32.std())}
        print(name, "fp32-vs-fp64 EPE", noise, "max", noise_max, "std", float(d32.std()))
        del mat_in
    np.savez_compressed(os.path.join(GOLD, "e2e.npz"), **e2e)
    meta["gen_seconds"] = round(time.time() - t0, 1)
    with open(os.path.join(GOLD, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("done in", meta["gen_seconds"], "s")


if __name__ == "__main__":
    main()
