#!/usr/bin/env python3
"""bf16 path probe: EPE vs the f32 path / the reference fixture, and timing at
configs 2 (576x960 D192 B1), 3 (384x1248 D192 B8) and 4 (576x960 D192 B8/GPU)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd.config import LEAStereoArgs, default_arch_args  # noqa: E402
from leastereo_amd.model import LEAStereo  # noqa: E402
from oracle import torch_ref as ref  # noqa: E402
from tests.golden_util import golden, meta, normal, state_dict  # noqa: E402


def model(maxdisp, precision):
    m = LEAStereo(default_arch_args(LEAStereoArgs(maxdisp=maxdisp)), "cuda", precision=precision)
    m.load_state_dict(state_dict(), strict=True)
    return m.cuda().eval()


def timed(m, l, r, n=10):
    with torch.no_grad():
        for _ in range(3):
            m(l, r)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(n):
            m(l, r)
        torch.cuda.synchronize()
    return (time.time() - t0) / n


res = {}
c = meta()["cases"]["e2e/b1_h96_w192_md48"]
l, r = normal(c["seeds"][0], (1, 3, 96, 192)).cuda(), normal(c["seeds"][1], (1, 3, 96, 192)).cuda()
with torch.no_grad():
    d = model(48, "bf16")(l, r).cpu()
res["golden_e2e_epe_bf16_vs_ref_f32"] = ref.epe(d, torch.from_numpy(golden("e2e")["b1_h96_w192_md48/disp32"]))
for name, (b, h, w, md) in {"c2": (1, 576, 960, 192), "c3": (8, 384, 1248, 192), "c4": (8, 576, 960, 192)}.items():
    l, r = normal(11, (b, 3, h, w)).cuda(), normal(12, (b, 3, h, w)).cuda()
    mb, mf = model(md, "bf16"), model(md, "f32")
    with torch.no_grad():
        db, df = mb(l, r), mf(l, r)
    res[name] = {"epe_bf16_vs_f32": ref.epe(db.cpu(), df.cpu()),
                 "bf16_s": timed(mb, l, r), "f32_s": timed(mf, l, r, 3), "batch": b}
    res[name]["bf16_pairs_s"] = b / res[name]["bf16_s"]
    res[name]["f32_pairs_s"] = b / res[name]["f32_s"]
    print(name, res[name], flush=True)
print(json.dumps(res))
