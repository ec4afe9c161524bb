#!/usr/bin/env python3
"""Per-layer A/B of a library tuning setter on the C2 matching-net conv shapes, in ONE
process (r06): for each layer, every value of ``--setter`` is timed with HIP events in
interleaved rounds (the value order reversed on odd rounds), after a warm layer, and the
outputs of all values are compared bit for bit (``--exact 1``) -- a kernel change that is
meant to be bit-identical is checked in the same run that times it.

  python tools/setter_ab.py --setter lea_conv3d_wino2p_set_wpre --values 0,1 \\
      [--only conv12_128to64_k3_L1,...] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leastereo_amd import _lib, kernels  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402

# the layers the pipelined W x D kernel runs at C2 (DESIGN.md §4 by-shape split)
WINO2P = "stem1_32to32_k3_L0,conv12_128to64_k3_L1,cell_16to32_k3_L1_s1grp2,cell_32to96_k3_L2_s1grp,cell_32to32_k3_L2"
# launches per C2 forward where LAYERS' count is the pre-r03 split (the 16 -> 48 L1 group runs as
# 16 -> 32 on this kernel + 16 -> 16 on the per-lane tile since r03)
COUNTS = {"cell_16to32_k3_L1_s1grp2": 6, "cell_16to48_k3_L1_s1grp": 0, "cell_16to16_k3_L1": 24}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--setter", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--only", default=WINO2P)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--exact", type=int, default=1)
    ap.add_argument("--restore", type=int, default=None, help="setter value after the run")
    a = ap.parse_args()
    lib = _lib.load()
    setter = getattr(lib, a.setter)
    values = [int(v) for v in a.values.split(",")]
    dev = "cuda"
    only = a.only.split(",")
    report = {"setter": a.setter, "values": values, "layers": {}}
    warm = True
    for name in only:
        cin, cout, k, (d, h, w), count, *acc = LAYERS[name]
        count = COUNTS.get(name, count)
        acc = bool(acc and acc[0])
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(1, cin, d, h, w, device=dev, generator=g)
        wt = torch.randn(cout, cin, 3, 3, 3, device=dev, generator=g) / (cin * 27) ** 0.5
        scale = torch.rand(cout, device=dev, generator=g) + 0.5
        shift = torch.randn(cout, device=dev, generator=g) * 0.1
        r = torch.randn(1, cout, d, h, w, device=dev, generator=g)
        pw = kernels.pack_conv_weight_wino(wt)
        ys = {v: r.clone() for v in values}

        def run(v):
            _lib.check(setter(v), a.setter)
            y = ys[v]
            if acc:
                y.copy_(r)
            kernels.conv3d_bnrelu_wino(x, pw, cout, scale, shift, True, y, acc)

        if warm:  # the first layer a process times runs at a lower clock
            for _ in range(30):
                run(values[0])
            warm = False
        times = {v: [] for v in values}
        names = {}
        for rnd in range(a.rounds):
            order = values if rnd % 2 == 0 else values[::-1]
            for v in order:
                _lib.check(setter(v), a.setter)
                names[v] = kernels.wino_kernel_name(1, cout, d, h, w, cin=cin)
                run(v)
                torch.cuda.synchronize()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
                for _ in range(a.iters):
                    run(v)
                e[1].record()
                torch.cuda.synchronize()
                times[v].append(e[0].elapsed_time(e[1]) / a.iters * 1e3)
        base = values[0]
        same = {v: bool(torch.equal(ys[v], ys[base])) for v in values}
        row = {"kernel": names, "count_per_forward": count,
               "us_median": {v: statistics.median(t) for v, t in times.items()},
               "us_min": {v: min(t) for v, t in times.items()}, "bit_identical_to_first": same}
        report["layers"][name] = row
        print(name, " ".join(f"{v}: {row['us_median'][v]:.1f}us" for v in values),
              "identical" if all(same.values()) else f"DIFFERENT {same}", flush=True)
        if a.exact and not all(same.values()):
            print(json.dumps(report))
            sys.exit(3)
    tot = {v: sum(r["us_median"][v] * r["count_per_forward"] for r in report["layers"].values()) for v in values}
    report["forward_us"] = tot
    print("per forward (count-weighted):", " ".join(f"{v}: {t:.1f}us" for v, t in tot.items()))
    if a.restore is not None:
        _lib.check(setter(a.restore), a.setter)
    print(json.dumps(report))


if __name__ == "__main__":
    main()
