#!/usr/bin/env python3
"""Benchmark: LEAStereo inference (feature net -> cost volume -> matching net ->
disparity regression) on synthetic stereo pairs, one process per GPU.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
is launched by torch.distributed.run (one rank per GPU, RCCL).  A step is one
forward of ``--batch`` pairs per rank with inputs already resident in HBM.
Rank 0 prints one JSON line.

Workload (BASELINE.json configs[1]): SceneFlow 576x960, maxdisp 192, fp32,
batch 1 per GPU; random-init weights of the reference architecture
(leastereo_amd.weights recipe; no checkpoints exist upstream) and synthetic
N(0,1) images (the post-standardisation statistics of predict.py:162-184).

Extras in the JSON line:
  roofline      the dominant conv kernel instantiation timed with HIP events
                inside the timed region (algorithmic FLOPs / event time)
  cpu_baseline  the CPU oracle (oracle/torch_ref.py, a restatement of the
                reference's exact aten op sequence) on the host cores, rank 0, N=1
  epe_px        per rank: HIP disparity vs the reference's own fp32 output on the
                golden e2e case, all-gathered over ranks (one RCCL all-gather)
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from leastereo_amd import kernels, parallel  # noqa: E402
from leastereo_amd.config import LEAStereoArgs, default_arch_args  # noqa: E402
from leastereo_amd.model import LEAStereo  # noqa: E402
from leastereo_amd.weights import synthetic_state_dict  # noqa: E402

METRIC = "stereo pairs/s at 576×960 D=192, 1/2/4/8 GPU; EPE vs reference"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, fp32 (vector = MFMA) dense
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, spec


# BASELINE.json configs: c2 is the headline workload (defaults);
# c3/c4 are the bf16 ones (c4 = 8 pairs per GPU of the 64-pair global batch)
CONFIGS = {
    "c2": dict(height=576, width=960, maxdisp=192, batch=1, precision="f32"),
    "c3": dict(height=384, width=1248, maxdisp=192, batch=8, precision="bf16"),
    "c4": dict(height=576, width=960, maxdisp=192, batch=8, precision="bf16"),
    "c5": dict(height=1008, width=1512, maxdisp=264, batch=1, precision="f32"),
}
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, bf16 dense (no sparsity)
# Whole-path roofline time per step, SURVEY.md §8d (sum over the matching net's
# layers of max(FLOP/peak, bytes/8 TB/s), reference op accounting), per config
T_ROOF_MS = {("c2", 1): 11.36, ("c3", 8): 10.91, ("c4", 8): 12.59, ("c5", 1): 43.1}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=1, help="pairs per GPU per step")
    p.add_argument("--height", type=int, default=576)
    p.add_argument("--width", type=int, default=960)
    p.add_argument("--maxdisp", type=int, default=192)
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle (rank 0, N=1)")
    p.add_argument("--cpu-steps", type=int, default=2)
    p.add_argument("--epe", type=int, default=1, help="check EPE vs the reference golden disparity")
    p.add_argument("--breakdown", type=int, default=0, help="print per-kernel conv times to stderr")
    p.add_argument("--graph", type=int, default=0,
                   help="time a HIP-graph replay of the forward (LEAStereo.graphed) instead of eager launches")
    p.add_argument("--precision", choices=("f32", "bf16"), default="f32",
                   help="matching-net arithmetic (bf16 = BASELINE configs 3/4)")
    p.add_argument("--config", choices=sorted(CONFIGS), default=None,
                   help="preset: c2 (default workload) / c3 / c4 (per GPU) / c5 of BASELINE.json")
    a = p.parse_args()
    if a.config:
        for k, v in CONFIGS[a.config].items():
            setattr(a, k, v)
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(maxdisp, device, precision="f32"):
    args = default_arch_args(LEAStereoArgs(maxdisp=maxdisp))
    model = LEAStereo(args, device, precision=precision)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    model.load_state_dict(synthetic_state_dict(shapes), strict=True)
    return model.to(device).eval()


def cpu_baseline(args, model, left0, right0, disp0):
    """CPU leg: the oracle (oracle/torch_ref.py, the reference's aten op sequence
    restated) on the host cores, on a bounded sample of the same workload: the
    benchmark's own first pair, ``--cpu-steps`` times.  Its output doubles as
    the parity check of the HIP disparity for that pair (EPE reported)."""
    from oracle import torch_ref as ref
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    a = arch_arrays()
    left, right = left0.cpu(), right0.cpu()
    with torch.no_grad():
        ref.leastereo_forward(sd, left[..., :96, :192].contiguous(), right[..., :96, :192].contiguous(),
                              48, a)  # warm the CPU kernels on a small case
        t0 = time.perf_counter()
        for _ in range(args.cpu_steps):
            want = ref.leastereo_forward(sd, left, right, args.maxdisp, a)
        dt = time.perf_counter() - t0
    cpu_model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": args.cpu_steps / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_steps} forward(s) of the benchmark's first pair at "
                      f"{args.height}x{args.width} D={args.maxdisp} fp32 (oracle/torch_ref.py on "
                      f"torch CPU, {cpu_model})",
            "s_per_pair": dt / args.cpu_steps,
            "epe_px_hip_vs_this": float((disp0.cpu().double() - want.double()).abs().mean())}


def arch_arrays():
    import numpy as np
    from leastereo_amd.config import ARCH_DIR
    return {k: np.load(os.path.join(ARCH_DIR, f)) for k, f in (
        ("net_arch_fea", "feature_network_path.npy"), ("cell_arch_fea", "feature_genotype.npy"),
        ("net_arch_mat", "matching_network_path.npy"), ("cell_arch_mat", "matching_genotype.npy"))}


def golden_epe(device, precision="f32"):
    """HIP disparity vs the reference's own fp32 output (tests/golden/e2e.npz,
    produced by tools/gen_golden.py from /root/reference) on its seeded input."""
    import numpy as np
    from leastereo_amd.weights import seeded_normal
    gold = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gold, "meta.json")) as f:
        case = json.load(f)["cases"]["e2e/b1_h96_w192_md48"]
    want = np.load(os.path.join(gold, "e2e.npz"))["b1_h96_w192_md48/disp32"]
    m = build_model(case["maxdisp"], device, precision)
    shape = (1, 3, case["height"], case["width"])
    left = torch.from_numpy(seeded_normal(case["seeds"][0], shape)).to(device)
    right = torch.from_numpy(seeded_normal(case["seeds"][1], shape)).to(device)
    with torch.no_grad():
        got = m(left, right).cpu().double().numpy()
    return float(np.abs(got - want).mean())


def algorithm_name(kernel: str) -> str:
    """The convolution algorithm a conv kernel instantiation runs."""
    if kernel.startswith("conv3d_wino2_kernel<"):
        return "winograd F(4,3) along W x F(2,3) along D"
    if kernel.startswith("conv3d_wino_kernel<"):
        return f"winograd F({kernel.split('<')[1].split(',')[0]},3) along W"
    return "direct convolution"


def _quantile(xs, q):
    """Linear-interpolated quantile of a sorted list."""
    pos = q * (len(xs) - 1)
    i = int(pos)
    j = min(i + 1, len(xs) - 1)
    return xs[i] + (xs[j] - xs[i]) * (pos - i)


def main():
    args = parse()
    info = parallel.rank_info()
    world, rank = info.world, info.rank
    device = torch.device("cuda", info.local_rank)
    if world > 1:
        torch.cuda.set_device(device)
    parallel.init("nccl", info, device)  # nccl = RCCL over xGMI on ROCm
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False

    model = build_model(args.maxdisp, device, args.precision)
    model.check_shape(args.height, args.width)
    # weak scaling: every rank owns args.batch pairs of the global batch (shard of
    # world*batch pairs), generated on its own device from a rank-seeded stream
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    left = torch.randn(args.batch, 3, args.height, args.width, device=device, generator=g)
    right = torch.randn(args.batch, 3, args.height, args.width, device=device, generator=g)

    def step():
        return model(left, right)

    if args.graph:
        graphed = model.graphed(args.batch, args.height, args.width)

        def step():  # noqa: F811  (inputs already resident: replay only)
            graphed.graph.replay()
            return graphed.out
        graphed.x.copy_(left)
        graphed.y.copy_(right)

    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            out = step()
        # find the dominant conv kernel instantiation (untimed eager pass)
        with kernels.KernelProbe() as probe:
            model(left, right)
        per_kernel = probe.summary()
        dominant = max(per_kernel, key=lambda n: per_kernel[n]["ms"])
        if args.breakdown and info.is_main:
            for n, d in sorted(per_kernel.items(), key=lambda kv: -kv[1]["ms"]):
                log(f"{n:40s} launches {d['launches']:3d}  {d['ms']:8.3f} ms  "
                    f"{d['flops'] / d['ms'] / 1e9:8.1f} TFLOP/s  {d['bytes'] / d['ms'] / 1e6:8.1f} GB/s")

        parallel.barrier()
        torch.cuda.synchronize()
        with kernels.KernelProbe([dominant]) as probe:
            # per-step latency: HIP events between consecutive steps (SURVEY §8d's
            # median and p10/p90), on the stream the forward is launched on
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            t0 = time.perf_counter()
            ev[0].record()
            for i in range(args.steps):
                out = step()
                ev[i + 1].record()
            torch.cuda.synchronize()
            parallel.barrier()
            elapsed = time.perf_counter() - t0
        if args.graph:  # replays bypass the launch-time probe: time one eager forward after
            with kernels.KernelProbe([dominant]) as probe:
                model(left, right)
        dom = probe.summary()[dominant]
        step_ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps))
    elapsed = parallel.max_over_ranks(elapsed, device)

    epe = None
    if args.epe:  # after the timed region: one all-gather of the per-rank parity check
        e = torch.tensor([golden_epe(device, args.precision)], device=device, dtype=torch.float32)
        epe = [float(v) for v in parallel.gather_per_pair(e).cpu()]

    flops_per_launch = dom["flops"] / dom["launches"]
    ms_per_launch = dom["ms"] / dom["launches"]
    achieved = flops_per_launch / (ms_per_launch * 1e-3) / 1e12
    mfma_tflops = dom["mfma_flops"] / dom["launches"] / (ms_per_launch * 1e-3) / 1e12
    traffic = None
    tf_file = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if os.path.exists(tf_file):
        with open(tf_file) as f:
            tf = json.load(f)
        # per-config entries (tools/traffic_merge.py) first: bytes per launch depend on shapes
        cfg_name = next((k for k, v in CONFIGS.items() if all(getattr(args, f) == x for f, x in v.items())), None)
        traffic = (tf.get(f"{dominant}@{cfg_name}") or tf.get(dominant, {})).get("bytes_per_launch")

    bf16 = args.precision == "bf16"
    peak = BF16_MFMA_PEAK_TFLOPS if bf16 else FP32_MFMA_PEAK_TFLOPS
    workload = {(576, 960, 192, 1, "f32"): "SceneFlow 576x960 D=192 fp32, batch 1 per GPU (BASELINE configs[1])",
                (384, 1248, 192, 8, "bf16"): "KITTI2015 384x1248 D=192 bf16, batch 8 (BASELINE configs[2])",
                (576, 960, 192, 8, "bf16"): "SceneFlow 576x960 D=192 bf16, 8 pairs per GPU (BASELINE configs[3])",
                (1008, 1512, 264, 1, "f32"): "Middlebury 1008x1512 D=264 fp32, batch 1 (BASELINE configs[4], D256 is illegal)",
                }.get((args.height, args.width, args.maxdisp, args.batch, args.precision),
                      f"{args.height}x{args.width} D={args.maxdisp} {args.precision}, batch {args.batch} per GPU")
    result = {
        "metric": METRIC,
        "value": world * args.batch * args.steps / elapsed,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "step_ms": {"median": _quantile(step_ms, 0.5), "p10": _quantile(step_ms, 0.1),
                    "p90": _quantile(step_ms, 0.9), "source": "HIP events between steps, this rank"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic N(0,1) stereo pairs generated on device; random-init weights of the "
                "reference architecture (SceneFlow search result)",
        "config": {"workload": workload,
                   "height": args.height, "width": args.width, "maxdisp": args.maxdisp,
                   "global_batch": world * args.batch,
                   "parallelism": f"dp{world} (independent pairs per rank, no collective in the step)",
                   "launch": "hip graph replay" if args.graph else "eager"},
        "roofline": {"bound": "mfma", "kernel": dominant, "achieved": achieved,
                     "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "launches_per_step": dom["launches"] / args.steps,
                     "flops_per_launch": flops_per_launch, "ms_per_launch": ms_per_launch,
                     # products the kernel actually issues: Winograd F(2,3) does 4 per 6 of
                     # the direct convolution whose FLOPs define `achieved`
                     "algorithm": algorithm_name(dominant),
                     "mfma_executed": mfma_tflops, "mfma_executed_frac": mfma_tflops / peak},
        "epe_px": None if epe is None else {
            "vs": "reference LEAStereo fp32 disparity (tests/golden e2e b1_h96_w192_md48)",
            "max_over_ranks": max(epe), "per_rank": epe},
    }
    cfg = next((k for k, v in CONFIGS.items() if all(getattr(args, f) == x for f, x in v.items())), None)
    t_roof = T_ROOF_MS.get((cfg, args.batch))
    if t_roof is not None:
        result["path_roofline"] = {"t_roof_ms": t_roof, "frac": t_roof / result["ms_per_step"],
                                   "source": "SURVEY.md §8d: sum over matching-net layers of "
                                             "max(FLOP / MFMA peak, bytes / 8 TB/s)"}
    if bf16 and result["epe_px"] is not None:
        result["epe_px"]["vs"] += " (bf16 matching net: no upstream tolerance; see DESIGN.md)"
    if info.is_main and world == 1 and args.cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, model, left[:1], right[:1], out[:1])
    if info.is_main:
        print(json.dumps(result), flush=True)
    parallel.finalize()


if __name__ == "__main__":
    main()
