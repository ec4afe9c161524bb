#!/usr/bin/env python3
"""Benchmark: LEAStereo inference (feature net -> cost volume -> matching net ->
disparity regression) on synthetic stereo pairs, one process per GPU.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  For N > 1 the
driver launches it under torch.distributed.run (one rank per GPU, RCCL); started
directly with ``--gpus N > 1`` and no WORLD_SIZE in the environment, bench.py starts
that launcher itself as a child process (before anything touches a GPU) and exits
with its status.  A rank whose world size differs from ``--gpus`` refuses to run.
A step is one forward of ``--batch`` pairs per rank with inputs already resident in
HBM.  Rank 0 prints one JSON line.

Workload (BASELINE.json configs[1]): SceneFlow 576x960, maxdisp 192, fp32, batch 1
per GPU; random-init weights of the reference architecture (leastereo_amd.weights
recipe; no checkpoints exist upstream) and synthetic N(0,1) images (the
post-standardisation statistics of predict.py:162-184).  ``--config c3|c4|c5`` picks
the other BASELINE configs (c4 = 8 pairs per GPU of the 64-pair global batch).

Extras in the JSON line:
  roofline       the dominant conv kernel instantiation timed with HIP events inside
                 the timed region; ``achieved`` counts the MFMA products the kernel
                 issues (Winograd products, padded cout blocks), so ``frac`` is the
                 matrix-core utilisation; the direct-convolution equivalent is a
                 separate key
  path_roofline  sum over every launch of one forward of max(issued MFMA FLOP / peak,
                 VALU FLOP / peak, algorithmic bytes / 8 TB/s), for the algorithms
                 actually run, over the measured step time; plus the HBM-only fraction
  pair_epe_px    per pair of every rank's shard: |HIP - a second HIP path| (f32: the
                 matching net on the direct-conv engine over the in-place cost volume, the
                 feature net's 3x3 convs on the DMA/MFMA engine with unfused stems, the
                 gather resample and the LDS disparity kernel -- only the streamed 1x1
                 kernel is common; bf16: the f32 path on those engines), all-gathered
                 over ranks (the data path's one collective)
  epe_px         per rank: HIP vs the reference's own fp32 output (golden e2e case)
  cpu_baseline   the CPU oracle (oracle/torch_ref.py, the reference's aten op sequence
                 restated) on the host's physical cores, rank 0, N = 1: C2 (this
                 workload's first pair) and C1 (the SceneFlow sample pair), 1 warm-up +
                 3 timed each, HIP-vs-CPU and HIP-vs-fp64 EPE
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import platform
import socket
import subprocess
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
FP32_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md: fp32 matrix = fp32 vector, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, bf16 dense (no sparsity)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, spec

# BASELINE.json configs: c2 is the headline workload (defaults);
# c3/c4 are the bf16 ones (c4 = 8 pairs per GPU of the 64-pair global batch)
CONFIGS = {
    "c2": dict(height=576, width=960, maxdisp=192, batch=1, precision="f32"),
    "c3": dict(height=384, width=1248, maxdisp=192, batch=8, precision="bf16"),
    "c4": dict(height=576, width=960, maxdisp=192, batch=8, precision="bf16"),
    "c5": dict(height=1008, width=1512, maxdisp=264, batch=1, precision="f32"),
}
# SURVEY.md §8d's roofline of the reference algorithm (direct convolutions, a
# materialised cost volume): kept for comparison beside the issued-work roofline
T_ROOF_REFERENCE_MS = {("c2", 1): 11.36, ("c3", 8): 10.91, ("c4", 8): 12.59, ("c5", 1): 43.1}
# BASELINE.md §3's HBM-only time of the reference algorithm (its ConvBR-fused accounting: conv
# in + out + weights once, resample in + out, one operand per cell sum; the materialised
# cost volume excluded) -- the denominator BASELINE.md states the ">= 55 %" bar against
HBM_ONLY_REFERENCE_MS = {("c2", 1): 2.67, ("c3", 8): 9.25, ("c4", 8): 10.68, ("c5", 1): 10.12}
WORKLOADS = {"c2": "SceneFlow 576x960 D=192 fp32, batch 1 per GPU (BASELINE configs[1])",
             "c3": "KITTI2015 384x1248 D=192 bf16, batch 8 (BASELINE configs[2])",
             "c4": "SceneFlow 576x960 D=192 bf16, 8 pairs per GPU (BASELINE configs[3])",
             "c5": "Middlebury 1008x1512 D=264 fp32, batch 1 (BASELINE configs[4], D256 is illegal)"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=1, help="pairs per GPU per step")
    p.add_argument("--height", type=int, default=576)
    p.add_argument("--width", type=int, default=960)
    p.add_argument("--maxdisp", type=int, default=192)
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle (rank 0, N=1)")
    p.add_argument("--cpu-timed", type=int, default=3, help="timed CPU forwards per config (+1 warm-up)")
    p.add_argument("--cpu-configs", default="c2,c1", help="CPU baseline configs (c2 = this workload)")
    p.add_argument("--cpu-fp64", type=int, default=1, help="HIP vs a float64 CPU forward at C2")
    p.add_argument("--gpu-eager", default="default",
                   help="torch-ROCm GPU-eager leg of the reference op sequence at C1 (BASELINE.md §4), "
                        "comma list of MIOpen modes: default (immediate mode) and/or benchmark "
                        "(torch.backends.cudnn.benchmark: MIOpen find per shape); empty to skip")
    p.add_argument("--gpu-eager-c2", type=int, default=0,
                   help="1: the GPU-eager leg at the timed workload too (first pair, 1 warm-up + 1 timed "
                        "forward per mode)")
    p.add_argument("--epe", type=int, default=1, help="check EPE vs the reference golden disparity")
    p.add_argument("--pair-check", type=int, default=1,
                   help="per-pair EPE of every rank's shard vs an independent HIP path, all-gathered")
    p.add_argument("--breakdown", type=int, default=0, help="print per-kernel times to stderr")
    p.add_argument("--graph", type=int, default=1,
                   help="1: time a HIP-graph replay of the forward (LEAStereo.graphed: one host call per "
                        "step, same kernels; same-box A/B at C2 +1.2 %%, profiles/r03_graph_ab.txt); "
                        "0: eager launches")
    p.add_argument("--precision", choices=("f32", "bf16"), default="f32",
                   help="matching-net arithmetic (bf16 = BASELINE configs 3/4)")
    p.add_argument("--config", choices=sorted(CONFIGS), default=None,
                   help="preset: c2 (default workload) / c3 / c4 (per GPU) / c5 of BASELINE.json")
    p.add_argument("--extra-configs", default="auto",
                   help="BASELINE configs timed after the headline one (graph replays, no CPU legs), "
                        "comma list; auto = c3,c5 at N = 1 and c4 at N > 1; empty to skip")
    p.add_argument("--extra-steps", type=int, default=10, help="timed steps per extra config")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="N > 1 process group: nccl (= RCCL over xGMI) or gloo (rehearsal of the N-rank "
                        "path on fewer GPUs: every rank on cuda:0 when the box has fewer GPUs than ranks)")
    p.add_argument("--stub", type=int, default=0, help=argparse.SUPPRESS)  # tests: no GPU, gloo
    a = p.parse_args(argv)
    if a.config:
        for k, v in CONFIGS[a.config].items():
            setattr(a, k, v)
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv) -> int:
    """Start ``n`` ranks of this script under torch.distributed.run (one process per
    GPU, rendezvous on 127.0.0.1) as a child process and return its exit status.
    Runs before anything in this process touches a GPU (no exec from here)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------ models
@contextlib.contextmanager
def independent_check_engines():
    """The per-pair check's engines (bench.py's pair_epe_px): every switchable kernel the timed
    path runs swapped for its alternative -- the feature net's few-channel 3x3 tile and pair
    launch (lea_conv2d_set_small(0), FeatureExecutor.PAIR_S0), the fused stems (FUSED_STEM),
    the separable resample (lea_resample_set_mode(2): the per-output gather), the fused tap-sum
    head (lea_tapsum_set_rows(0): pass 1 through the workspace, then the per-row gather pass)
    and the row-staged disparity kernel (the online-softmin LDS kernel).  The process-wide settings go back to
    what the LEASTEREO_* environment (or the default) set afterwards."""
    from leastereo_amd import _lib, executor
    lib = _lib.load()
    fe = executor.FeatureExecutor
    saved = (fe.FUSED_STEM, fe.PAIR_S0)
    env = lambda var, default: int(os.environ.get(var) or default)  # noqa: E731
    switches = (("lea_disparity_set_register_form", 0, "LEASTEREO_DISP_REG", 4),
                ("lea_conv2d_set_small", 0, "LEASTEREO_CONV2D_SMALL", 1),
                ("lea_resample_set_mode", 2, "LEASTEREO_RESAMPLE_MODE", 0),
                ("lea_tapsum_set_rows", 0, "LEASTEREO_TAPSUM_ROWS", 2))
    try:
        for fn, value, _, _ in switches:
            _lib.check(getattr(lib, fn)(value), fn)
        fe.FUSED_STEM, fe.PAIR_S0 = False, False
        yield
    finally:
        fe.FUSED_STEM, fe.PAIR_S0 = saved
        for fn, _, var, default in switches:
            _lib.check(getattr(lib, fn)(env(var, default)), fn)


def build_model(maxdisp, device, precision="f32"):
    args = default_arch_args(LEAStereoArgs(maxdisp=maxdisp))
    model = LEAStereo(args, device, precision=precision)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    model.load_state_dict(synthetic_state_dict(shapes), strict=True)
    return model.to(device).eval()


def config_name(args):
    return next((k for k, v in CONFIGS.items() if all(getattr(args, f) == x for f, x in v.items())), None)


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


# ------------------------------------------------------------------------ CPU baseline
def host_cores():
    """Physical cores this process may use: the distinct (package, core) pairs of the
    CPUs in its affinity mask, capped by the cgroup CPU quota (a container's share of
    a large host), plus the CPU model (lscpu's "Model name")."""
    aff = sorted(os.sched_getaffinity(0))
    phys = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            with open(base + "core_id") as f:
                phys.add((pkg, f.read().strip()))
        except OSError:
            phys.add(("?", str(c)))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    use = len(phys) if quota is None else min(len(phys), quota)
    return {"threads": use, "physical_cores_in_affinity": len(phys), "logical_cpus_in_affinity": len(aff),
            "cgroup_cpu_quota": quota, "model": model}


def rank_threads(world: int) -> int:
    """Host threads per rank: the physical cores the process may use split over the
    node's ranks (8 ranks on a 16-core share would otherwise each start 16 threads
    for the model build and the pair check)."""
    return max(1, host_cores()["threads"] // max(1, world))


def gather_step_stats(step_ms, device):
    """All-gather every rank's (median, p10, p90) step time [ms] so a straggler shows
    up in rank 0's line; [] per rank in rank order."""
    mine = torch.tensor([_quantile(step_ms, 0.5), _quantile(step_ms, 0.1), _quantile(step_ms, 0.9)],
                        dtype=torch.float64, device=device)
    allv = parallel.gather_per_pair(mine).view(-1, 3).cpu()
    return [{"rank": r, "median": float(v[0]), "p10": float(v[1]), "p90": float(v[2])}
            for r, v in enumerate(allv)]


def _time_cpu(fn, timed):
    fn()  # warm-up
    t0 = time.perf_counter()
    for _ in range(timed):
        out = fn()
    return (time.perf_counter() - t0) / timed, out


def _time_hip(model, left, right, n=20):
    with torch.no_grad():
        for _ in range(3):
            model(left, right)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            out = model(left, right)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n, out


def cpu_baseline(args, model, left0, right0, disp0, hip_step_s, device):
    """CPU leg: the oracle (oracle/torch_ref.py, the reference's aten
    op sequence restated) on the host's physical cores, 1 warm-up + ``--cpu-timed``
    forwards per config, fp32, B = 1, beside the HIP path on the same inputs.  C2 is
    this benchmark's first pair; C1 is predict.py's preprocessing of the reference's
    SceneFlow sample pair (tests/golden/c1_sceneflow.npz) at 288x576 D96."""
    from oracle import torch_ref as ref
    cores = host_cores()
    torch.set_num_threads(cores["threads"])
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    a = arch_arrays()
    res = {"kind": "port", "unit": "pairs/s", "cores": cores["threads"], "host": cores, "configs": {}}
    cfgs = [c for c in args.cpu_configs.split(",") if c]
    with torch.no_grad():
        for cfg in cfgs:
            if cfg == "c2" or cfg == config_name(args):
                l, r, md = left0.cpu(), right0.cpu(), args.maxdisp
                hip_out, hip_s = disp0.cpu(), hip_step_s / args.batch
                tag = f"{args.height}x{args.width} D={args.maxdisp}"
            elif cfg == "c1":
                from tests.golden_util import c1_inputs
                l, r = c1_inputs()
                md = 96
                m1 = build_model(md, device, "f32")
                hip_s, hip_out = _time_hip(m1, l.to(device), r.to(device))
                hip_out = hip_out.cpu()
                tag = "SceneFlow sample pair 0001 (predict.py preprocessing), 288x576 D=96"
            else:
                raise ValueError(f"unknown CPU baseline config {cfg}")
            s_pair, want = _time_cpu(lambda: ref.leastereo_forward(sd, l, r, md, a), args.cpu_timed)
            entry = {"workload": tag, "cpu_s_per_pair": s_pair, "cpu_pairs_s": 1.0 / s_pair,
                     "hip_pairs_s": 1.0 / hip_s, "hip_vs_cpu_speedup": s_pair / hip_s,
                     "epe_px_hip_vs_cpu_f32": ref.epe(hip_out, want),
                     "timing": f"1 warm-up + {args.cpu_timed} timed forwards, B=1 fp32"}
            if args.cpu_fp64 and cfg == "c2":
                sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
                t0 = time.perf_counter()
                want64 = ref.leastereo_forward(sd64, l.double(), r.double(), md, a)
                entry["fp64_s"] = time.perf_counter() - t0
                entry["epe_px_hip_vs_fp64"] = ref.epe(hip_out, want64)
                entry["epe_px_cpu_f32_vs_fp64"] = ref.epe(want, want64)
            res["configs"][cfg] = entry
        modes = [m for m in args.gpu_eager.split(",") if m]
        if modes:
            c2 = None
            if args.gpu_eager_c2:
                c2 = (left0, right0, args.maxdisp, hip_step_s / args.batch, disp0,
                      f"{args.height}x{args.width} D={args.maxdisp}")
            res["torch_gpu_eager"] = gpu_eager_baseline(sd, a, device, modes, args.cpu_timed, c2)
    head = res["configs"].get("c2") or next(iter(res["configs"].values()))
    res["value"] = head["cpu_pairs_s"]
    res["sample"] = (f"oracle/torch_ref.py on torch CPU ({cores['model']}, {cores['threads']} threads = "
                     f"physical cores available to the process), {head['timing']}: "
                     + "; ".join(f"{k}: {v['workload']}" for k, v in res["configs"].items()))
    return res


def gpu_eager_baseline(sd, arch, device, modes, timed, c2=None):
    """BASELINE.md §4's torch-ROCm GPU-eager column: the reference's aten op sequence
    (oracle/torch_ref.py, as predict.py:227-229 runs the model) on this GPU through
    MIOpen, fp32 (no TF32), at C1 -- the SceneFlow sample pair, 288x576 D96 -- beside
    the HIP path on the same pair.  ``c2`` = (left, right, maxdisp, hip_s, hip_out, tag):
    the same at the timed workload's first pair (``--gpu-eager-c2 1``), 1 warm-up + 1 timed
    forward per mode -- MIOpen's 3D convolutions at 576x960 D192 take seconds per forward."""
    from oracle import torch_ref as ref
    from tests.golden_util import c1_inputs
    l, r = (t.to(device) for t in c1_inputs())
    sd_dev = {k: v.to(device) for k, v in sd.items()}
    hip_s, hip_out = _time_hip(build_model(96, device, "f32"), l, r)
    out = _eager_modes(ref, sd_dev, arch, l, r, 96, hip_s, hip_out, modes, timed)
    out["workload"] = "SceneFlow sample pair 0001 (predict.py preprocessing), 288x576 D=96, B=1 fp32"
    if c2 is not None:
        l2, r2, md2, hip2_s, hip2_out, tag = c2
        out["c2"] = _eager_modes(ref, sd_dev, arch, l2, r2, md2, hip2_s, hip2_out, modes, 1, warm_default=1,
                                 warm_benchmark=1)
        out["c2"]["workload"] = tag + ", the timed workload's first pair, B=1 fp32"
    del sd_dev
    torch.cuda.empty_cache()
    return out


def _eager_modes(ref, sd_dev, arch, l, r, md, hip_s, hip_out, modes, timed, warm_default=1, warm_benchmark=3):
    out = {"hip_pairs_s": 1.0 / hip_s, "modes": {}}
    prev = torch.backends.cudnn.benchmark
    try:
        for mode in modes:
            torch.backends.cudnn.benchmark = mode == "benchmark"
            # benchmark: MIOpen's find on the first call(s)
            warm = warm_default if mode == "default" else warm_benchmark
            log(f"gpu-eager {tuple(l.shape)} D{md} mode={mode}: {warm} warm-up + {timed} timed")
            t0 = time.perf_counter()
            with torch.no_grad():
                for _ in range(warm):
                    ref.leastereo_forward(sd_dev, l, r, md, arch)
                torch.cuda.synchronize()
                t_warm = time.perf_counter() - t0
                t0 = time.perf_counter()
                for _ in range(timed):
                    want = ref.leastereo_forward(sd_dev, l, r, md, arch)
                torch.cuda.synchronize()
            s = (time.perf_counter() - t0) / timed
            out["modes"][mode] = {
                "pairs_s": 1.0 / s, "s_per_pair": s, "warmup_s": t_warm,
                "hip_vs_eager_speedup": s / hip_s, "epe_px_hip_vs_eager": ref.epe(hip_out, want),
                "timing": f"{warm} warm-up + {timed} timed forwards, torch.backends.cudnn.benchmark="
                          f"{mode == 'benchmark'}, allow_tf32=False"}
            del want
    finally:
        torch.backends.cudnn.benchmark = prev
    return out


# ------------------------------------------------------------------------ roofline
def algorithm_name(kernel: str) -> str:
    """The convolution algorithm a conv kernel instantiation runs."""
    if kernel.startswith("conv3d_wino44"):
        return "winograd F(4,3) along W x F(4,3) along D"
    if kernel.startswith("conv3d_wino2"):
        return "winograd F(4,3) along W x F(2,3) along D"
    if kernel.startswith("conv3d_wino_kernel<"):
        return f"winograd F({kernel.split('<')[1].split(',')[0]},3) along W"
    return "direct convolution"


def _matrix_peak(name: str) -> float:
    return BF16_MFMA_PEAK_TFLOPS if ("bf16" in name or "c8" in name) else FP32_PEAK_TFLOPS


def path_roofline(records):
    """T_roof of one forward for the algorithms it runs: per launch max(issued MFMA FLOP
    / matrix peak, VALU FLOP / fp32 peak, algorithmic bytes / HBM peak), summed; and
    the HBM-only time (sum of bytes / HBM peak)."""
    t_roof = t_hbm = t_mat = 0.0
    for name, flops, nbytes, _e0, _e1, mfma, _shape in records:
        t_m = mfma / (_matrix_peak(name) * 1e12) if mfma else flops / (FP32_PEAK_TFLOPS * 1e12)
        t_b = nbytes / (HBM_PEAK_GBS * 1e9)
        t_roof += max(t_m, t_b)
        t_hbm += t_b
        t_mat += t_m
    return t_roof * 1e3, t_hbm * 1e3, t_mat * 1e3, len(records)


def _quantile(xs, q):
    """Linear-interpolated quantile of a sorted list."""
    pos = q * (len(xs) - 1)
    i = int(pos)
    j = min(i + 1, len(xs) - 1)
    return xs[i] + (xs[j] - xs[i]) * (pos - i)


# ------------------------------------------------------------------------ ranks
def run_stub(args, info):
    """Launcher / sharding / gather plumbing with a CPU step (tests, gloo): each rank
    'processes' its shard of world*batch pairs and reports pair index * 1e-3 as its
    per-pair value, so the gathered vector shows the order the ranks' shards land in."""
    parallel.init("gloo", info, None)
    threads = rank_threads(info.world)
    torch.set_num_threads(threads)
    shard = parallel.shard(info.world * args.batch, info)
    parallel.barrier()
    t0 = time.perf_counter()
    step_ms = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        torch.zeros(args.batch, 8, 8).add_(1.0)
        step_ms.append((time.perf_counter() - ts) * 1e3 + 10.0 * info.rank)  # rank-tagged: order check
    parallel.barrier()
    elapsed = parallel.max_over_ranks(time.perf_counter() - t0, torch.device("cpu"))
    per_rank = gather_step_stats(sorted(step_ms), torch.device("cpu"))
    all_threads = parallel.gather_per_pair(torch.tensor([torch.get_num_threads()], dtype=torch.int64))
    per_pair = parallel.gather_per_pair(torch.tensor([i * 1e-3 for i in shard], dtype=torch.float32))
    shards = parallel.gather_per_pair(torch.tensor([shard.start, shard.stop], dtype=torch.int64))
    if info.is_main:
        print(json.dumps({"metric": METRIC, "value": info.world * args.batch * args.steps / max(elapsed, 1e-9),
                          "unit": "pairs/s", "n_gpus": info.world, "steps": args.steps, "stub": True,
                          "shards": shards.view(-1, 2).tolist(),
                          "per_rank_step_ms": per_rank, "threads_per_rank": all_threads.tolist(),
                          "host_threads": host_cores()["threads"],
                          "pair_epe_px": {"per_pair": [float(v) for v in per_pair]}}), flush=True)
    parallel.finalize()


def measure(a, info, device, *, steps, warmup, pair_check, epe):
    """One configuration on this rank: build the model, capture the forward (``a.graph``),
    ``warmup`` untimed steps, one probed eager forward (the path roofline and the dominant
    conv kernel), then EXACTLY ``steps`` timed steps bracketed by barrier + synchronize on
    both sides, the max over ranks; after the timed region the per-pair check of this
    rank's shard and the golden EPE.  Returns the pieces ``run`` assembles."""
    world, rank = info.world, info.rank
    model = build_model(a.maxdisp, device, a.precision)
    model.check_shape(a.height, a.width)
    # weak scaling: rank r owns pairs shard(r) of the world*batch global batch, generated
    # on its own device from a rank-seeded stream
    shard = parallel.shard(world * a.batch, info)
    assert len(shard) == a.batch
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    left = torch.randn(a.batch, 3, a.height, a.width, device=device, generator=g)
    right = torch.randn(a.batch, 3, a.height, a.width, device=device, generator=g)

    def step():
        return model(left, right)

    if a.graph:
        graphed = model.graphed(a.batch, a.height, a.width)

        def step():  # noqa: F811  (inputs already resident: replay only)
            graphed.graph.replay()
            return graphed.out
        graphed.x.copy_(left)
        graphed.y.copy_(right)

    with torch.no_grad():
        for _ in range(max(warmup, 1)):
            out = step()
        # every launch of one (untimed) eager forward: the path roofline, and the
        # dominant conv kernel instantiation
        with kernels.KernelProbe() as probe:
            model(left, right)
        per_kernel = probe.summary()
        t_roof_ms, t_hbm_ms, t_mat_ms, n_launch = path_roofline(probe.records)
        convs = {n: d for n, d in per_kernel.items() if d["mfma_flops"] > 0}
        dominant = max(convs, key=lambda n: convs[n]["ms"])
        if getattr(a, "breakdown", 0) and info.is_main:
            for n, d in sorted(per_kernel.items(), key=lambda kv: -kv[1]["ms"]):
                log(f"{n:48s} launches {d['launches']:3d}  {d['ms']:8.3f} ms  "
                    f"{d['mfma_flops'] / d['ms'] / 1e9:8.1f} TFLOP/s issued  "
                    f"{d['bytes'] / d['ms'] / 1e6:8.1f} GB/s")

        parallel.barrier()
        torch.cuda.synchronize()
        with kernels.KernelProbe([dominant]) as probe:
            # per-step latency: HIP events between consecutive steps (SURVEY §8d's
            # median and p10/p90), on the stream the forward is launched on
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
            t0 = time.perf_counter()
            ev[0].record()
            for i in range(steps):
                out = step()
                ev[i + 1].record()
            torch.cuda.synchronize()
            parallel.barrier()
            elapsed = time.perf_counter() - t0
        if a.graph:  # replays bypass the launch-time probe: time one eager forward after
            with kernels.KernelProbe([dominant]) as probe:
                model(left, right)
        dom = probe.summary()[dominant]
        dom_shapes = probe.by_shape(dominant)
        step_ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
    elapsed = parallel.max_over_ranks(elapsed, device)
    per_rank_steps = gather_step_stats(step_ms, device)

    # after the timed region: the per-pair check of this rank's shard against an
    # independent HIP path, then the data path's one collective (all-gather over ranks)
    pair = None
    if pair_check:
        ref_prec = "f32_direct" if a.precision == "f32" else "f32"
        with independent_check_engines():
            with torch.no_grad():
                check = build_model(a.maxdisp, device, ref_prec)(left, right)
                torch.cuda.synchronize()
        e = (out.double() - check.double()).abs().mean(dim=(1, 2)).float()
        del check
        per_pair = [float(v) for v in parallel.gather_per_pair(e).cpu()]
        pair = {"vs": ("HIP f32 on engines the timed path does not run: the matching net on the "
                       "direct-conv engine over the in-place cost volume (no Winograd, no factored "
                       "stem0), the feature net's 3x3 convs on the DMA/MFMA engine (no few-channel "
                       "tile, no pair launch) with unfused stems, the per-output gather resample and "
                       "the online-softmin LDS disparity kernel; only the streamed 1x1 conv kernel "
                       "is common to both" if a.precision == "f32" else
                       "HIP f32 path, same weights, the feature net's 3x3 convs on the DMA/MFMA engine "
                       "with unfused stems, the per-output gather resample, online-softmin LDS "
                       "disparity kernel"),
                "pairs": world * a.batch, "max": max(per_pair), "mean": sum(per_pair) / len(per_pair),
                "per_pair": per_pair}
    epe_v = None
    if epe:
        e = torch.tensor([golden_epe(device, a.precision)], device=device, dtype=torch.float32)
        epe_v = [float(v) for v in parallel.gather_per_pair(e).cpu()]
    return dict(model=model, left=left, right=right, out=out, elapsed=elapsed, step_ms=step_ms,
                per_rank_steps=per_rank_steps, dominant=dominant, dom=dom, dom_shapes=dom_shapes,
                t_roof_ms=t_roof_ms, t_hbm_ms=t_hbm_ms, t_mat_ms=t_mat_ms, n_launch=n_launch,
                pair=pair, epe=epe_v, steps=steps)


def roofline_fields(a, m):
    """The dominant kernel's ``roofline`` and the forward's ``path_roofline`` objects of a
    measured configuration (``measure``)."""
    dominant, dom, dom_shapes = m["dominant"], m["dom"], m["dom_shapes"]
    launches = dom["launches"]
    ms_per_launch = dom["ms"] / launches
    issued = dom["mfma_flops"] / launches
    direct = dom["flops"] / launches
    peak = BF16_MFMA_PEAK_TFLOPS if a.precision == "bf16" else FP32_PEAK_TFLOPS
    achieved = issued / (ms_per_launch * 1e-3) / 1e12
    alg_bytes = dom["bytes"] / launches  # inputs + output (+ residual) + weights, once
    traffic = None
    cfg = config_name(a)
    tf_file = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if os.path.exists(tf_file):
        with open(tf_file) as f:
            tf = json.load(f)
        # per-config entries (tools/traffic_merge.py); the plain entries are the c2 workload's
        # (bytes per launch depend on the shapes)
        entry = tf.get(f"{dominant}@{cfg}") or (tf.get(dominant) if cfg == "c2" else None) or {}
        traffic = entry.get("bytes_per_launch")
    ms_step = m["elapsed"] / m["steps"] * 1e3
    probed_steps = 1 if a.graph else m["steps"]  # forwards the dominant kernel's probe saw
    roof = {"bound": "mfma", "kernel": dominant, "algorithm": algorithm_name(dominant),
            "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
            "traffic": traffic, "algorithmic_bytes_per_launch": alg_bytes,
            "traffic_over_algorithmic": None if traffic is None else traffic / alg_bytes,
            "work": "MFMA FLOPs the kernel issues per launch (Winograd products, cout "
                    "padded to its blocks); DESIGN.md §4 gives the per-launch formula",
            "flops_per_launch": issued, "ms_per_launch": ms_per_launch,
            "launches_per_step": launches / probed_steps,
            "timed_over": "one eager forward after the timed graph replays (replays bypass "
                          "the launch probe)" if a.graph else "every step of the timed region",
            "by_shape": [{"shape": "B%d %d->%d @ %dx%dx%d k%d" % sh if sh else None,
                          "launches_per_step": d["launches"] / probed_steps,
                          "ms_per_launch": d["ms"] / d["launches"],
                          "issued_tflops": d["mfma_flops"] / d["ms"] / 1e9,
                          "frac": d["mfma_flops"] / d["ms"] / 1e9 / peak}
                         for sh, d in sorted(dom_shapes.items(), key=lambda kv: -kv[1]["ms"])],
            "direct_equivalent": {"flops_per_launch": direct,
                                  "achieved": direct / (ms_per_launch * 1e-3) / 1e12,
                                  "issued_per_direct_flop": issued / direct,
                                  "note": "the reference algorithm's (direct convolution's) "
                                          "FLOPs for the same outputs; not a utilisation.  A "
                                          "Winograd tile that issues fewer products per output "
                                          "lowers frac at equal speed: compare kernels by time "
                                          "or by this rate (DESIGN.md §4 Round 6)"}}
    path = {"t_roof_ms": m["t_roof_ms"], "frac": m["t_roof_ms"] / ms_step,
            "hbm_only_ms": m["t_hbm_ms"], "hbm_frac": m["t_hbm_ms"] / ms_step,
            "hbm_frac_rule": "bytes this implementation's kernels must move (each launch's "
                             "inputs + output + residual + weights once; the factored stem0 "
                             "and fused layers as run) / 8 TB/s, over the step",
            "hbm_frac_baseline_accounting": (
                None if HBM_ONLY_REFERENCE_MS.get((cfg, a.batch)) is None else
                HBM_ONLY_REFERENCE_MS[(cfg, a.batch)] / ms_step),
            "hbm_frac_baseline_rule": "BASELINE.md §3: the reference algorithm's ConvBR-fused "
                                      "bytes (C2 21.36 GB fp32, C3 74.0 / C4 85.4 GB per 8 "
                                      "pairs bf16) / 8 TB/s, over the step",
            "matrix_only_ms": m["t_mat_ms"], "launches": m["n_launch"],
            "source": "one eager forward: sum over its launches of max(issued MFMA FLOP / "
                      "peak, VALU FLOP / fp32 peak, algorithmic bytes / 8 TB/s)",
            "reference_algorithm_t_roof_ms": T_ROOF_REFERENCE_MS.get((cfg, a.batch))}
    return roof, path


def extra_legs(args, world):
    """BASELINE configs timed after the headline leg: at N = 1 the bf16
    KITTI batch (c3) and Middlebury (c5); at N > 1 config 4 (bf16, 8 pairs per GPU), the
    one BASELINE.md §4 names for the scaling curve.  The headline config is never repeated."""
    if args.extra_configs != "auto":
        names = [c for c in args.extra_configs.split(",") if c]
    else:
        names = ["c3", "c5"] if world == 1 else ["c4"]
    return [c for c in names if c != config_name(args)]


def leg_args(args, cfg):
    a = argparse.Namespace(**vars(args))
    for k, v in CONFIGS[cfg].items():
        setattr(a, k, v)
    return a


def run(args, info):
    world = info.world
    backend = args.dist_backend
    if backend == "gloo" and torch.cuda.device_count() < world:
        # gloo rehearsal of the N-rank path on a box with fewer GPUs (tests/test_gpu_bench.py):
        # every rank on cuda:0; the device tensors' collectives go through host copies
        device = torch.device("cuda", 0)
    else:
        device = torch.device("cuda", info.local_rank)
    if world > 1:
        torch.cuda.set_device(device)
    parallel.init(backend, info, device)  # nccl = RCCL over xGMI on ROCm
    torch.set_num_threads(rank_threads(world))  # the cpu_baseline leg (N = 1) resets it
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False

    m = measure(args, info, device, steps=args.steps, warmup=args.warmup,
                pair_check=args.pair_check, epe=args.epe)
    roof, path = roofline_fields(args, m)
    ms_step = m["elapsed"] / args.steps * 1e3
    step_ms = m["step_ms"]
    cfg = config_name(args)
    bf16 = args.precision == "bf16"
    workload = WORKLOADS.get(cfg, f"{args.height}x{args.width} D={args.maxdisp} {args.precision}, "
                                  f"batch {args.batch} per GPU")
    result = {
        "metric": METRIC,
        "value": world * args.batch * args.steps / m["elapsed"],
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "step_ms": {"median": _quantile(step_ms, 0.5), "p10": _quantile(step_ms, 0.1),
                    "p90": _quantile(step_ms, 0.9), "source": "HIP events between steps, this rank"},
        "per_rank_step_ms": m["per_rank_steps"],
        "host_threads_per_rank": torch.get_num_threads(),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic N(0,1) stereo pairs generated on device; random-init weights of the "
                "reference architecture (SceneFlow search result)",
        "config": {"workload": workload,
                   "height": args.height, "width": args.width, "maxdisp": args.maxdisp,
                   "global_batch": world * args.batch,
                   "parallelism": f"dp{world} (pairs sharded over ranks, no collective in the step)",
                   "launch": "hip graph replay" if args.graph else "eager",
                   "dist_backend": backend if world > 1 else None},
        "roofline": roof,
        "path_roofline": path,
        "pair_epe_px": m["pair"],
        "epe_px": None if m["epe"] is None else {
            "vs": "reference LEAStereo fp32 disparity (tests/golden e2e b1_h96_w192_md48)"
                  + (" (bf16 matching net: no upstream tolerance; see DESIGN.md)" if bf16 else ""),
            "max_over_ranks": max(m["epe"]), "per_rank": m["epe"]},
    }
    if info.is_main and world == 1 and args.cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, m["model"], m["left"][:1], m["right"][:1], m["out"][:1],
                                              float(_quantile(step_ms, 0.5)) * 1e-3, device)
        torch.set_num_threads(rank_threads(world))
    legs = extra_legs(args, world)
    if legs:
        del m
        torch.cuda.empty_cache()
        result["configs"] = {}
    for name in legs:
        # the other BASELINE configs on the same box in the same run (top-level fields stay
        # the headline config's): graph replays only, no CPU or eager legs; at N > 1 the
        # per-pair check and its all-gather run too (north_star's one RCCL gather of per-pair EPE)
        a = leg_args(args, name)
        lm = measure(a, info, device, steps=args.extra_steps, warmup=2, pair_check=world > 1, epe=False)
        lroof, lpath = roofline_fields(a, lm)
        lms = lm["elapsed"] / args.extra_steps * 1e3
        result["configs"][name] = {
            "workload": WORKLOADS[name], "value": world * a.batch * args.extra_steps / lm["elapsed"],
            "unit": "pairs/s", "dtype": a.precision, "global_batch": world * a.batch,
            "steps": args.extra_steps, "warmup": 2, "ms_per_step": lms,
            "step_ms": {"median": _quantile(lm["step_ms"], 0.5), "p10": _quantile(lm["step_ms"], 0.1),
                        "p90": _quantile(lm["step_ms"], 0.9)},
            "per_rank_step_ms": lm["per_rank_steps"],
            "roofline": {k: lroof[k] for k in ("kernel", "achieved", "peak", "unit", "frac", "traffic",
                                               "traffic_over_algorithmic", "ms_per_launch",
                                               "launches_per_step", "by_shape")},
            "path_roofline": {k: lpath[k] for k in ("t_roof_ms", "frac", "hbm_frac",
                                                    "hbm_frac_baseline_accounting")},
            "pair_epe_px": lm["pair"],
            "timing": f"{args.extra_steps} timed graph replays after 2 warm-up, barrier + synchronize "
                      "on both sides, max over ranks"}
        del lm
        torch.cuda.empty_cache()
    if info.is_main:
        print(json.dumps(result), flush=True)
    parallel.finalize()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, argv))
    info = parallel.rank_info()
    if info.world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but the launcher started {info.world} rank(s)")
        sys.exit(2)
    (run_stub if args.stub else run)(args, info)


if __name__ == "__main__":
    main()
