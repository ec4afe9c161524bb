"""Multi-process (world_size 2, gloo on CPU) tests of the batch-parallel plumbing
bench.py uses on MI355X with RCCL: sharding, max-over-ranks timing and the single
all-gather of per-pair EPE."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from leastereo_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        info = parallel.rank_info()
        parallel.init("gloo", info)
        sh = parallel.shard(8 * world, info)
        t = parallel.max_over_ranks(1.0 + rank, torch.device("cpu"))
        per_pair = torch.arange(len(sh), dtype=torch.float32) + 100 * rank
        allp = parallel.gather_per_pair(per_pair)
        parallel.barrier()
        q.put((rank, list(sh), t, allp.tolist()))
        parallel.finalize()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, "error", repr(e), None))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shard_time_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res), res
    shards = [r[1] for r in res]
    assert sum(shards, []) == list(range(8 * world))       # disjoint, complete, ordered
    assert all(r[2] == float(world) for r in res)           # max over ranks
    expect = sum(([100 * r + i for i in range(8)] for r in range(world)), [])
    assert all(r[3] == expect for r in res)                  # rank-ordered gather on all ranks


def test_single_process_defaults():
    info = parallel.RankInfo(0, 1, 0)
    assert list(parallel.shard(5, info)) == [0, 1, 2, 3, 4]
    assert parallel.max_over_ranks(2.5, torch.device("cpu")) == 2.5
    x = torch.ones(3)
    assert parallel.gather_per_pair(x) is x
    assert not dist.is_initialized()


# ---- bench.py's own launcher (the entry the driver and users start) ----
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=REPO)


@pytest.mark.parametrize("world,batch", [(2, 4), (3, 2)])
def test_bench_launcher_spawns_ranks_and_gathers(world, batch):
    """``python bench.py --gpus N`` (no torchrun env) starts N ranks itself; every rank
    takes its contiguous shard of world*batch pairs and rank 0 prints the gathered
    per-pair vector in rank order (stub step: no GPU, gloo)."""
    import json
    r = _bench("--gpus", str(world), "--batch", str(batch), "--steps", "3", "--stub", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["stub"]
    assert d["shards"] == [[k * batch, (k + 1) * batch] for k in range(world)]
    assert d["pair_epe_px"]["per_pair"] == pytest.approx([i * 1e-3 for i in range(world * batch)])
    # every rank's step statistics reach rank 0 in rank order (the stub tags rank r's
    # step times with +10 r ms: a first torch op can take milliseconds), and the host threads are split over the ranks
    per_rank = d["per_rank_step_ms"]
    assert [p["rank"] for p in per_rank] == list(range(world))
    assert all(10 * r <= p["median"] < 10 * r + 9 and p["p10"] <= p["median"] <= p["p90"]
               for r, p in enumerate(per_rank)), per_rank
    assert d["threads_per_rank"] == [max(1, d["host_threads"] // world)] * world


def test_bench_refuses_world_size_mismatch():
    """A rank whose launcher started a different world than --gpus says exits non-zero."""
    r = _bench("--gpus", "2", "--stub", "1", "--steps", "1",
               env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "--gpus 2" in r.stderr


def test_bench_parse_presets():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = bench.parse(["--config", "c4"])
    assert (a.height, a.width, a.maxdisp, a.batch, a.precision) == (576, 960, 192, 8, "bf16")
    assert bench.config_name(a) == "c4"
    a = bench.parse([])
    assert bench.config_name(a) == "c2" and a.gpus == 1
    # host core accounting is self-consistent
    h = bench.host_cores()
    assert 1 <= h["threads"] <= h["logical_cpus_in_affinity"]
    assert h["physical_cores_in_affinity"] <= h["logical_cpus_in_affinity"]


def test_bench_extra_legs():
    """The configs timed after the headline one: c3 + c5 at N = 1, c4 at
    N > 1, never the headline config itself; an explicit list or none on request."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.extra_legs(bench.parse([]), 1) == ["c3", "c5"]
    assert bench.extra_legs(bench.parse([]), 8) == ["c4"]
    assert bench.extra_legs(bench.parse(["--config", "c4"]), 8) == []
    assert bench.extra_legs(bench.parse(["--config", "c3"]), 1) == ["c5"]
    assert bench.extra_legs(bench.parse(["--extra-configs", ""]), 1) == []
    assert bench.extra_legs(bench.parse(["--extra-configs", "c4,c5"]), 1) == ["c4", "c5"]
    a = bench.parse(["--steps", "7"])
    leg = bench.leg_args(a, "c5")
    assert (leg.height, leg.width, leg.maxdisp, leg.batch, leg.precision) == (1008, 1512, 264, 1, "f32")
    assert bench.config_name(leg) == "c5" and bench.config_name(a) == "c2" and leg.steps == 7
    assert bench.parse(["--gpus", "2", "--dist-backend", "gloo"]).dist_backend == "gloo"
