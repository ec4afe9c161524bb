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
