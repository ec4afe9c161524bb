"""Batch-parallel inference over the GPUs of one node: one process per GPU.

The reference's only multi-GPU mechanism is ``nn.DataParallel`` (predict.py:49-50):
one process replicating weights and scattering the batch on every call.  Stereo
pairs are independent, so here each rank owns a contiguous shard of the pairs and
runs the whole hot path locally; there is no collective inside a step.  After the
timed region one all-gather (RCCL over xGMI with the ``nccl`` backend; ``gloo`` in
the CPU tests) collects per-pair EPE, and one all-reduce(MAX) the per-rank time.

Everything here is backend-agnostic torch.distributed plumbing, so the same code
runs under ``gloo`` on CPU (tests/test_parallel_gloo.py) and RCCL on MI355X.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world: int
    local_rank: int

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def rank_info() -> RankInfo:
    """torchrun-style environment (RANK / WORLD_SIZE / LOCAL_RANK), defaults N=1."""
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, info: RankInfo, device: torch.device | None = None):
    """Join the process group when world > 1 (MASTER_ADDR/PORT from the env)."""
    if info.world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None
                                       and device.type == "cuda") else {}
        dist.init_process_group(backend, rank=info.rank, world_size=info.world, **kw)


def shard(n_pairs: int, info: RankInfo) -> range:
    """Contiguous shard of a global batch: rank r gets pairs [r*n/W, (r+1)*n/W)
    (weak scaling in bench.py: n = world * pairs_per_gpu)."""
    lo = n_pairs * info.rank // info.world
    hi = n_pairs * (info.rank + 1) // info.world
    return range(lo, hi)


def _host_staged() -> bool:
    """gloo's collectives take host tensors: a device tensor goes through a host copy
    (the gloo rehearsal of the N-rank GPU path; RCCL works on the device tensors)."""
    return dist.get_backend() == "gloo"


def max_over_ranks(value: float, device: torch.device) -> float:
    """Slowest rank's time (the job's time)."""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        if _host_staged():
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_per_pair(values: torch.Tensor) -> torch.Tensor:
    """All-gather equally sized per-rank 1-D tensors (per-pair EPE) -> rank-ordered
    concatenation on every rank.  The single collective of the data path."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return values
    src = values.cpu() if _host_staged() else values
    out = torch.empty(dist.get_world_size() * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src.contiguous())
    return out.to(values.device)


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def finalize():
    if dist.is_initialized():
        dist.destroy_process_group()
