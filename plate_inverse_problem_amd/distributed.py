"""Frequency sharding across ranks (one process per GPU) + the single all-reduce.

The reference has no distributed code; its only parallelism is OpenMP over
the frequency batch (``InnerState.h:276-288``).  Every loss of
``Problem.getLossFunction`` is a mean of per-frequency terms
(``Problem.py:948-975``), so the sweep partitions into contiguous frequency
blocks with NO data-path exchange; the only collective is one
``all_reduce(SUM)`` of the packed ``[loss_sum, w_0..w_17]`` partials (19 complex
= 304 B) per loss/gradient evaluation -- RCCL over xGMI with the ``nccl``
backend, ``gloo`` in CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def shard_range(n_total: int, rank: int | None = None, world_size: int | None = None) -> tuple[int, int]:
    """Contiguous block ``[lo, hi)`` of ``n_total`` items owned by ``rank``
    (sizes differ by at most one; every item owned exactly once)."""
    r, w = world()
    rank = r if rank is None else rank
    world_size = w if world_size is None else world_size
    base, extra = divmod(n_total, world_size)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    """Sum ``t`` over all ranks (no-op without an initialised process group).

    Complex tensors are reduced through their real view.  With the ``nccl``
    (RCCL) backend the tensor must live on this rank's GPU; with ``gloo`` on CPU.
    """
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    backend = dist.get_backend()
    dev = t.device
    work = t
    if backend == "gloo" and dev.type != "cpu":
        work = t.cpu()
    elif backend == "nccl" and dev.type != "cuda":
        work = t.to(torch.device("cuda", torch.cuda.current_device()))
    buf = torch.view_as_real(work).contiguous() if work.is_complex() else work.contiguous()
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    out = torch.view_as_complex(buf) if work.is_complex() else buf
    return out.to(dev)
