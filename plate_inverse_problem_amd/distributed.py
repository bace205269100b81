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

# collectives issued by all_reduce_sum / all_gather_cat since import (tests check that the
# collective path really ran, including at world size 1)
N_COLLECTIVES = 0


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def init_from_env(device: torch.device | None = None) -> tuple[int, int, str | None]:
    """Join the process group a launcher (``torch.distributed.run``) describes in the environment.

    Initialises whenever the launcher set ``WORLD_SIZE`` -- also for a single rank, so that the
    RCCL path runs at world size 1 too -- with ``PFR_DIST_BACKEND`` (default ``nccl`` = RCCL on
    ROCm; ``device`` is this rank's GPU, bound to the group).  Returns (rank, world size, backend or
    None when no launcher environment is present)."""
    if "WORLD_SIZE" not in os.environ or not dist.is_available():
        return 0, 1, None
    if not dist.is_initialized():
        backend = os.environ.get("PFR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size(), dist.get_backend()


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


def _comm_tensor(t: torch.Tensor) -> torch.Tensor:
    """``t`` where the backend can reduce it: host memory for gloo, this rank's GPU for nccl."""
    backend = dist.get_backend()
    if backend == "gloo" and t.device.type != "cpu":
        return t.cpu()
    if backend == "nccl" and t.device.type != "cuda":
        return t.to(torch.device("cuda", torch.cuda.current_device()))
    return t


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    """Sum ``t`` over all ranks (no-op without an initialised process group; with one, the
    collective runs at every world size, 1 included).

    Complex tensors are reduced through their real view.  With the ``nccl``
    (RCCL) backend the tensor must live on this rank's GPU; with ``gloo`` on CPU.
    """
    global N_COLLECTIVES
    if not (dist.is_available() and dist.is_initialized()):
        return t
    work = _comm_tensor(t)
    buf = torch.view_as_real(work).contiguous() if work.is_complex() else work.contiguous()
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    N_COLLECTIVES += 1
    out = torch.view_as_complex(buf) if work.is_complex() else buf
    return out.to(t.device)


def all_gather_cat(t: torch.Tensor, n_total: int) -> torch.Tensor:
    """Concatenate every rank's ``shard_range`` block (1-D ``t`` of this rank's length) into the
    full ``n_total`` vector on every rank (``solveForward`` over sharded frequencies; SURVEY.md
    section 8(e)).  No-op without an initialised process group."""
    global N_COLLECTIVES
    if not (dist.is_available() and dist.is_initialized()):
        return t
    r, w = world()
    sizes = [shard_range(n_total, k, w) for k in range(w)]
    width = max(hi - lo for lo, hi in sizes)
    work = _comm_tensor(t)
    real = torch.view_as_real(work) if work.is_complex() else work
    pad = torch.zeros((width,) + tuple(real.shape[1:]), dtype=real.dtype, device=real.device)
    pad[:real.shape[0]] = real
    parts = [torch.empty_like(pad) for _ in range(w)]
    dist.all_gather(parts, pad.contiguous())
    N_COLLECTIVES += 1
    out = torch.cat([p[:hi - lo] for p, (lo, hi) in zip(parts, sizes)])
    if work.is_complex():
        out = torch.view_as_complex(out.contiguous())
    return out.to(t.device)
