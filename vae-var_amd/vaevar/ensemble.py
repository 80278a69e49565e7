"""Ensemble sharding: independent analyses (ensemble members / assimilation windows), one process per
GPU, no communication in the inner loop, one gather of the analyses at the end.

Backend "nccl" is RCCL on ROCm (xGMI point-to-point: the gather to rank 0 receives on its direct links
in parallel); "gloo" runs the same code on CPU for the multi-process tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def init(backend: str | None = None):
    """Process group of this rank; backend: "nccl" (RCCL) with a GPU, else "gloo" (VAEVAR_DIST_BACKEND overrides,
    e.g. gloo for several ranks sharing one GPU in a test: RCCL refuses two ranks on one device)."""
    rank, size, local = world()
    if size > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("VAEVAR_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, size, local


def member_of(analysis: int, size: int) -> int:
    """Analysis b runs on rank b mod world_size."""
    return analysis % size


def my_members(n_analyses: int, rank: int, size: int):
    return [b for b in range(n_analyses) if member_of(b, size) == rank]


def barrier():
    if dist.is_initialized():
        dist.barrier()


def _cpu_backend() -> bool:
    return dist.get_backend() == "gloo"


def reduce_scalar(x: float, op: str, device=None) -> float:
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=None if _cpu_backend() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def gather_analyses(xa: torch.Tensor, dst: int = 0):
    """All ranks' analysis fields on rank `dst` (list indexed by rank), None elsewhere."""
    if not dist.is_initialized():
        return [xa]
    rank, size = dist.get_rank(), dist.get_world_size()
    x = xa.contiguous().cpu() if _cpu_backend() else xa.contiguous()
    out = [torch.empty_like(x) for _ in range(size)] if rank == dst else None
    dist.gather(x, out, dst=dst)
    return out
