"""Process-group helpers for ray-sharded multi-GPU runs (one process per GPU).

The product's multi-GPU path is native: libarx's groups (arx_group_*, RenderGroup) shard the
rays and all-reduce the int64 IR histogram with RCCL themselves.  torch.distributed is only an
optional caller-side convenience: the bootstrap of a one-process-per-GPU group (broadcasting
rank 0's RCCL unique id), barriers and max-over-ranks timing in bench.py, and an alternative
histogram all-reduce (allreduce_histogram) for callers that keep the histogram in a torch tensor
(arx_attach_histogram).

The reference is single-GPU (device 0 hard-coded, AudioRenderer.cpp:252).  Rank r of W traces
the global ray ids [r*N/W, (r+1)*N/W) of the same launch (the Philox key is the global id, so
the union of shards is exactly the single-GPU launch) into an int64 fixed-point histogram, and
ONE all-reduce (SUM, int64) over xGMI combines the 2*ir_len bins -- exact, so the IR is bitwise
independent of W.  That all-reduce is the path's only exchange step.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Balanced contiguous split of [0, n_total)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return n_total * rank // world, n_total * (rank + 1) // world


def env_rank_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str | None = None, force: bool = False) -> tuple[int, int, int]:
    """Join the process group when launched with WORLD_SIZE > 1 (or always with force=True: a
    one-rank group, to rehearse the multi-process path on one GPU)."""
    rank, world, local = env_rank_world()
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def allreduce_histogram(hist: torch.Tensor) -> torch.Tensor:
    """In-place exact SUM of the int64 IR histograms of all ranks."""
    if hist.dtype != torch.int64:
        raise TypeError("IR histogram must be int64 fixed point")
    if dist.is_initialized():
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
    return hist


def broadcast_object(objs: list, src: int = 0) -> list:
    """In-place broadcast of a list of picklable objects from rank src (e.g. the RCCL unique id)."""
    if dist.is_initialized():
        dist.broadcast_object_list(objs, src=src)
    return objs


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(value: float, device: torch.device | None = None) -> float:
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, device: torch.device | None = None) -> int:
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
