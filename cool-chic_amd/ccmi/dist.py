"""Image-parallel multi-GPU plumbing (one process per GPU, torch.distributed).

Cool-chic's units of work are independent images/frames (the reference runs one SLURM
job per image, sbatch-files/submit-coolchic-encoding.sh:5-8), so the hot path shards
with NO data-path collective: each rank decodes / forwards its own frames.  The only
communication is dataset-level aggregation at the end of a run:
one all_gather of small per-image records and one all_reduce of counters.  With the
"nccl" backend this is RCCL over xGMI on MI355X; tests run it with "gloo" on CPU.
"""

from __future__ import annotations

import os
from typing import Any, Sequence


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard(items: Sequence[Any], rank: int, world: int) -> list:
    """Static round-robin assignment of independent units (images) to ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return [x for i, x in enumerate(items) if i % world == rank]


def gather_records(records: list, group=None) -> list:
    """all_gather of per-image records (name, bpp, psnr, seconds, ...) -> flat list on every rank."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return list(records)
    out: list = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, list(records), group=group)
    return [r for part in out for r in part]


def reduce_counters(counters: dict, op: str = "sum", device=None, group=None) -> dict:
    """all_reduce of scalar counters (pixels decoded, kernel seconds, ...): op in {sum, max}."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return dict(counters)
    keys = sorted(counters)
    t = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=group)
    return {k: float(v) for k, v in zip(keys, t.tolist())}
