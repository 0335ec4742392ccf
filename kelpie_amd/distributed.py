"""One process per GPU: shard candidate explanations across ranks, gather results.

The post-training path partitions naturally: each candidate
evaluation needs only the frozen tables (a full replica per rank), its rows
and its random draws.  Ranks therefore take disjoint predictions and never
exchange data on the hot path; the only collective is one gather of the
fixed-size result records (relevance, scores, ranks) to rank 0 at the end
(RCCL over xGMI with the ``nccl`` backend, or ``gloo`` on CPU).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed when launched by torchrun; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("KELPIE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend)
    return rank, world, local


def shard(items, rank, world):
    """Contiguous shard of a list (candidates / predictions) for this rank."""
    n = len(items)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return items[lo:hi]


RECORD = 5  # relevance, pt score, base score, pt rank, base rank (as float64)


def gather_records(records: np.ndarray, device=None):
    """Gather [n_i, RECORD] float64 result records from every rank to all ranks.

    Ranks may hold different counts; the records are padded to the max count,
    all-gathered once, and trimmed."""
    records = np.ascontiguousarray(records, dtype=np.float64).reshape(-1, RECORD)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return records
    world = dist.get_world_size()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    n = torch.tensor([records.shape[0]], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    buf = torch.zeros((m, RECORD), dtype=torch.float64, device=device)
    if records.shape[0]:
        buf[:records.shape[0]] = torch.from_numpy(records).to(device)
    out = torch.zeros((world * m, RECORD), dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(out, buf)
    out = out.cpu().numpy().reshape(world, m, RECORD)
    return np.concatenate([out[r, :counts[r]] for r in range(world)])


def max_over_ranks(value: float, device=None) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
