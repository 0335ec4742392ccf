"""One process per GPU: shard candidate explanations across ranks, gather results.

The post-training path partitions naturally: each candidate
evaluation needs only the frozen tables (a full replica per rank), its rows and its
random draws.  What does not partition is the reference's random stream: one
process-global generator state, seeded once (explain.py:144) and consumed in call
order across every prediction (post_training_engine.py:52, the optimizers' per-epoch
draws, engine.py:125, stochastic_builder.py:161-165).  A rank that starts a later
prediction from a fresh seed returns different results than the sequential run.

``SlotSharding`` keeps the results identical to the 1-rank (and reference) run: every
rank walks every engine batch's draws in the same order -- so every generator stays in
lockstep -- but only the slots it *claims* are scheduled in full (kelpie init, edited
rows, rank filter, draw values) and post-trained on its GPU; for the other slots it
only advances the generators (the torch ones by one deferred discard per run of such
slots, the numpy one by simulating the TransE shuffles, whose consumption is
data-dependent).  Claims are made while scheduling, in slot order, by the same
greedy rule on every rank: a slot goes to the rank with the least claimed row count so
far (ties to the lowest rank).  One all-gather of fixed-size (slot, score, rank)
records per batch (RCCL over xGMI with the ``nccl`` backend, ``gloo`` on CPU; every
rank sends a block of the same size, known from the claims, so it is a single
collective with no count exchange) gives
every rank every result, so the builder's accept / early-exit / ``random.random()``
replay runs identically on all ranks; each rank's record set carries a status row, so
a rank whose device work failed makes every rank raise instead of leaving the others
blocked in the gather.  ``select_entities_to_convert`` shards its conversion test by
entity range and all-gathers the keep mask.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend=None, force=False):
    """Initialise torch.distributed when launched by torchrun; returns (rank, world, local_rank).
    ``force``: initialise a process group even for a world of one (tests that drive the
    collective path on a single device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
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


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"


class SlotSharding:
    """Split each engine batch's slots over the ranks (see the module docstring)."""

    def __init__(self, rank=None, world=None, device=None, force_collective=False):
        init = dist.is_initialized()
        self.rank = dist.get_rank() if rank is None and init else (rank or 0)
        self.world = dist.get_world_size() if world is None and init else (world or 1)
        self.device = device
        # run the gathers through the process group even at world 1 (a one-rank RCCL
        # group on one GPU exercises the device-tensor all_gather_into_tensor path)
        self.force_collective = force_collective
        self.gathers = 0
        self.collectives = 0  # collective calls issued (the slot gather: one per batch)
        self.loads = [0] * self.world

    def begin_batch(self, costs=None):
        """Start claiming the slots of a new engine batch.  With ``costs`` (every slot's
        cost in schedule order, engine._plan_costs) the slots are cut into ``world``
        contiguous runs of about equal total cost -- slot i goes to the rank whose share
        of the cost range holds the midpoint of its cost -- and the claims follow that
        plan; without, each claim goes online to the least loaded rank."""
        self.loads = [0] * self.world
        self._plan, self._plan_pos = None, 0
        if costs:
            tot = float(sum(costs))
            owners, cum = [], 0.0
            for c in costs:
                owners.append(min(self.world - 1, int((cum + 0.5 * c) * self.world / tot)))
                cum += c
            self._plan, self._plan_costs = owners, list(costs)

    def claim_owner(self, cost) -> int:
        """Assign the next slot of the batch (in scheduling order) to the rank with the
        least claimed cost so far, ties to the lowest rank, and return that rank.  Every
        rank makes the same calls in the same order, so all agree on every owner."""
        loads = self.loads
        plan = getattr(self, "_plan", None)
        if plan is not None and self._plan_pos < len(plan):
            i = self._plan_pos
            if int(cost) != int(self._plan_costs[i]):
                raise RuntimeError("slot sharding: the schedule departed from the planned slot costs")
            self._plan_pos += 1
            loads[plan[i]] += int(cost)
            return plan[i]
        r = loads.index(min(loads))  # the first (lowest) rank among the least loaded
        loads[r] += int(cost)
        return r

    def claim(self, cost) -> bool:
        """:meth:`claim_owner`, True if the slot is this rank's."""
        return self.claim_owner(cost) == self.rank

    def gather_slots(self, idx, score, rank, n, failed=False, counts=None):
        """Every rank's (slot index, score, rank) records -> full [n] score / rank arrays.

        ``counts[r]``: the slots rank r owns (every rank knows them from the claims), so
        every rank sends the same fixed-size block -- its records, padding rows (index
        -2) and a status row (index -1, its failure flag) -- in ONE all-gather, with no
        count exchange.  A rank whose device work failed sends only padding and its
        status; if any rank failed, every rank raises after the gather."""
        if counts is None:  # a caller without the owners: exchange the counts first
            counts = self._gather_counts(len(idx))
        m = int(max(counts)) + 1 if len(counts) else 1
        if len(idx) > m - 1:
            # never raise before the collective (the other ranks would wait in it):
            # send nothing but the failure status, and every rank raises after the gather
            idx, score, rank, failed = idx[:0], score[:0], rank[:0], True
        recs = np.zeros((m, 3), np.float64)
        recs[:, 0] = -2.0
        if len(idx):
            recs[:len(idx), 0] = idx
            recs[:len(idx), 1] = np.asarray(score, np.float64)
            recs[:len(idx), 2] = np.asarray(rank, np.float64)
        recs[-1] = (-1.0, 1.0 if failed else 0.0, float(self.rank))
        allr = self._gather_fixed(recs)
        bad = [int(rk) for i, st, rk in allr if i == -1 and st != 0]
        if bad:
            raise RuntimeError(f"slot sharding: the device work of rank(s) {bad} failed")
        out_s = np.zeros(n, np.float32)
        out_r = np.zeros(n, np.int64)
        seen = np.zeros(n, np.int32)
        for i, sc, rk in allr:
            i = int(i)
            if i < 0:
                continue
            out_s[i], out_r[i] = sc, int(rk)
            seen[i] += 1
        if not np.all(seen == 1):
            raise RuntimeError("slot sharding: a slot was not post-trained exactly once")
        return out_s, out_r

    def gather_mask(self, lo, hi, keep, n):
        """Keep flags of the entity range [lo, hi) from every rank -> the full [n] mask."""
        # every rank's range is [n r / w, n (r + 1) / w): fixed-size blocks, one collective
        m = max(1, max((n * (r + 1)) // self.world - (n * r) // self.world for r in range(self.world)))
        recs = np.zeros((m, 2), np.float64)
        recs[:, 0] = -1.0
        recs[:hi - lo, 0] = np.arange(lo, hi)
        recs[:hi - lo, 1] = np.asarray(keep, np.float64)
        allr = self._gather_fixed(recs)
        allr = allr[allr[:, 0] >= 0]
        out = np.zeros(n, bool)
        out[allr[:, 0].astype(np.int64)] = allr[:, 1] != 0
        return out

    def _gather_fixed(self, recs):
        """All-gather one [m, width] float64 block per rank (the same m on every rank):
        one collective, no host synchronisation before it."""
        self.gathers += 1
        self.collectives += 1
        if not dist.is_initialized() or (self.world == 1 and not self.force_collective):
            return recs
        device = self.device or _device()
        buf = torch.from_numpy(np.ascontiguousarray(recs)).to(device)
        out = torch.empty((self.world * recs.shape[0], recs.shape[1]), dtype=torch.float64, device=device)
        dist.all_gather_into_tensor(out, buf)
        return out.cpu().numpy()

    def _gather_counts(self, n):
        self.collectives += 1
        if self.world == 1 or not dist.is_initialized():
            return [n]
        device = self.device or _device()
        cnt = torch.tensor([n], dtype=torch.int64, device=device)
        counts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(counts, cnt)
        return [int(c.item()) for c in counts]

