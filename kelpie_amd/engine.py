"""MI355X-native post-training relevance engines.

Drop-in for the reference's ``src/relevance_engines/post_training_engine.py``:
same class names, constructor ``(model, dataset, hp)``, ``set_cache()``,
``compute_relevance(pred, triples) -> float``, ``select_entities_to_convert``
and the same errors.  Underneath, every ``compute_relevance`` call becomes one
or more *slots* of a batched HIP launch (``kp_posttrain_rank``), and
``compute_relevance_batch(pred, rules)`` evaluates many candidates in one
launch while consuming the reference's random draws in the reference's order
(``kelpie_amd.rng``), so a batch returns exactly what the sequential calls
would.
"""
from __future__ import annotations

import math
import os
import random
import time
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .hparams import optimizer_hp
from .data import MANY_TO_ONE, ONE_TO_ONE, Dataset, KelpieView
from .models import FrozenModel
from .rng import ReferenceRNG, StateCheckpoint


def _sigmoid(x):
    # post_training_engine.py:19-20 (math.exp overflows below -709 like the reference)
    return 1 / (1 + math.exp(-x))


@dataclass(slots=True)
class _Slot:
    x0: np.ndarray
    rows: np.ndarray
    rng: np.ndarray
    pred: tuple
    filt: list
    result: dict = field(default=None)
    # False: another rank post-trains this slot (kelpie_amd.distributed); only the
    # generators were advanced past its draws, and x0 / rows / rng / filt may be None
    own: bool = True
    # the rank that post-trains it (sharded batches; every rank records every owner, so
    # each knows every rank's record count in the gather)
    owner: int = 0
    # rows and filter held by the library's host scheduler instead of rows / filt:
    # (SchedBatch, its slot index, row count, filter length) (kelpie_amd/_lib.py)
    native: tuple = None


def _contiguous_draws(slots, total, ctx=None):
    """The slots' draws as one int32 array.  When they lie back to back in one pooled
    page-locked arena (rng.ReferenceRNG._take with a GPU present), that span itself: the
    library reads it by DMA, no copy.  Otherwise a copy: handing the library a view of a
    pageable arena measured slower end to end (its upload from pages first touched by
    the RNG worker threads took 10-20 ms per TransE batch against 3 ms after a copy into
    a reused buffer, profiles/r02zd_transe_draws_upload.txt).  The copy goes into a
    buffer kept with the device context ``ctx`` (no fresh pages per batch; the context's
    previous batch is done with it) and runs in the library without the interpreter lock,
    so the next batch's scheduling thread is not held up."""
    if total == 0:
        return np.zeros(1, np.int32)
    arrays = [s.rng.reshape(-1) for s in slots]
    live = [a for a in arrays if a.size]
    lease = _lib.arena_of(live[0]) if live else None
    if lease is not None:
        # the draws were written back to back into one page-locked arena in slot order
        # (the usual case): hand the library that span (a view of the lease, which keeps
        # the arena busy while the library reads it), uploaded by DMA
        start = live[0].__array_interface__["data"][0]
        pos = start
        for a in live:
            if _lib.arena_of(a) is not lease or a.__array_interface__["data"][0] != pos or a.dtype.itemsize != 4:
                break
            pos += 4 * a.size
        else:
            off = (start - lease.__array_interface__["data"][0]) // 4
            return lease[off:off + total]
    if ctx is None or any(a.dtype.itemsize != 4 for a in arrays):
        return np.concatenate(arrays).astype(np.int32, copy=False)
    buf = getattr(ctx, "_draw_buf", None)
    if buf is None or buf.size < total:
        buf = np.empty(int(total * 1.25) + 1024, np.int32)
        ctx._draw_buf = buf
    return _lib.gather_i32([np.ascontiguousarray(a) for a in arrays], buf)


class RelevanceEngine:
    """engine.py:13-20 + select_entities_to_convert (engine.py:22-126)."""

    def __init__(self, model: FrozenModel, dataset: Dataset):
        self.model = model
        self.dataset = dataset
        self._o_to_training = None
        # kelpie_amd.distributed.SlotSharding: every rank schedules every batch and
        # post-trains its share of the slots; None = this process does all of them
        self.sharding = None

    @property
    def o_to_training_triples(self):
        if self._o_to_training is None:
            d = {}
            for h, r, t in self.dataset.training_triples.tolist():
                d.setdefault(t, []).append((h, r, t))
            self._o_to_training = d
        return self._o_to_training

    def select_entities_to_convert(self, pred, k: int, degree_cap=None, criage=False):
        ds = self.dataset
        s, p, o = (int(v) for v in pred)
        ents = []
        for e in range(ds.num_entities):
            if e == s:
                continue
            deg = ds.entity_to_degree.get(e, 0)
            if deg < 1:
                continue
            if degree_cap and deg > degree_cap:
                continue
            if criage and e not in self.o_to_training_triples:
                continue
            if (e, p) in ds.to_filter:
                if ds.relation_to_type[p] in (ONE_TO_ONE, MANY_TO_ONE):
                    continue
                if o in ds.to_filter[(e, p)]:
                    continue
            ents.append(e)
        if not ents:
            # the reference returns here WITHOUT resetting entities_to_convert
            # (engine.py:90-91): a sufficient pipeline then reuses the previous
            # prediction's conversion entities
            return []
        fo, fl = [0], []
        for e in ents:
            F = ds.to_filter.get((e, p), [])
            fl.extend(F)
            fo.append(len(fl))
        sh = self.sharding
        if sh is not None and (sh.world > 1 or getattr(sh, "force_collective", False)):
            # entity-range shard of the conversion test, keep mask all-gathered
            lo, hi = len(ents) * sh.rank // sh.world, len(ents) * (sh.rank + 1) // sh.world
            part = np.zeros(0, bool)
            if hi > lo:
                part = self.model.ctx.convertible(np.array(ents[lo:hi]), p, o, np.array(fo[lo:hi + 1]) - fo[lo],
                                                  np.array(fl[fo[lo]:fo[hi]], dtype=np.int64))
            keep = sh.gather_mask(lo, hi, part, len(ents))
        else:
            keep = self.model.ctx.convertible(np.array(ents), p, o, np.array(fo), np.array(fl, dtype=np.int64))
        overall = [e for e, kflag in zip(ents, keep) if kflag]
        chosen = random.sample(overall, k=min(k, len(overall)))  # engine.py:125 (python RNG)
        self.entities_to_convert = chosen
        return chosen


class PostTrainingEngine(RelevanceEngine):
    """post_training_engine.py:17-125."""

    def __init__(self, model: FrozenModel, dataset: Dataset, hp: dict, rng: ReferenceRNG | None = None):
        RelevanceEngine.__init__(self, model=model, dataset=dataset)
        # the reference's optimizer hp class (post_training_engine.py:71): a missing or
        # mistyped field raises pydantic.ValidationError here, before any device work
        self.hp = optimizer_hp(model.name, hp)
        self.rng = rng or ReferenceRNG()
        self._fused = []  # TransE calls whose edits and draws _flush_fused makes in two library calls
        self._sched = None
        self._kp_hp = model.kp_hp(hp)
        if getattr(model, "is_kelpie", False):
            raise Exception("Already a post-trainable KelpieModel.")
        self.set_cache()
        self.last_batch_stats = {}

    def set_cache(self):
        self.base_pt_results = {}
        self.kelpie_dataset_cache_size = 20
        self.kelpie_dataset_cache = OrderedDict()

    def _get_kelpie_dataset(self, original_entity: int) -> KelpieView:
        e = int(original_entity)
        if e not in self.kelpie_dataset_cache:
            self.kelpie_dataset_cache[e] = KelpieView(self.dataset, e)
            self.kelpie_dataset_cache.move_to_end(e)
            if len(self.kelpie_dataset_cache) > self.kelpie_dataset_cache_size:
                self.kelpie_dataset_cache.popitem(last=False)
        return self.kelpie_dataset_cache[e]

    # ------------------------------------------------------------------ slot assembly
    def _slot(self, x0, rows, kelpie_pred, filt):
        draws = self.model.posttrain_draws(rows, self.hp, self.rng)
        return _Slot(x0=x0, rows=rows, rng=draws, pred=tuple(int(v) for v in kelpie_pred), filt=list(filt))

    def _sharded(self):
        sh = self.sharding
        # a one-rank sharding with force_collective takes the sharded path too (its
        # gathers then run through the process group: the RCCL test on one GPU)
        return sh is not None and (sh.world > 1 or getattr(sh, "force_collective", False))

    def _skip_slot(self, kp, rows=None, n_rows=0):
        """A slot another rank post-trains: advance the generators past its draws only."""
        self.model.posttrain_skip(rows, n_rows, self.hp, self.rng)
        return _Slot(x0=None, rows=None, rng=None, pred=tuple(int(v) for v in kp), filt=None, own=False)

    def _schedule(self, pred, triples, mode, slots, pending_base):
        """Consume the draws of one reference compute_relevance call (post_training_engine.py:46-62)
        and append its slots.  Returns (pt_slot, base_key)."""
        pred = tuple(int(v) for v in pred)
        view = self._get_kelpie_dataset(pred[0])
        if getattr(self.model, "fused_call_draws", False):
            return self._schedule_fused(pred, view, triples, mode, slots, pending_base)
        if self._sharded():
            return self._schedule_sharded(pred, view, triples, mode, slots, pending_base)
        init = self.rng.rand_init(self.model.dimension)
        x_base = self.model.kelpie_init(init, self.rng)  # base KelpieModel is built every call (A-Q6)
        kp = view.as_kelpie_triple(pred)
        if pred not in self.base_pt_results and pred not in pending_base:
            pending_base[pred] = len(slots)
            slots.append(self._slot(x_base, view.base_rows, kp, view.filter_for(kp[1])))
        x_pt = self.model.kelpie_init(init, self.rng)
        rows, delta = view.removed(triples) if mode == "necessary" else view.added(triples)
        filt = view.filter_for(kp[1], delta.get(kp[1]))
        slots.append(self._slot(x_pt, rows, kp, filt))
        return len(slots) - 1, pred

    def _schedule_sharded(self, pred, view, triples, mode, slots, pending_base):
        """_schedule when the batch is sharded over ranks (kelpie_amd.distributed): every
        rank walks the same draws in the same order, but only the slots this rank claims
        get their kelpie init, rows, filter and draw values; for the others the
        generators are only advanced (one deferred torch discard for a run of them), so a
        rank's host work is its share of the slots plus the generator walk."""
        m, rng, sh = self.model, self.rng, self.sharding
        kp = view.as_kelpie_triple(pred)
        need_base = pred not in self.base_pt_results and pred not in pending_base
        base_owner = sh.claim_owner(max(1, len(view.base_rows))) if need_base else -1
        own_base = base_owner == sh.rank
        edit = view.removed if mode == "necessary" else view.added
        try:
            n_pt, _ = edit(triples, rows=False)  # the reference raises after the draws below
            err = None
        except Exception as e:  # noqa: BLE001 -- re-raised at the reference's point
            err, n_pt = e, 0
        pt_owner = sh.claim_owner(max(1, n_pt)) if err is None else -1
        own_pt = pt_owner == sh.rank
        if own_base or own_pt:
            init = rng.rand_init(m.dimension)
        else:
            init = None
            rng.skip_rand_init(m.dimension)
        # the base KelpieModel is built every call (A-Q6), then (uncached) post-trained
        x_base = m.kelpie_init(init, rng) if own_base else m.kelpie_skip(rng)
        if need_base:
            pending_base[pred] = len(slots)
            if own_base:
                slots.append(self._slot(x_base, view.base_rows, kp, view.filter_for(kp[1])))
            else:
                slots.append(self._skip_slot(kp, view.base_rows, len(view.base_rows)))
            slots[-1].owner = base_owner
        x_pt = m.kelpie_init(init, rng) if own_pt else m.kelpie_skip(rng)
        if err is not None:
            raise err
        if own_pt or m.skip_needs_rows:
            rows, delta = edit(triples)
        if own_pt:
            slots.append(self._slot(x_pt, rows, kp, view.filter_for(kp[1], delta.get(kp[1]))))
        else:
            slots.append(self._skip_slot(kp, rows if m.skip_needs_rows else None, n_pt))
        slots[-1].owner = pt_owner
        return len(slots) - 1, pred

    def _schedule_fused(self, pred, view, triples, mode, slots, pending_base):
        """_schedule for TransE: the call's slots are appended now and the call is queued;
        :meth:`_flush_fused` then makes the edits and rank filters of every queued call in
        one library call (kp_sched_add_calls, csrc/kp_sched.cpp) and their draws in another
        (ReferenceRNG.transe_calls), in order.  The edit draws nothing; if it fails, the
        flush makes the draws the reference makes before raising (everything but the
        post-trained model's epochs), drops the calls after it, and raises its error."""
        kp = view.as_kelpie_triple(pred)
        need_base = pred not in self.base_pt_results and pred not in pending_base
        sharded = self._sharded()
        nb = view.n_base_rows
        base_owner = pt_owner = 0
        if sharded and need_base:
            base_owner = self.sharding.claim_owner(max(1, nb))
        own_base = need_base and (not sharded or base_owner == self.sharding.rank)
        if sharded:
            # owners from row counts known before the edit: the base rows +- the rule's
            # rows (kelpie_amd.distributed); every rank still runs every edit's checks
            est = nb + 2 * len(triples) if mode == "sufficient" else nb - 2 * len(triples)
            pt_owner = self.sharding.claim_owner(max(1, est))
            own_pt = pt_owner == self.sharding.rank
        else:
            own_pt = True
        sb = self._sched_batch()
        base = None
        if need_base:
            pending_base[pred] = len(slots)
            base = _Slot(None, None, None, kp, None, None, own_base, base_owner, (sb, sb.n_slots))
            sb.n_slots += 1
            slots.append(base)
        pt = _Slot(None, None, None, kp, None, None, own_pt, pt_owner, (sb, sb.n_slots))
        sb.n_slots += 1
        slots.append(pt)
        # a queued call: (view, kelpie triple, rule triples, flags, base slot, pt slot)
        self._fused.append((view, kp, [(int(a), int(b), int(c)) for a, b, c in triples],
                            (1 if need_base else 0) | (2 if own_base else 0) | (4 if own_pt else 0)
                            | (8 if mode == "sufficient" else 0), base, pt))
        if len(self._fused) >= (self._FUSED_FLUSH if self._sched is not None else self._FUSED_FIRST):
            # hand the draws to the library's workers early: their numpy shuffles then run
            # while this thread queues the next calls (the batch's first flush sooner, so
            # the sequential numpy chain starts right away)
            self._flush_fused()
        return len(slots) - 1, pred

    def _schedule_fused_pred(self, pred, rules, mode, slots, pending_base):
        """:meth:`_schedule_fused` for every rule of one prediction (no checkpoints, no
        empty rule): the same slots, claims and queued calls in the same order, with the
        prediction's view, kelpie triple and row count looked up once.  Returns the
        prediction's [(pt slot index, base key)]."""
        pred = tuple(int(v) for v in pred)
        view = self._get_kelpie_dataset(pred[0])
        kp = view.as_kelpie_triple(pred)
        sharded = self._sharded()
        sh = self.sharding
        nb = view.n_base_rows
        sufficient = mode == "sufficient"
        first = self._sched is None
        sb = self._sched_batch()
        fused, flush_at = self._fused, self._FUSED_FIRST if first else self._FUSED_FLUSH
        out = []
        suf = 8 if sufficient else 0
        append = slots.append
        for rule in rules:
            triples = [(int(a), int(b), int(c)) for a, b, c in rule]
            need_base = pred not in self.base_pt_results and pred not in pending_base
            base_owner = pt_owner = 0
            if sharded and need_base:
                base_owner = sh.claim_owner(max(1, nb))
            own_base = need_base and (not sharded or base_owner == sh.rank)
            if sharded:
                est = nb + 2 * len(triples) if sufficient else nb - 2 * len(triples)
                pt_owner = sh.claim_owner(max(1, est))
                own_pt = pt_owner == sh.rank
            else:
                own_pt = True
            base = None
            j = sb.n_slots
            if need_base:
                pending_base[pred] = len(slots)
                base = _Slot(None, None, None, kp, None, None, own_base, base_owner, (sb, j))
                append(base)
                j += 1
            pt = _Slot(None, None, None, kp, None, None, own_pt, pt_owner, (sb, j))
            append(pt)
            sb.n_slots = j + 1
            fused.append((view, kp, triples, (1 if need_base else 0) | (2 if own_base else 0) | (4 if own_pt else 0)
                          | suf, base, pt))
            out.append((len(slots) - 1, pred))
            if len(fused) >= flush_at:
                self._flush_fused()
                fused, flush_at = self._fused, self._FUSED_FLUSH
        return out

    def _sched_batch(self):
        """This batch's native scheduler batch (created on its first TransE call)."""
        if self._sched is None:
            self._sched = _lib.SchedBatch()
            self._sched.dim = self.model.dimension
        return self._sched

    # queued TransE calls per library call (KELPIE_TE_FLUSH: A/B of the per-flush overhead
    # against how early the draws reach the workers).  Alternating on two boxes, 30 steps
    # (profiles/r05/r05aj/, r05ak/): 64 averaged 57.9k cand/s over seven runs, 24 50.9k, 48
    # 55.6k over four
    _FUSED_FLUSH = int(os.environ.get("KELPIE_TE_FLUSH", "64"))
    _FUSED_FIRST = 4  # ... for a batch's first one

    @staticmethod
    def _edit_error(call, code, k):
        """The exception KelpieView.removed / added raise (kelpie_dataset.py:92-158)."""
        if code == 1:
            return AssertionError()
        if code == 2:
            v = call[0]
            o, kel = v.original_entity, v.kelpie_entity
            t = call[2][k]
            return KeyError((kel if t[0] == o else t[0], t[1], kel if t[2] == o else t[2]))
        return ValueError("list.remove(x): x not in list")

    def _flush_fused(self):
        """Make the queued TransE calls' edits, rank filters (kp_sched_add_calls) and draws
        (kp_rng_transe_calls, asynchronous) and record them with the scheduler batch: one
        record per flush, whose arrays the pack reads by slot (:meth:`_pack_native`), so no
        per-call Python work is left here beyond building the call arrays."""
        calls, self._fused = self._fused, []
        if not calls:
            return
        m, hp = self.model, self.hp
        sb = self._sched_batch()
        nviews = [c[0].native for c in calls]
        sb.views.extend(nviews)  # its C++ slots point into these views: they live as long as the batch
        off = np.zeros(len(calls) + 1, np.int32)
        np.cumsum([len(c[2]) for c in calls], out=off[1:])
        flags = np.fromiter((c[3] for c in calls), np.int32, len(calls))
        idx, rows, nf, (fc, code, k) = sb.add_calls([v.h for v in nviews], [c[1][1] for c in calls], flags, off,
                                                   [t for c in calls for t in c[2]])
        n = len(calls) if fc < 0 else fc + 1  # the reference stops at the failing call
        has_base = (flags[:n] & 1) != 0
        r_base = np.where(has_base, rows[:n, 0], -1)
        r_pt = rows[:n, 1].copy()
        if fc >= 0:
            r_pt[fc] = -1
        want = ((flags[:n] >> 1) & 3) if self._sharded() else None
        xb, xp, out, sz = self.rng.transe_calls(m.dimension, m.dimension, r_base, r_pt, int(hp["epochs"]),
                                                int(hp["negative_triples_ratio"]), m.dataset.num_entities + 1,
                                                want=want, raw=True)
        # the flush's slots in creation order: per call its base slot (if any), then its pt slot
        first = calls[0][4] if calls[0][4] is not None else calls[0][5]
        present = np.empty((n, 2), bool)
        present[:, 0] = has_base
        present[:, 1] = True
        if fc >= 0:
            present[fc, 1] = False
        sb.recs.append({"j0": first.native[1], "present": present.ravel(), "idx": idx[:n].ravel(),
                        "rows": rows[:n].ravel(), "nf": nf[:n].ravel(), "sz": sz.ravel(), "xb": xb, "xp": xp,
                        "out": out})
        sb.packed = None
        if fc >= 0:
            raise self._edit_error(calls[fc], code, k)

    def _plan_costs(self, items):
        """The claim cost of every slot the batch will schedule, in schedule order, without
        drawing anything: a base slot (first call of an uncached prediction) costs its
        base rows, a post-trained slot its rows after the edit (the costs _schedule_sharded
        claims with); the list stops where the schedule stops (an edit that raises)."""
        costs, pending = [], set()
        for pred, triples, mode in self._calls(items):
            pred = tuple(int(v) for v in pred)
            view = self._get_kelpie_dataset(pred[0])
            if pred not in self.base_pt_results and pred not in pending:
                pending.add(pred)
                costs.append(max(1, len(view.base_rows)))
            edit = view.removed if mode == "necessary" else view.added
            try:
                n_pt, _ = edit(triples, rows=False)
            except Exception:  # noqa: BLE001 -- the schedule raises there too
                break
            costs.append(max(1, n_pt))
        return costs

    def _schedule_all(self, items, checkpoints):
        """_schedule_multi, with every queued TransE call's draws made before it returns or raises."""
        self._sched = None  # this batch's natively assembled slots (TransE), made on first use
        if self._sharded():
            # ComplEx / ConvE: every rank owns one contiguous run of the batch's slots, so it
            # skips the others' draws in two long runs (before and after its own), each one
            # MT19937 jump-ahead instead of a walk (kp_mt19937_discard); TransE's fused calls
            # keep the online greedy claims (its numpy stream cannot be jumped)
            fused = getattr(self.model, "fused_call_draws", False)
            self.sharding.begin_batch(None if fused else self._plan_costs(items))
        try:
            return self._schedule_multi(items, checkpoints)
        finally:
            self._flush_fused()

    def _run(self, slots, ctx=None, gate=None):
        """Post-train and rank ``slots`` on the device.  With ``self.sharding`` only this
        rank's share runs; ``_collect`` then gathers every rank's results.  ``gate``: called
        (blocking) before the library call, after the batch is packed; False cancels the
        batch (no device work, None returned) -- a held look-ahead window (submit_batch)."""
        if not slots:
            return {}
        if self._sharded():
            if gate is not None and not gate():
                return None
            # the slots this rank claimed while scheduling; a failure is reported to the
            # other ranks through the gather (_collect) instead of leaving them waiting in it
            mine = [i for i, s in enumerate(slots) if s.own]
            stats = {"slots": 0, "rows": 0, "pack_s": 0.0, "lib_s": 0.0}
            score, rank, err = [], [], None
            if any(slots[i].owner != self.sharding.rank for i in mine):
                # an owned slot must carry this rank as its owner (the record counts of the
                # gather come from the owners): report it through the gather, never before it
                err, mine = RuntimeError("slot sharding: an owned slot records another rank as its owner"), []
            if mine:
                try:
                    stats = self._run_slots([slots[i] for i in mine], ctx, fill=False)
                    score, rank = stats.pop("_score"), stats.pop("_rank")
                except Exception as e:  # noqa: BLE001 -- raised on every rank by _collect
                    err, mine = e, []
            counts = np.bincount([s.owner for s in slots], minlength=self.sharding.world)
            stats["_local"] = (mine, score, rank, len(slots), err, counts)
            self.last_batch_stats = stats
            return stats
        return self._run_slots(slots, ctx, fill=True, gate=gate)

    def _collect(self, slots, stats):
        """All-gather the ranks' slot results of a sharded batch (in batch order on every rank)."""
        local = stats.pop("_local", None) if stats else None
        if local is None:
            return
        mine, score, rank, n, err, counts = local
        t0 = time.perf_counter()
        try:
            all_s, all_r = self.sharding.gather_slots(mine, score, rank, n, failed=err is not None, counts=counts)
        except Exception:
            if err is not None:
                raise err
            raise
        for i, s in enumerate(slots):
            s.result = {"target_score": float(all_s[i]), "target_rank": int(all_r[i])}
        stats["gather_s"] = time.perf_counter() - t0

    def _pack(self, slots, ctx=None):
        """The library call's batch arrays (x0, row_off, rows, rng_off, rng, pred, filt_off, filt)."""
        n = len(slots)
        if slots and slots[0].native is not None:
            return self._pack_native(slots, ctx)
        x0 = np.stack([s.x0 for s in slots]).astype(np.float32)
        row_off = np.zeros(n + 1, np.int32)
        row_off[1:] = np.cumsum([len(s.rows) for s in slots])
        rows = np.concatenate([s.rows.reshape(-1, 3) for s in slots]).astype(np.int32) if row_off[-1] \
            else np.zeros((0, 3), np.int32)
        rng_off = np.zeros(n + 1, np.int64)
        rng_off[1:] = np.cumsum([s.rng.size for s in slots])
        rng = _contiguous_draws(slots, int(rng_off[-1]), ctx)
        pred = np.array([s.pred for s in slots], np.int32)
        filt_off = np.zeros(n + 1, np.int32)
        filt_off[1:] = np.cumsum([len(s.filt) for s in slots])
        filt = np.concatenate([np.asarray(s.filt, np.int32) for s in slots]) if filt_off[-1] \
            else np.zeros(1, np.int32)
        assert x0.shape == (n, self.model.dimension)
        return x0, row_off, rows, rng_off, rng, pred, filt_off, filt

    @staticmethod
    def _native_arrays(sb):
        """The scheduler batch's flush records as per-slot arrays (indexed by the slot's
        creation number j): scheduler slot index, row and filter counts, draw count and
        offset, and the kelpie init row.  Read after the batch's draws are complete."""
        if sb.packed is not None and sb.packed[0] == len(sb.recs):
            return sb.packed[1]
        N = sb.n_slots
        idx = np.full(N, -1, np.int32)
        nrow = np.zeros(N, np.int32)
        nfl = np.zeros(N, np.int32)
        nsz = np.zeros(N, np.int64)
        x0 = np.zeros((N, sb.dim), np.float32)
        outs, spans = [], []
        for r in sb.recs:
            pres = r["present"]
            m = int(pres.sum())
            js = r["j0"] + np.arange(m)
            idx[js] = r["idx"][pres]
            nrow[js] = r["rows"][pres]
            nfl[js] = r["nf"][pres]
            nsz[js] = r["sz"][pres]
            n = len(pres) // 2
            both = np.empty((n, 2, sb.dim), np.float32)
            both[:, 0] = r["xb"][:n]
            both[:, 1] = r["xp"][:n]
            x0[js] = both.reshape(2 * n, sb.dim)[pres]
            outs.append(r["out"])
            spans.append((int(js[0]) if m else r["j0"], m))
        # draw offsets per slot within the batch's concatenated draws (records in order)
        doff = np.zeros(N + 1, np.int64)
        np.cumsum(nsz, out=doff[1:])
        arrays = {"idx": idx, "nrow": nrow, "nfl": nfl, "nsz": nsz, "doff": doff, "x0": x0, "outs": outs}
        sb.packed = (len(sb.recs), arrays)
        return arrays

    def _pack_native(self, slots, ctx=None):
        """_pack for the TransE fast path: rows and filters written by the library's
        scheduler (kp_sched_pack), kelpie init rows and draws taken from the flush
        records by slot number."""
        n = len(slots)
        nat = [s.native for s in slots]
        sb = nat[0][0]
        assert all(t[0] is sb for t in nat), "one scheduler batch per device batch"
        a = self._native_arrays(sb)
        js = np.fromiter((t[1] for t in nat), np.int64, n)
        full = n == sb.n_slots and bool(np.all(js == np.arange(n)))
        row_off = np.zeros(n + 1, np.int32)
        np.cumsum(a["nrow"][js], out=row_off[1:])
        filt_off = np.zeros(n + 1, np.int32)
        np.cumsum(a["nfl"][js], out=filt_off[1:])
        rows = np.empty((int(row_off[-1]), 3), np.int32)
        filt = np.empty(max(1, int(filt_off[-1])), np.int32)
        sb.pack(a["idx"][js], rows, filt)
        rng_off = np.zeros(n + 1, np.int64)
        np.cumsum(a["nsz"][js], out=rng_off[1:])
        rng = self._native_draws(a, js, full, int(rng_off[-1]), ctx)
        x0 = a["x0"] if full else a["x0"][js]
        pred = np.array([s.pred for s in slots], np.int32)
        return x0, row_off, rows, rng_off, rng, pred, filt_off, filt

    @staticmethod
    def _native_draws(a, js, full, total, ctx):
        """The draws of slots ``js`` back to back: the span of the page-locked arena the
        flushes' draws were written into when they lie there in slot order (the usual
        case: handed to the library as it is, uploaded by DMA), else a gather."""
        if total == 0:
            return np.zeros(1, np.int32)
        outs = [o for o in a["outs"] if o is not None and o.size]
        if full and outs:
            lease = _lib.arena_of(outs[0])
            start = outs[0].__array_interface__["data"][0]
            pos = start
            for o in outs:
                if lease is None or _lib.arena_of(o) is not lease or o.__array_interface__["data"][0] != pos:
                    break
                pos += 4 * o.size
            else:
                if (pos - start) // 4 == total:
                    off = (start - lease.__array_interface__["data"][0]) // 4
                    return lease[off:off + total]
        flat = np.concatenate(outs) if outs else np.zeros(0, np.int32)
        if full:
            return np.ascontiguousarray(flat[:total], np.int32)
        doff, nsz = a["doff"], a["nsz"]
        parts = [flat[doff[j]:doff[j] + nsz[j]] for j in js.tolist() if nsz[j]]
        return np.concatenate(parts).astype(np.int32, copy=False) if parts else np.zeros(1, np.int32)

    def _run_slots(self, slots, ctx, fill, gate=None):
        t_run = time.perf_counter()
        n = len(slots)
        ctx = ctx or self.model.ctx
        packed = self._pack(slots, ctx)
        if gate is not None and not gate():
            return None
        t_lib = time.perf_counter()
        score, rank, _ = ctx.posttrain_rank(self._kp_hp, *packed)
        t_end = time.perf_counter()
        if fill:
            for i, s in enumerate(slots):
                s.result = {"target_score": float(score[i]), "target_rank": int(rank[i])}
        stats = {"slots": n, "rows": int(packed[1][-1]), "pack_s": t_lib - t_run, "lib_s": t_end - t_lib,
                 **ctx.last_timing()}
        if not fill:
            stats["_score"], stats["_rank"] = np.array(score), np.array(rank)
        if hasattr(ctx, "hot_intervals"):
            stats["hot_iv"] = ctx.hot_intervals()
        self.last_batch_stats = stats
        return stats

    def _base_result(self, key, slots, pending_base):
        if key in self.base_pt_results:
            return self.base_pt_results[key]
        res = slots[pending_base[key]].result
        self.base_pt_results[key] = res
        return res

    # ------------------------------------------------------------------ reference API
    def compute_relevance(self, pred, triples: list):
        return self.compute_relevance_batch(pred, [triples])[0]

    def compute_relevance_batch(self, pred, rules, checkpoints: list | None = None):
        raise NotImplementedError

    def _schedule_multi(self, items, checkpoints):
        raise NotImplementedError

    def _finalize_multi(self, slots, pending, jobs):
        raise NotImplementedError

    def _multi(self, items, checkpoints=None):
        t0 = time.perf_counter()
        self._deferred_error = None
        with self.rng.deferred():
            slots, pending, jobs = self._schedule_all(items, checkpoints)
        t_sched = time.perf_counter() - t0
        self._run(slots)
        self._collect(slots, self.last_batch_stats)
        self.last_batch_stats["schedule_s"] = t_sched
        outs = self._finalize_multi(slots, pending, jobs)
        self._raise_deferred(slots, pending)
        return outs

    def _batch_items(self, pred, rules):
        """compute_relevance_batch's one-item batch (the sufficient engine adds its
        conversion entities)."""
        return [(pred, rules)]

    def submit_batch(self, pred, rules, checkpoints: list | None = None, hold=False):
        """The first half of ``compute_relevance_batch``: schedule the rules' reference-order
        draws on this thread (with ``checkpoints`` as there) and start their device work on
        the next of two pipeline contexts, without waiting; :meth:`finish_batch` returns the
        relevances.  A later submit may be scheduled while this batch runs -- the
        builder's next speculative window (kelpie_amd/builder.py) -- and rewinding the
        generators to one of this batch's checkpoints undoes both.

        ``hold``: the batch's draws wait and its slots are packed on the batch thread, but
        its library call waits for :meth:`release_batch` (or :meth:`finish_batch`); a
        ``finish_batch(discard=True)`` before that cancels it without any device work."""
        import threading

        from . import rng as _rng_mod
        ctxs = self.model.contexts(2)
        self._submit_n = getattr(self, "_submit_n", -1) + 1
        ctx = ctxs[self._submit_n % len(ctxs)]
        busy = getattr(self, "_ctx_last", {}).get(id(ctx))
        if busy is not None:
            busy["thread"].join()  # a context runs one batch at a time (one context: no overlap)
        self._deferred_error = None
        with self.rng.deferred(detach=True) as d:
            slots, pending, jobs = self._schedule_all(self._batch_items(pred, rules), checkpoints)
        st = {"slots": slots, "pending": pending, "jobs": jobs, "deferred": self._deferred_error,
              "ticket": d.last_ticket, "error": None, "stats": None, "go": threading.Event(), "cancel": False}
        self._deferred_error = None
        if not hold:
            st["go"].set()

        def gate():
            st["go"].wait()
            return not st["cancel"]

        def run():
            try:
                _rng_mod.wait_ticket(st["ticket"])
                stats = self._run(slots, ctx=ctx, gate=gate)
                st["stats"] = dict(stats) if stats is not None else None
            except BaseException as e:  # re-raised by finish_batch
                st["error"] = e

        st["thread"] = threading.Thread(target=run, daemon=True)
        st["thread"].start()
        self._ctx_last = {**getattr(self, "_ctx_last", {}), id(ctx): st}
        return st

    def release_batch(self, st):
        """Let a held :meth:`submit_batch` batch start its device work."""
        st["go"].set()

    def finish_batch(self, st, discard=False):
        """Wait for a :meth:`submit_batch` batch and return its relevances (``discard``: only
        wait -- a speculative window the builder does not use -- and return None; a held
        batch not yet released is cancelled instead, with no device work)."""
        if discard and not st["go"].is_set():
            st["cancel"] = True
        st["go"].set()
        st["thread"].join()
        if discard:
            return None
        if st["error"] is not None:
            raise st["error"]
        self._collect(st["slots"], st["stats"])
        outs = self._finalize_multi(st["slots"], st["pending"], st["jobs"])
        self._deferred_error = st["deferred"]
        self._raise_deferred(st["slots"], st["pending"])
        return outs[0]

    def _raise_deferred(self, slots, pending):
        """Re-raise the reference's error of a call the batch stopped at, after caching
        the base post-training it had already run (post_training_engine.py:46-62)."""
        err, self._deferred_error = getattr(self, "_deferred_error", None), None
        if err is None:
            return
        for key, i in pending.items():
            self.base_pt_results.setdefault(key, slots[i].result)
        raise err

    def warm_contexts(self, items, depth=None):
        """Run the batch ``items`` once on every extra pipeline context, so their
        workspaces are allocated and the attention table image is built outside a
        timed region.  Consumes no random draws: the generator states are restored."""
        import os
        if depth is None:
            depth = int(os.environ.get("KELPIE_PIPELINE_DEPTH", "2"))
        ctxs = self.model.contexts(max(1, depth))
        if len(ctxs) < 2:
            return
        cp = StateCheckpoint()
        try:
            self.set_cache()
            self._deferred_error = None
            with self.rng.deferred():
                slots, _, _ = self._schedule_all(items, None)
            self._deferred_error = None
            for ctx in ctxs[1:]:
                st = self._run(slots, ctx=ctx)
                # a warm-up has no gather (_collect), so a sharded run's captured device
                # error is raised here (each rank warms the slots it owns)
                local = st.get("_local") if st else None
                if local is not None and local[4] is not None:
                    raise local[4]
        finally:
            cp.restore()
            self.set_cache()

    def compute_relevance_pipeline(self, batches, depth=None):
        """Equivalent to ``[(self.set_cache(), self.compute_relevance_multi(b))[1] for b in batches]``
        but the host schedules batch k+1 (its reference-order random draws and
        slot assembly) while batch k runs on the device: the library call
        releases the GIL.  Draw order is unchanged because scheduling stays
        sequential on this thread; each batch starts from a cleared cache, so no
        batch's schedule depends on another's results.  ``last_batch_stats`` is
        a list of the per-batch stats.

        With ``depth`` > 1 (default ``KELPIE_PIPELINE_DEPTH``, else 2) up to that many
        batches are in flight, each on its own device context
        (``FrozenModel.contexts``: own stream and workspaces over a replica of the
        frozen tables), so one batch's library-side planning, uploads and result
        download overlap the other's kernels instead of leaving the device idle."""
        import collections
        import os
        import threading

        if depth is None:
            depth = int(os.environ.get("KELPIE_PIPELINE_DEPTH", "2"))
        ctxs = self.model.contexts(max(1, depth))
        # The scheduling thread and the batch threads' packing share the interpreter lock;
        # KELPIE_GIL_SWITCH_US shortens the interpreter's switch interval while the
        # pipeline runs (A/B switch; unset: the interpreter's default)
        import gc
        import sys
        # no cyclic garbage collection while batches are in flight (KELPIE_PIPELINE_NOGC=0
        # keeps it): a collection pass on the scheduling thread holds the interpreter lock
        # for milliseconds while the batch threads wait to pack and launch (headline +1.5 %,
        # three alternating pairs on one box, profiles/r04q/); the objects are freed by
        # reference counting either way, and collection resumes when the call returns
        nogc = os.environ.get("KELPIE_PIPELINE_NOGC", "1") == "1" and gc.isenabled()
        if nogc:
            gc.disable()
        old_switch = sys.getswitchinterval()
        if os.environ.get("KELPIE_GIL_SWITCH_US"):
            sys.setswitchinterval(float(os.environ["KELPIE_GIL_SWITCH_US"]) * 1e-6)

        from . import rng as _rng_mod

        # KELPIE_PIPELINE_TRACE=<path>: a JSON list of (seconds, event, batch) per pipeline
        # stage, for host timelines (diagnostics; tools/pipeline_trace.py)
        trace_path = os.environ.get("KELPIE_PIPELINE_TRACE")
        trace = [] if trace_path else None

        def tr(ev, b):
            if trace is not None:
                trace.append((time.perf_counter(), ev, b))

        # one long-lived worker thread per device context, fed through a queue: starting a
        # batch is a put, not a thread start (Thread.start waits for the new thread to run:
        # ~0.4 ms of the scheduling thread per TransE batch, trace r05r)
        import queue as _queue

        class _Worker:
            def __init__(self):
                self.q = _queue.SimpleQueue()
                self.t = threading.Thread(target=self._loop, daemon=True)
                self.t.start()

            def _loop(self):
                while True:
                    st = self.q.get()
                    if st is None:
                        return
                    try:
                        run(st)
                    finally:
                        st["done"].set()

        class _Handle:  # Thread's join / is_alive over a worker's queued batch
            def __init__(self, worker, st):
                self.ev = st["done"] = threading.Event()
                worker.q.put(st)

            def join(self):
                self.ev.wait()

            def is_alive(self):
                return not self.ev.is_set()

        workers = {}
        use_workers = os.environ.get("KELPIE_PIPELINE_WORKERS", "1") == "1"

        def run(state):
            try:
                b = state["b"]
                tr("run", b)
                # this batch's deferred draws (the scheduling thread did not wait for them)
                _rng_mod.wait_ticket(state.get("ticket"))
                tr("draws", b)
                state["stats"] = dict(self._run(state["slots"], ctx=state["ctx"]))
                tr("ran", b)
            except BaseException as e:  # re-raised on the scheduling thread
                state["error"] = e

        tr("enter", -1)
        outs, stats, inflight = [], [], collections.deque()
        late_collect = os.environ.get("KELPIE_PIPELINE_EARLY_START", "1") == "0"  # A/B: collect, then start
        detach = os.environ.get("KELPIE_PIPELINE_DETACH", "1") == "1"

        def finish(state):
            state["thread"].join()
            tr("finish", state["b"])
            if state.get("error") is not None:
                raise state["error"]
            self.base_pt_results = {}
            self._collect(state["slots"], state["stats"])
            o = self._finalize_multi(state["slots"], state["pending"], state["jobs"])
            st = state["stats"]
            st["schedule_s"] = state["schedule_s"]
            stats.append(st)
            outs.append(o)
            self._deferred_error = state.get("deferred")
            tr("finished", state["b"])
            self._raise_deferred(state["slots"], state["pending"])

        # KELPIE_PIPELINE_LOOKAHEAD=N: batches scheduled ahead of the contexts, so that a freed
        # context starts the next batch at once instead of after that batch's schedule (the
        # headline trace r05n shows a context idle ~3 ms while the next batch was scheduled).
        # Measured, alternating on one box (profiles/r05/r05w/): 1 against 0, headline
        # 868 / 878 / 875 vs 884 / 894 / 891 cand/s, ConvE 454 / 456 vs 456 / 457; default 0
        # (each batch scheduled when the previous one has started)
        lookahead = max(0, int(os.environ.get("KELPIE_PIPELINE_LOOKAHEAD", "0")))
        ready = collections.deque()
        todo = iter(enumerate(batches))
        stop = False

        def schedule_next():
            """Schedule the next batch into `ready`; False when there is none."""
            nonlocal stop
            nxt = next(todo, None)
            if nxt is None:
                stop = True
                return False
            b, items = nxt
            self.set_cache()
            t0 = time.perf_counter()
            tr("schedule", b)
            self._deferred_error = None
            # detached: the next batch is scheduled while the workers still make this
            # one's draws (TransE: the sequential numpy chain); the batch thread waits
            # for them before packing (KELPIE_PIPELINE_DETACH=0: wait here, A/B)
            with self.rng.deferred(detach=detach) as drng:
                slots, pending, jobs = self._schedule_all(items, None)
            err, self._deferred_error = self._deferred_error, None
            tr("scheduled", b)
            ready.append({"slots": slots, "pending": pending, "jobs": jobs,
                          "schedule_s": time.perf_counter() - t0, "error": None, "deferred": err,
                          "ticket": drng.last_ticket, "b": b})
            if err is not None:
                stop = True  # the sequential reference stops at the failing call
            return True

        def start_next(done):
            """Start the oldest ready batch on its context (batch b uses context b % depth:
            the batch before it there is in `done` or was finished earlier), then collect
            the finished ones: their collection (and the gather, sharded) runs while the
            new batch packs and launches instead of ahead of it."""
            if late_collect or any(d.get("error") is not None for d in done):
                for d in done:
                    finish(d)  # raises the first device failure before the next batch starts
                done = []
            state = ready.popleft()
            state["ctx"] = ctxs[state["b"] % len(ctxs)]
            ci = state["b"] % len(ctxs)
            if not use_workers:  # KELPIE_PIPELINE_WORKERS=0: a thread per batch (A/B)
                state["thread"] = threading.Thread(target=run, args=(state,), daemon=True)
                state["thread"].start()
            else:
                if ci not in workers:
                    workers[ci] = _Worker()
                state["thread"] = _Handle(workers[ci], state)
            inflight.append(state)
            for d in done:
                finish(d)

        def join_oldest():
            old = inflight.popleft()
            old["thread"].join()
            tr("joined", old["b"])
            return old

        try:
            while True:
                if ready and (len(inflight) < len(ctxs) or not inflight[0]["thread"].is_alive()):
                    start_next([join_oldest()] if len(inflight) >= len(ctxs) else [])
                elif not stop and len(ready) <= lookahead:
                    schedule_next()
                elif ready:
                    start_next([join_oldest()])  # scheduled far enough ahead: wait for a context
                else:
                    break
            while inflight:
                finish(inflight.popleft())
        finally:
            for st in inflight:  # an earlier batch raised: let the others' device work end
                st["thread"].join()
            for w in workers.values():
                w.q.put(None)
            sys.setswitchinterval(old_switch)
            if nogc:
                gc.enable()
            tr("unwound", -1)
            if sys.exc_info()[0] is None:
                _rng_mod.sync()  # the generators are current again when the call returns
            else:
                try:
                    _rng_mod.sync()
                except Exception:  # noqa: BLE001 -- the error in flight is the one to report
                    pass
            tr("exit", -1)
            if trace is not None:
                import json
                with open(trace_path, "a") as f:
                    f.write(json.dumps(trace) + "\n")
        self.last_batch_stats = stats
        return outs


class NecessaryPostTrainingEngine(PostTrainingEngine):
    """post_training_engine.py:128-157."""

    def compute_relevance_batch(self, pred, rules, checkpoints: list | None = None):
        """Relevances of ``rules`` for ``pred``, identical to calling
        ``compute_relevance`` on each rule in order.  When ``checkpoints`` is a
        list, the generator state after each rule's draws is appended to it."""
        return self.compute_relevance_multi([(pred, rules)], checkpoints)[0]

    def compute_relevance_multi(self, items, checkpoints: list | None = None):
        """[(pred, rules), ...] -> [[relevance per rule], ...] in ONE device batch;
        equal to the sequential compute_relevance calls in that order."""
        return self._multi(items, checkpoints)

    def _calls(self, items):
        """(pred, rule, mode) of every call _schedule_multi makes, in order."""
        for pred, rules in items:
            for rule in rules:
                yield pred, [tuple(t) for t in rule], "necessary"
                if not rule:
                    return

    def _schedule_multi(self, items, checkpoints):
        slots, pending, jobs = [], {}, []
        fast = checkpoints is None and getattr(self.model, "fused_call_draws", False)
        for pred, rules in items:
            if fast and all(len(r) for r in rules):
                jobs.append(self._schedule_fused_pred(pred, rules, "necessary", slots, pending))
                continue
            pj = []
            for rule in rules:
                rule = [tuple(t) for t in rule]
                idx = self._schedule(pred, rule, "necessary", slots, pending)
                if not rule:
                    # KelpieDataset.undo_removal raises after the post-training
                    # (kelpie_dataset.py:166-167): its draws are spent, nothing after it runs
                    self._deferred_error = Exception("No removal to undo.")
                    jobs.append(pj)
                    return slots, pending, jobs
                pj.append(idx)
                if checkpoints is not None:
                    self._flush_fused()
                    checkpoints.append(StateCheckpoint())
            jobs.append(pj)
        return slots, pending, jobs

    def _finalize_multi(self, slots, pending, jobs):
        minimizer = self.model.is_minimizer()
        outs = []
        self.last_results = []
        rank_w, sig_w, lens = [], [], []
        for pj in jobs:
            lens.append(len(pj))
            for pt_idx, key in pj:
                base = self._base_result(key, slots, pending)
                pt = slots[pt_idx].result
                rank_w.append(pt["target_rank"] - base["target_rank"])
                if minimizer:
                    score_worsening = pt["target_score"] - base["target_score"]
                else:
                    score_worsening = base["target_score"] - pt["target_score"]
                sig_w.append(_sigmoid(score_worsening))
                self.last_results.append((pt, base))
        # int64 tensor + python float -> float32 tensor (A-Q5): one float32 add per call,
        # element-wise over the batch (the same bits as the scalar form)
        rel = (np.asarray(rank_w, np.int64).astype(np.float32) + np.asarray(sig_w, np.float64).astype(np.float32)).tolist()
        k = 0
        for n in lens:
            outs.append(rel[k:k + n])
            k += n
        return outs


class SufficientPostTrainingEngine(PostTrainingEngine):
    """post_training_engine.py:160-207."""

    def __init__(self, model, dataset, hp, rng=None):
        super().__init__(model, dataset, hp, rng)
        self.entities_to_convert = []

    def compute_relevance_batch(self, pred, rules, checkpoints: list | None = None):
        return self.compute_relevance_multi([(pred, rules, self.entities_to_convert)], checkpoints)[0]

    def _batch_items(self, pred, rules):
        return [(pred, rules, self.entities_to_convert)]

    def compute_relevance_multi(self, items, checkpoints: list | None = None):
        """[(pred, rules, entities_to_convert), ...] in ONE device batch."""
        return self._multi(items, checkpoints)

    def _calls(self, items):
        """(pred, rule, mode) of every call _schedule_multi makes, in order."""
        for pred, rules, ents in items:
            pred = tuple(int(v) for v in pred)
            s = pred[0]
            for rule in rules:
                if not ents:
                    return
                for e in ents:
                    crule = Dataset.replace_entity_in_triples([tuple(t) for t in rule], s, e)
                    yield Dataset.replace_entity_in_triple(pred, s, e), crule, "sufficient"
                    if not crule:
                        return

    def _schedule_multi(self, items, checkpoints):
        slots, pending, jobs = [], {}, []
        for pred, rules, ents in items:
            pred = tuple(int(v) for v in pred)
            s = pred[0]
            pj = []
            for rule in rules:
                if not ents:
                    self._deferred_error = ZeroDivisionError("division by zero")  # sum([]) / len([])
                    jobs.append(pj)
                    return slots, pending, jobs
                rj = []
                for e in ents:
                    crule = Dataset.replace_entity_in_triples([tuple(t) for t in rule], s, e)
                    cpred = Dataset.replace_entity_in_triple(pred, s, e)
                    rj.append(self._schedule(cpred, crule, "sufficient", slots, pending))
                    if not crule:
                        # KelpieDataset.undo_addition raises after the first conversion's
                        # post-training (kelpie_dataset.py:191-192)
                        self._deferred_error = Exception("No addition to undo.")
                        jobs.append(pj)
                        return slots, pending, jobs
                pj.append(rj)
                if checkpoints is not None:
                    self._flush_fused()
                    checkpoints.append(StateCheckpoint())
            jobs.append(pj)
        return slots, pending, jobs

    def _finalize_multi(self, slots, pending, jobs):
        minimizer = self.model.is_minimizer()
        outs = []
        self.last_results = []
        for pj in jobs:
            out = []
            for rj in pj:
                rels, det = [], []
                for pt_idx, key in rj:
                    base = self._base_result(key, slots, pending)
                    pt = slots[pt_idx].result
                    det.append((pt, base))
                    rank_improvement = base["target_rank"] - pt["target_rank"]
                    if minimizer:
                        score_improvement = base["target_score"] - pt["target_score"]
                    else:
                        score_improvement = pt["target_score"] - base["target_score"]
                    rel = float(np.float32(np.float32(rank_improvement) + np.float32(_sigmoid(score_improvement))))
                    rel /= float(base["target_rank"])
                    rels.append(rel)
                self.last_results.append(det)
                out.append(sum(rels) / len(rels))
            outs.append(out)
        return outs
