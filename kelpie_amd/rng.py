"""Host RNG protocol: the reference's random draws, in the reference's order.

Post-training is stochastic.  The reference draws from
three process-global generators while it runs candidate after candidate:

* torch CPU generator: the kelpie init ``torch.rand(1, D)``
  (post_training_engine.py:52), TransE's ``xavier_normal_`` on the kelpie row
  (transe.py:93-95), the ``reset_parameters()`` of the throw-away Conv2d /
  Linear every ``KelpieConvE`` builds (conve.py:46-52 via :202),
  ``torch.randperm`` per ComplEx epoch (multiclass_nll_optimizer.py:148),
  ``torch.randint`` negatives per TransE epoch (pairwise_ranking_optimizer.py:171-172)
  and ConvE's hidden-dropout masks (Dropout left in train mode, model.py:114-125);
* numpy global ``RandomState``: ``np.random.shuffle`` of the TransE rows
  (pairwise_ranking_optimizer.py:166);
* python ``random``: builder termination and conversion-entity sampling.

The batched GPU engine evaluates many candidates at once, so the host draws
every candidate's numbers up front, in exactly the reference's sequence, from
the same generators, and ships them to the kernels (RNG-as-input).  Seeded
identically, the engine therefore sees bit-identical draws to the reference.

Draws whose VALUES the kernels never need are skipped by advancing the
generator state (:func:`kelpie_amd._lib.mt19937_discard`): a ComplEx epoch
whose rows fit one minibatch only reorders the batch, and a ConvE model
construction only burns ``32*9 + 32 + hidden*dim + dim`` outputs.
Consumption counts (randperm(n): n-1 outputs, randint: one per element,
bernoulli_: two per element) are pinned by ``tests/test_rng_protocol.py``.
"""
from __future__ import annotations

import contextlib
import math
import os
import threading

import numpy as np
import torch

from . import _lib


def _get_state():
    # get_rng_state() returns a fresh copy of the generator state: its numpy view is ours
    return torch.get_rng_state().numpy()


def _set_state(st):
    torch.set_rng_state(torch.from_numpy(st))


_STATE_LEN = None

# KP_RNG_ASYNC=0: the TransE torch-stream walk on the scheduling thread (A/B switch)
_ASYNC = __import__('os').environ.get('KP_RNG_ASYNC', '1') != '0'


def _state_shape():
    """A buffer shaped like torch's generator state (for calls that do not read it)."""
    global _STATE_LEN
    if _STATE_LEN is None:
        _STATE_LEN = torch.get_rng_state().numel()
    return np.zeros(_STATE_LEN, np.uint8)


def _np_mt_state_address() -> int:
    """Address of the global RandomState's ``mt19937_state`` (numpy/random/src/mt19937/mt19937.h)."""
    return int(np.random.mtrand._rand._bit_generator.ctypes.state_address)


# TransE draws queued by ReferenceRNG.deferred() and not yet waited for: the live numpy
# state belongs to the library's worker until sync()
_outstanding = False


# every arena the library's workers may still be writing into stays referenced here
# until sync(): a caller that drops its draw arrays early must not free them under the
# workers
_inflight = []
_PINNED_ARENAS = os.environ.get("KP_PINNED_ARENA", "1") != "0"


# torch-generator outputs owed by draws whose values nobody needs (the slots another
# rank post-trains, kelpie_amd.distributed): accumulated and applied as ONE discard
# before the next real torch draw or state read
_skip = 0


# True while a library walk (kp_rng_transe_calls_async) carries the torch stream: torch's
# own state is stale until _torch_current() takes the stream back
_torch_async = False


# set when a background walk or draw task failed (sync): the generators then sit at a
# state the reference never reaches, so every later draw or state read raises until the
# caller reseeds and calls clear_poison(), or restores a StateCheckpoint
_poisoned = None


# ticket -> the arrays a detached block's workers write (its arena, the walk's outputs):
# kept alive until the ticket is waited for or a full sync, then released, so that a
# pipeline's arenas go back to the page-locked pool batch by batch instead of all at the
# end of the call (with every arena held, the pool ran dry after 4 batches and each later
# batch took a fresh 64 MiB pageable arena: first-touch faults in the draw workers and a
# ~50 ms release at the call's end, TransE FB15k-237 on the box)
_detached = {}
_detached_lock = threading.Lock()  # batch threads release while the scheduling thread adds


def wait_ticket(ticket):
    """Wait for the draws of a detached deferred block (ReferenceRNG.deferred(detach=True))
    and of every block before it; a failed draw marks the stream lost."""
    global _poisoned
    if ticket is None:
        return
    try:
        _lib.rng_batch_wait(ticket)
    except Exception as exc:
        _poisoned = repr(exc)
        raise
    # this block's and every earlier block's draws are complete
    with _detached_lock:
        for t in [t for t in _detached if t <= ticket]:
            del _detached[t]


def clear_poison():
    """Accept the generators' current state again after a failed background draw (call
    after reseeding them)."""
    global _poisoned
    _poisoned = None


def _check_poison():
    if _poisoned is not None:
        raise RuntimeError("reference RNG stream lost by a failed background draw (" + _poisoned + "); reseed the "
                           "generators and call kelpie_amd.rng.clear_poison(), or restore a StateCheckpoint")


def _torch_current():
    """Make torch's generator current: take the stream back from an asynchronous walk."""
    global _torch_async
    _check_poison()
    if _torch_async:
        _torch_async = False
        st = torch.get_rng_state().numpy()
        _lib.torch_take(st)
        _set_state(st)


def _flush_skip():
    global _skip
    _torch_current()
    if _skip:
        n, _skip = _skip, 0
        st = _get_state()
        _lib.mt19937_discard(st, n)
        _set_state(st)


def sync():
    """Wait for every queued TransE draw (the numpy global state is then current) and
    apply any pending torch-generator advance."""
    global _outstanding, _torch_async, _skip
    if _outstanding:
        _outstanding = False
        try:
            _lib.rng_wait()
        except Exception as exc:
            # a failed walk or draw task: the stream it carried is partial, so drop the
            # asynchronous state and the pending advance instead of installing either
            # on a later draw, mark the stream lost, then report the failure
            global _poisoned
            _torch_async = False
            _skip = 0
            _inflight.clear()
            with _detached_lock:
                _detached.clear()
            _poisoned = repr(exc)
            raise
    _inflight.clear()
    with _detached_lock:
        _detached.clear()
    _flush_skip()  # also takes the torch stream back from an asynchronous walk


class ReferenceRNG:
    """Draws from the process-global torch / numpy generators (reference order)."""

    _defer_depth = 0

    @contextlib.contextmanager
    def deferred(self, detach=False):
        """Inside this block :meth:`transe_epochs` returns arrays that the library's
        workers fill in the background (kp_rng_transe_enqueue): the caller keeps
        scheduling while the shuffles and randints of earlier slots are generated.
        The arrays are complete, and numpy's global state current, on exit (or
        after :func:`sync`).

        ``detach``: on exit the block's draws are only closed as one batch
        (kp_rng_batch_close; ``self.last_ticket``) instead of waited for, so the caller
        can schedule the next block while the workers still make these draws; whoever
        reads this block's arrays first calls :func:`wait_ticket` (the pipeline's batch
        thread, before packing).  The generators stay with the workers until the next
        :func:`sync` (a state read or a torch draw on this thread syncs first)."""
        self._defer_depth += 1
        if self._defer_depth == 1:
            self._arena, self._arena_pos = None, 0
        self.last_ticket = None
        try:
            yield self
        finally:
            self._defer_depth -= 1
            if self._defer_depth == 0:
                self._arena = None
                if detach and _outstanding and not _skip:
                    self.last_ticket = _lib.rng_batch_close()
                    # the block's arrays now belong to its ticket (wait_ticket releases them)
                    with _detached_lock:
                        _detached[self.last_ticket] = list(_inflight)
                    _inflight.clear()
                else:
                    sync()

    # The deferred draws of one block are laid out back to back in an arena, so the
    # engine ships a batch's draws without concatenating them (engine._run).  A fresh
    # arena per block: the arrays of an earlier batch may still be in flight.
    # int32 words of a fresh arena: one TransE FB15k-237 batch's draws (~6 M words) fit, so
    # they stay one contiguous span.  A pooled page-locked arena (_lib.pinned_i32) is
    # committed and locked when allocated: the pool holds at most KP_PINNED_ARENAS (6) of
    # them, 384 MiB per process; a pageable one commits only the pages written.
    _ARENA = 1 << 24

    def _take(self, n: int) -> np.ndarray:
        if self._arena is None or self._arena_pos + n > self._arena.size:
            size = max(self._ARENA, n)
            # page-locked and reused when the library can give it (the device reads the
            # batch's draws from here by DMA, engine._contiguous_draws); else pageable
            a = _lib.pinned_i32(size) if _PINNED_ARENAS else None
            self._arena, self._arena_pos = (a if a is not None else np.empty(size, np.int32)), 0
            _inflight.append(self._arena)
        out = self._arena[self._arena_pos:self._arena_pos + n]
        self._arena_pos += n
        return out

    # ---------------------------------------------------------------- model construction
    def rand_init(self, D: int) -> np.ndarray:
        _flush_skip()
        return torch.rand(1, D).numpy()[0]  # float32 already

    def skip_rand_init(self, D: int):
        """Consume torch.rand(1, D) without its values (one output per float32 element)."""
        self.discard(D)

    def xavier_row(self, d: int) -> np.ndarray:
        # xavier_normal_ on a (1, d) parameter: normal_(0, sqrt(2 / (d + 1)))
        _flush_skip()
        return torch.empty(1, d).normal_(0.0, math.sqrt(2.0 / float(d + 1))).numpy()[0]  # float32 already

    def discard(self, n: int):
        """Advance the torch generator by n outputs (deferred to the next real draw)."""
        global _skip
        _check_poison()
        if n > 0:
            _skip += int(n)
        if not self._defer_depth:
            _flush_skip()  # outside a deferred block nobody else flushes it

    def conve_construction(self, hidden: int, dim: int):
        self.discard(32 * 9 + 32 + hidden * dim + dim)

    # ---------------------------------------------------------------- per-optimizer draws
    def complex_epochs(self, R: int, epochs: int, batch_size: int, want: bool = True) -> np.ndarray:
        """Per-epoch ``torch.randperm(R)`` (R - 1 outputs each); values are only needed
        when an epoch has more than one minibatch (and ``want``: the slot is post-trained
        here)."""
        if R > batch_size and want:
            _flush_skip()
            return np.concatenate([torch.randperm(R).numpy().astype(np.int32) for _ in range(epochs)]) \
                if epochs else np.zeros(0, np.int32)
        self.discard(epochs * max(R - 1, 0))
        return np.zeros(0, np.int32)

    def transe_epochs(self, R: int, epochs: int, ratio: int, n_entities: int) -> np.ndarray:
        """Per epoch [row order (R) | negative entity (R) | head_or_tail (R)].

        The row order composes the in-place ``np.random.shuffle`` of every epoch;
        of the ``ratio*R`` randint draws only the first R are stepped (SURVEY A-Q2).
        Generated in C++ from the two generators' states (kp_rng_transe_epochs)."""
        if epochs <= 0:
            return np.zeros(0, np.int32)
        global _outstanding
        _flush_skip()
        st = _get_state()
        # numpy's global MT19937 is advanced in place through its C state struct
        # (BitGenerator.ctypes.state_address -> {uint32 key[624]; int pos}):
        # get_state/set_state would cost ~0.1 ms per slot
        addr = _np_mt_state_address()
        if self._defer_depth:
            out = _lib.transe_enqueue(st, addr, addr + 4 * 624, R, epochs, ratio, n_entities,
                                      self._take(epochs * 3 * R))
            _outstanding = True
        else:
            sync()
            out = _lib.transe_epochs(st, addr, addr + 4 * 624, R, epochs, ratio, n_entities)
        _set_state(st)
        return out

    def transe_calls(self, D: int, d: int, R_base, R_pt, epochs: int, ratio: int, n_entities: int, want=None,
                     raw=False):
        """Every draw of n TransE compute_relevance calls in one library call
        (kp_rng_transe_calls).  Per call: ``torch.rand(1, D)``, the base row's
        ``xavier_normal_``, the base post-training's epoch draws (``R_base[i]`` >= 0),
        the post-trained row's ``xavier_normal_`` and its epoch draws (``R_pt[i]`` >= 0).
        Returns ``(x_base [n][d], x_pt [n][d], [(draws_base, draws_pt)] * n)``; the draws
        are complete on leaving :meth:`deferred` (or at once outside it).  ``want[i]``
        (bit 0 base, bit 1 pt; default all): an unwanted post-training's draws are not
        made, only the generators advance past them (its entry is an empty array).
        ``raw``: return ``(x_base, x_pt, out, sizes)`` instead, with ``sizes`` [n][2] the
        draw counts of each call's base and pt post-training, laid out back to back in
        ``out`` in call order (no per-call arrays: the engine's TransE fast path packs
        from them directly)."""
        _check_poison()
        global _outstanding, _torch_async
        addr = _np_mt_state_address()
        rbv = np.maximum(np.asarray(R_base, np.int64), 0)
        rpv = np.maximum(np.asarray(R_pt, np.int64), 0)
        wa = None if want is None else np.array(want, np.uint8)
        sz = np.empty((len(rbv), 2), np.int64)
        sz[:, 0] = epochs * 3 * rbv
        sz[:, 1] = epochs * 3 * rpv
        if wa is not None:
            sz[:, 0] *= (wa & 1) != 0
            sz[:, 1] *= (wa & 2) != 0
        total = int(sz.sum())
        std = float(np.float32(math.sqrt(2.0 / float(d + 1))))
        if self._defer_depth and _ASYNC:
            # the torch-stream walk runs on the library's walker thread; a walk already
            # carrying the stream continues it (the state passed is then not read)
            if _skip or not _torch_async:
                _flush_skip()
                st = _get_state()
            else:
                st = _state_shape()
            out = self._take(total) if total else None
            xb, xp, queued = _lib.transe_calls_async(st, addr, addr + 4 * 624, _lib.normal_cap(), D, d, std, R_base,
                                                     R_pt, epochs, ratio, n_entities, out, wa)
            _inflight.extend((xb, xp))  # the walk writes them until sync(), wanted or not
            if queued:
                _torch_async = True
            else:  # walked inline (no walker thread): st is the advanced stream, nothing carried
                _set_state(st)
            _outstanding = True
        else:
            _flush_skip()
            if not self._defer_depth:
                sync()
            st = _get_state()
            out = (self._take(total) if self._defer_depth else np.empty(total, np.int32)) if total else None
            xb, xp = _lib.transe_calls(st, addr, addr + 4 * 624, _lib.normal_cap(), D, d, std, R_base, R_pt, epochs,
                                       ratio, n_entities, out, wa)
            _outstanding = True
            if not self._defer_depth:
                sync()
            _set_state(st)
        if raw:
            return xb, xp, out, sz
        draws, off, empty = [], 0, np.zeros(0, np.int32)
        for a, b in sz.tolist():
            draws.append((out[off:off + a] if a else empty, out[off + a:off + a + b] if b else empty))
            off += a + b
        return xb, xp, draws

    def conve_masks(self, n_rows_per_step, segs) -> np.ndarray:
        """ConvE dropout keep bits for every step, packed per step and dropout in uint32
        words.  ``segs`` = [(elements per pair, rate)] of the dropouts with a non-zero
        rate, in the forward's order (input image, feature-map channels, hidden;
        conve.py:142,147,151)."""
        segs = [(int(n), float(p)) for n, p in segs if p > 0.0]
        if not segs or len(n_rows_per_step) == 0:
            return np.zeros(0, np.int32)
        keep = [(n, 1.0 - p) for n, p in segs]
        global _outstanding
        _flush_skip()
        st = _get_state()
        if self._defer_depth:
            words = _lib.conve_masks_enqueue(st, n_rows_per_step, keep,
                                             self._take(_lib.mask_words(n_rows_per_step, [n for n, _ in keep])))
            _outstanding = True
        else:
            words = _lib.conve_masks(st, n_rows_per_step, keep)
        _set_state(st)
        return words.view(np.int32)


class StateCheckpoint:
    """Snapshot of the torch / numpy generators (to rewind speculative draws)."""

    def __init__(self):
        sync()
        self.torch_state = torch.get_rng_state()
        self.np_state = np.random.get_state()

    def restore(self):
        global _poisoned
        try:
            sync()
        except Exception:  # noqa: BLE001 -- the restored state replaces whatever was lost
            pass
        _poisoned = None
        torch.set_rng_state(self.torch_state)
        np.random.set_state(self.np_state)
