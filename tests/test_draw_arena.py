"""The deferred-draw arenas (kelpie_amd.rng / _lib.pinned_i32) and how a batch's draws
reach the library (engine._contiguous_draws): a pooled arena is reused only once no
view of it is alive, and draws written back to back into one pooled arena are handed
over as that span (no copy), anything else as a gathered copy with the same values.
A pageable array stands in for the page-locked one (no GPU here)."""
import gc

import numpy as np
import pytest

from kelpie_amd import _lib, engine


class _Slot:
    def __init__(self, rng):
        self.rng = rng


@pytest.fixture
def pool(monkeypatch):
    p, idle = [], []
    monkeypatch.setattr(_lib, "_PINNED", p)
    monkeypatch.setattr(_lib, "_PINNED_IDLE", idle)
    monkeypatch.setattr(_lib, "_PINNED_MAX", 2)
    monkeypatch.setattr(_lib, "_PINNED_OK", True)

    def add(a):
        p.append(a)
        idle.append(True)
        return _lib._lease(len(p) - 1)
    return add


def test_pool_reuses_idle_arena_only(pool):
    lease = pool(np.arange(100, dtype=np.int32))
    assert _lib.is_pinned(lease)
    view = lease[10:20]  # a batch's draws alive
    flat = np.asarray(view).reshape(-1)  # a plain view of a view still holds the lease
    del lease, view
    gc.collect()
    assert not _lib._PINNED_IDLE[0]
    # busy: the pool is not full, but the next allocation needs the library; full pool -> None
    pool(np.zeros(10, np.int32))
    del flat
    gc.collect()
    assert _lib._PINNED_IDLE[0]
    got = _lib.pinned_i32(50)
    assert got is not None and got.base is _lib._PINNED[0] and not _lib._PINNED_IDLE[0]
    assert _lib.pinned_i32(50) is None  # the other array is busy too (its lease above) or small


def test_contiguous_span_is_handed_over_without_copy(pool):
    arena = pool(np.zeros(1000, np.int32))
    arena[:] = np.arange(1000)
    slots = [_Slot(arena[5:15]), _Slot(np.zeros(0, np.int32)), _Slot(arena[15:40]), _Slot(arena[40:41])]
    out = engine._contiguous_draws(slots, 36, None)
    assert _lib.arena_of(out) is arena
    assert out.__array_interface__["data"][0] == arena[5:].__array_interface__["data"][0]
    assert np.array_equal(out, np.arange(5, 41))


def test_gap_or_foreign_array_falls_back_to_copy(pool):
    arena = pool(np.arange(1000, dtype=np.int32))
    slots = [_Slot(arena[5:15]), _Slot(arena[20:30])]  # a gap
    out = engine._contiguous_draws(slots, 20, None)
    assert not np.shares_memory(out, arena)
    assert np.array_equal(out, np.concatenate([np.arange(5, 15), np.arange(20, 30)]))
    loose = np.arange(7, dtype=np.int32)  # not pooled
    out = engine._contiguous_draws([_Slot(loose)], 7, None)
    assert np.array_equal(out, loose)
