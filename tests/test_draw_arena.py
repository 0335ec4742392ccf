"""The deferred-draw arenas (kelpie_amd.rng / _lib.pinned_i32) and how a batch's draws
reach the library (engine._contiguous_draws): a pooled arena is reused only once no
view of it is alive, and draws written back to back into one pooled arena are handed
over as that span (no copy), anything else as a gathered copy with the same values.
A pageable array stands in for the page-locked one (no GPU here)."""
import sys

import numpy as np
import pytest

from kelpie_amd import _lib, engine


class _Slot:
    def __init__(self, rng):
        self.rng = rng


@pytest.fixture
def pool(monkeypatch):
    p = []
    monkeypatch.setattr(_lib, "_PINNED", p)
    monkeypatch.setattr(_lib, "_PINNED_MAX", 2)
    monkeypatch.setattr(_lib, "_PINNED_OK", True)
    return p


def test_pool_reuses_idle_arena_only(pool):
    a = np.arange(100, dtype=np.int32)
    pool.append(a)
    del a
    got = _lib.pinned_i32(50)
    assert got is pool[0]
    view = got[10:20]  # a batch's draws alive
    del got
    assert sys.getrefcount(pool[0]) > 3
    # busy: the pool is not full, but the next allocation needs the library; full pool -> None
    pool.append(np.zeros(10, np.int32))
    assert _lib.pinned_i32(50) is None
    del view
    assert _lib.pinned_i32(50) is pool[0]


def test_contiguous_span_is_handed_over_without_copy(pool):
    arena = np.zeros(1000, np.int32)
    pool.append(arena)
    arena[:] = np.arange(1000)
    slots = [_Slot(arena[5:15]), _Slot(np.zeros(0, np.int32)), _Slot(arena[15:40]), _Slot(arena[40:41])]
    out = engine._contiguous_draws(slots, 36, None)
    assert out.base is arena and out.__array_interface__["data"][0] == arena[5:].__array_interface__["data"][0]
    assert np.array_equal(out, np.arange(5, 41))


def test_gap_or_foreign_array_falls_back_to_copy(pool):
    arena = np.arange(1000, dtype=np.int32)
    pool.append(arena)
    slots = [_Slot(arena[5:15]), _Slot(arena[20:30])]  # a gap
    out = engine._contiguous_draws(slots, 20, None)
    assert not np.shares_memory(out, arena)
    assert np.array_equal(out, np.concatenate([np.arange(5, 15), np.arange(20, 30)]))
    loose = np.arange(7, dtype=np.int32)  # not pooled
    out = engine._contiguous_draws([_Slot(loose)], 7, None)
    assert np.array_equal(out, loose)
