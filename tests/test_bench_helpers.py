"""bench.py's roofline helpers (host only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_union_seconds_merges_overlapping_launches():
    # two contexts' launches interleaved on one time base: overlaps count once
    iv = [[0.0, 1.0], [0.5, 2.0], [3.0, 4.0], [3.5, 3.6], [2.0, 2.5]]
    assert bench.union_seconds(iv) == 3.5
    assert bench.union_seconds([[0.0, 1.0], [2.0, 3.0]]) == 2.0
    assert bench.union_seconds([]) == 0.0
