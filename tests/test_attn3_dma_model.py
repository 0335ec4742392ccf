"""kp_attn3's LDS address model (tools/attn3_dma_model.py): for every instantiated row
width and both LDS-DMA forms, no LDS read of a key tile touches a byte that an LDS-DMA
piece in flight during that tile writes, reads stay inside their tile buffer and pieces
inside theirs (the spread-DMA investigation)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import attn3_dma_model as m  # noqa: E402


@pytest.mark.parametrize("db", [4, 8, 13, 16, 25])
@pytest.mark.parametrize("bufdma", [False, True])
def test_no_read_overlaps_an_inflight_piece(db, bufdma):
    r = m.check(db, bufdma)
    assert r["overlaps"] == 0
    assert r["read_span"][1] <= r["tile_bytes"] <= r["buffer_bytes"]
