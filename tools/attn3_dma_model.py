"""Host-side address model of kp_attn3's LDS traffic (kelpie_amd/csrc/kp_attn3.hpp).

For one key tile t of a work unit it lists, byte range by byte range:

* every LDS-DMA piece in flight during the tile: the next tile's copy (or, in the
  buffer-descriptor form, the last tile's re-read of its own rows) into buffer
  (t + 1) & 1, pieces 1024 p .. 1024 p + 1023, issued as a burst after the S phase or
  spread over the O blocks (KP_DMA_SPREAD) / S steps and O blocks (KP_DMA_SPREAD >= 2);
* every LDS read of the tile by every lane of every wave: the S phase's ds_read_b128
  (rows c and 16 + c, k-step s, piece p, lane group g) and its 16-deep tail ds_read_b64,
  and the O phase's ds_read_b64_tr_b16 (rows 4 g + c / 4 and 16 + 4 g + c / 4, columns
  8 (c % 4) + 32 m of piece p),

with the kernel's own formulas (split3_row_bytes, attn3_buf_pieces), and asserts that
no read touches a byte an in-flight piece writes, that every read stays inside its own
tile buffer, and that every piece stays inside its buffer.  The same holds across the
tile-closing barrier (reads of buffer t & 1 end before it; the next tile's pieces start
after it) and across work units (issue(0, 0) follows the previous unit's final
vmcnt(0) + barrier), so a clean result here means the ConvE spread-DMA failure and the
unstable KP_S_CHAIN hash are not address overlaps.

    python tools/attn3_dma_model.py   # all instantiated widths, both read forms
"""
from __future__ import annotations


def split3_row_bytes(dp: int) -> int:
    return 3 * 2 * dp + (0 if (dp // 16) % 2 else 32)


def buf_pieces(db: int, bufdma: bool) -> int:
    pieces = (32 * split3_row_bytes(16 * db) + 1023) // 1024
    return (pieces + 3) // 4 * 4 if bufdma else pieces


def tile_reads(db: int):
    """[(lo, hi)) byte ranges, relative to the tile buffer, of every lane's reads."""
    dp = 16 * db
    row_b = split3_row_bytes(dp)
    part_b = 2 * dp
    nk, tail = dp // 32, (dp % 32) // 16
    sub_b = 16 * row_b
    out = []
    for w in range(4):  # every wave reads the whole tile (its own 16 queries)
        for lane in range(64):
            g, c = lane >> 4, lane & 15
            rb = c * row_b + 16 * g
            for u in range(2):
                for p in range(3):
                    for s in range(nk):
                        a = rb + u * sub_b + p * part_b + 64 * s
                        out.append((a, a + 16))  # ds_read_b128
                    if tail:
                        a = rb - 8 * g + u * sub_b + p * part_b + 64 * nk
                        out.append((a, a + 8))  # ds_read_b64
            ob = (4 * g + (c >> 2)) * row_b + 8 * (c & 3)
            for m in range(db):
                for p in range(3):
                    for half in (0, 16 * row_b):
                        a = ob + half + p * part_b + 32 * m
                        out.append((a, a + 8))  # ds_read_b64_tr_b16: 8 bytes per lane
    return out


def check(db: int, bufdma: bool) -> dict:
    dp = 16 * db
    tile_b = 32 * split3_row_bytes(dp)
    pieces = buf_pieces(db, bufdma)
    buf_b = 1024 * pieces
    assert tile_b <= buf_b
    reads = tile_reads(db)
    lo = min(a for a, _ in reads)
    hi = max(b for _, b in reads)
    assert lo >= 0 and hi <= tile_b, (db, lo, hi, tile_b)
    n_bad = 0
    for t in range(4):  # both buffer parities, with and without a last-tile re-read
        cur = (t & 1) * buf_b
        nxt = ((t + 1) & 1) * buf_b
        dma = [(nxt + 1024 * p, nxt + 1024 * p + 1024) for p in range(pieces)]
        for a, b in dma:
            assert nxt <= a and b <= nxt + buf_b
        for a, b in reads:
            ra, rb_ = cur + a, cur + b
            for da, dbb in dma:
                if ra < dbb and da < rb_:
                    n_bad += 1
    assert n_bad == 0, f"DB={db}: {n_bad} reads overlap an in-flight DMA piece"
    return {"DB": db, "bufdma": bufdma, "tile_bytes": tile_b, "buffer_bytes": buf_b, "pieces": pieces,
            "reads_per_tile": len(reads), "read_span": [lo, hi], "overlaps": n_bad}


def main():
    import json
    for db in (4, 8, 13, 16, 25):
        for bufdma in (False, True):
            print(json.dumps(check(db, bufdma)))


if __name__ == "__main__":
    main()
