"""Host-side check of the arithmetic kp_attn3 (kelpie_amd/csrc/kp_attn3.hpp) relies on:
an fp32 value splits exactly into three bf16 pieces, and the six kept products of
a.b differ from the exact product by less than fp32's own rounding.  numpy emulation
of bf16 round-to-nearest-even (v_cvt_pk_bf16_f32); no GPU needed."""
import numpy as np


def bf16_rne(x):
    """float32 -> nearest bf16 (ties to even), returned as float32."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    x = np.asarray(x, dtype=np.float32)
    h = bf16_rne(x)
    r1 = (x - h).astype(np.float32)
    m = bf16_rne(r1)
    r2 = (r1 - m).astype(np.float32)
    return h, m, bf16_rne(r2)


def test_split_is_exact():
    rng = np.random.default_rng(0)
    for scale in (1e-3, 1.0, 37.0, 1e-20, 1e20):
        x = (rng.standard_normal(200_000) * scale).astype(np.float32)
        h, m, l = split3(x)
        # every piece has at most 8 significant bits: it is its own bf16 rounding
        for p in (h, m, l):
            assert np.array_equal(bf16_rne(p), p)
        back = h.astype(np.float64) + m.astype(np.float64) + l.astype(np.float64)
        assert np.array_equal(back, x.astype(np.float64))


def test_six_products_within_fp32_rounding():
    rng = np.random.default_rng(1)
    a = rng.standard_normal((2000, 400)).astype(np.float32)
    b = rng.standard_normal((2000, 400)).astype(np.float32)
    a0, a1, a2 = (p.astype(np.float64) for p in split3(a))
    b0, b1, b2 = (p.astype(np.float64) for p in split3(b))
    kept = a0 * b0 + a0 * b1 + a1 * b0 + a0 * b2 + a1 * b1 + a2 * b0
    exact = a.astype(np.float64) * b.astype(np.float64)
    mag = np.abs(exact)
    # dropped terms a1 b2 + a2 b1 + a2 b2 (|a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|): below
    # 2^-24 |a||b| elementwise, the size of one fp32 rounding of the product
    assert np.all(np.abs(kept - exact) <= 2.0 ** -24 * mag + 1e-300)
    # the dot products: kept-term error far under one fp32 ulp of the sum of |products|
    err = np.abs(kept.sum(1) - exact.sum(1))
    assert np.all(err <= 2.0 ** -24 * mag.sum(1))
