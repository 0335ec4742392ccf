// kp_rng.cpp -- host C++ of the reference's random-draw protocol (SURVEY.md
// Appendix B), behind the kp_rng_* / kp_mt19937_discard entry points of
// include/kelpie_hip.h.
//
// The reference draws from two MT19937 generators while it post-trains one
// candidate after another:
//   * torch's CPU generator (aten/src/ATen/core/MT19937RNGEngine.h): the
//     per-epoch torch.randint negatives of KelpiePairwiseRankingOptimizer
//     (src/link_prediction/optimization/pairwise_ranking_optimizer.py:171-172),
//     the ConvE dropout bernoulli_ masks, and draws that only advance the state;
//   * numpy's global RandomState (numpy/random/src/mt19937): the per-epoch
//     np.random.shuffle of the TransE rows (pairwise_ranking_optimizer.py:166).
// The engine ships the draws to the kernels, so they are generated here from the
// generators' own state blobs, bit for bit, and the states are advanced in place.
//
// Speed matters because the TransE protocol is on the critical path of every
// engine batch (about 84k generator outputs per slot at FB15k-237 sizes):
//   * the two generators are independent streams, so a slot's numpy shuffles run
//     on a persistent helper thread while the calling thread produces the torch
//     draws;
//   * numpy outputs are tempered block-wise after each regeneration (vectorised)
//     and the shuffle works on a local copy of the state (no aliasing with the
//     output array);
//   * of the ratio*R torch.randint draws per epoch only the first R are stepped
//     (SURVEY A-Q2): the others are skipped by twisting, without tempering.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

#include <immintrin.h>
#include <unistd.h>

#include "kelpie_hip.h"

namespace {

constexpr int kN = 624, kM = 397;

// One MT19937 twist.  Three spans: i < N - M reads the old s[i + M]; N - M <= i < N - 1
// reads s[i + M - N], already rewritten (227 words back, so a 16-word vector of the span
// only reads finished words); the last word wraps to s[0].  The AVX-512 form (one
// ternary-logic xor per 16 words) runs 1.7x the AVX2 auto-vectorised loop; it is picked
// at run time, so a host without AVX-512 keeps the portable form.  Same words either way.
#define KP_MT_ONE(i, src)                                                            \
  {                                                                                  \
    const uint32_t y = (s[i] & 0x80000000u) | (s[(i) + 1] & 0x7fffffffu);            \
    s[i] = s[src] ^ (y >> 1) ^ ((0u - (s[(i) + 1] & 1u)) & 0x9908b0dfu);             \
  }
#define KP_MT_V16(i, src)                                                                               \
  {                                                                                                     \
    const __m512i a = _mm512_loadu_si512(s + (i)), b = _mm512_loadu_si512(s + (i) + 1),                \
                  c = _mm512_loadu_si512(s + (src));                                                     \
    const __m512i y = _mm512_or_si512(_mm512_and_si512(a, U), _mm512_and_si512(b, L));                  \
    const __m512i mag = _mm512_maskz_mov_epi32(_mm512_test_epi32_mask(b, one), A);                      \
    _mm512_storeu_si512(s + (i), _mm512_ternarylogic_epi32(c, _mm512_srli_epi32(y, 1), mag, 0x96));   \
  }
__attribute__((target("avx512f"))) void mt_twist512(uint32_t* s) {
  const __m512i U = _mm512_set1_epi32((int)0x80000000u), L = _mm512_set1_epi32(0x7fffffff),
                one = _mm512_set1_epi32(1), A = _mm512_set1_epi32((int)0x9908b0dfu);
  int i = 0;
  for (; i + 16 <= kN - kM; i += 16) KP_MT_V16(i, i + kM);
  for (; i < kN - kM; ++i) KP_MT_ONE(i, i + kM);
  for (; i + 16 <= kN - 1; i += 16) KP_MT_V16(i, i + kM - kN);
  for (; i < kN - 1; ++i) KP_MT_ONE(i, i + kM - kN);
  const uint32_t y = (s[kN - 1] & 0x80000000u) | (s[0] & 0x7fffffffu);  // wraps to s[0]
  s[kN - 1] = s[kM - 1] ^ (y >> 1) ^ ((0u - (s[0] & 1u)) & 0x9908b0dfu);
}
#undef KP_MT_V16
#undef KP_MT_ONE

// KP_RNG_NO_AVX512=1 keeps the portable form (A/B runs)
const bool g_has_avx512 = __builtin_cpu_supports("avx512f") && !std::getenv("KP_RNG_NO_AVX512");

inline void mt_twist(uint32_t* s) {
  if (g_has_avx512) {
    mt_twist512(s);
    return;
  }
  // three dependency-free spans (distance >= N-M), vectorised by the compiler
  for (int i = 0; i < kN - kM; ++i) {
    const uint32_t y = (s[i] & 0x80000000u) | (s[i + 1] & 0x7fffffffu);
    s[i] = s[i + kM] ^ (y >> 1) ^ ((0u - (s[i + 1] & 1u)) & 0x9908b0dfu);
  }
  for (int i = kN - kM; i < kN - 1; ++i) {
    const uint32_t y = (s[i] & 0x80000000u) | (s[i + 1] & 0x7fffffffu);
    s[i] = s[i + kM - kN] ^ (y >> 1) ^ ((0u - (s[i + 1] & 1u)) & 0x9908b0dfu);
  }
  const uint32_t y = (s[kN - 1] & 0x80000000u) | (s[0] & 0x7fffffffu);
  s[kN - 1] = s[kM - 1] ^ (y >> 1) ^ ((0u - (s[0] & 1u)) & 0x9908b0dfu);
}

inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// ---------------------------------------------------------------------------------
// MT19937 jump-ahead.  The generator is linear over GF(2): with T the map that advances
// the 624-word window (x_k .. x_{k+623}) by one word and P(x) its characteristic
// polynomial (degree 19937, primitive), T^D = g(T) for g = x^D mod P.  P is found once
// by Berlekamp-Massey on the low bits of a stream of untempered words; g by square-and-
// multiply in GF(2)[x] mod P; g(T) W by Horner over g's 19937 coefficients, each step
// one window advance plus (for a set coefficient) a 624-word xor.  A jump costs the same
// for every distance, so skipping the draws of the slots other ranks post-train (the
// ConvE constructions and dropout masks: ~8 M words per slot) no longer costs the walk.
// The lowest 31 bits of the window's first word do not feed the recurrence, so Horner
// leaves them unreliable: a jump by D is g = x^(D-1) followed by one plain advance.
// ---------------------------------------------------------------------------------
constexpr int kDeg = 19937;
constexpr int kPW = kDeg / 64 + 1;  // 312 words: coefficients x^0 .. x^19967

struct MtPoly {
  uint64_t w[kPW];
};

// one window advance on a circular 624-word buffer whose element 0 is at head h
inline void mt_step(uint32_t* b, int& h) {
  const uint32_t a = b[h], c = b[h + 1 < kN ? h + 1 : h + 1 - kN], m = b[(h + kM) % kN];
  const uint32_t y = (a & 0x80000000u) | (c & 0x7fffffffu);
  b[h] = m ^ (y >> 1) ^ ((0u - (c & 1u)) & 0x9908b0dfu);
  h = h + 1 < kN ? h + 1 : 0;
}

// P(x) by Berlekamp-Massey over the bit 0 of 2 * 19937 words of a seeded generator
const MtPoly& mt_charpoly() {
  static MtPoly P;
  static std::once_flag once;
  std::call_once(once, [] {
    constexpr int NB = 2 * kDeg;
    constexpr int SW = NB / 64 + 2;
    std::vector<uint64_t> seq(SW, 0), rev(SW + kPW + 2, 0);
    uint32_t st[kN];
    st[0] = 5489u;
    for (int i = 1; i < kN; ++i) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
    int h = 0;
    for (int i = 0; i < NB; ++i) {
      mt_step(st, h);
      const uint32_t x = st[(h + kN - 1) % kN];  // the word just made
      if (x & 1u) seq[i >> 6] |= 1ull << (i & 63);
    }
    // rev bit j = seq bit NB - 1 - j, so the window s[n-1], s[n-2], ... is rev from NB - n
    for (int i = 0; i < NB; ++i)
      if (seq[i >> 6] >> (i & 63) & 1) {
        const int j = NB - 1 - i;
        rev[j >> 6] |= 1ull << (j & 63);
      }
    auto rev_word = [&](int bit) -> uint64_t {  // rev bits [bit, bit + 64)
      const int q = bit >> 6, r = bit & 63;
      return r ? (rev[q] >> r) | (rev[q + 1] << (64 - r)) : rev[q];
    };
    std::vector<uint64_t> C(kPW + 2, 0), B(kPW + 2, 0), T(kPW + 2, 0);
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int n = 0; n < NB; ++n) {
      // d = s[n] ^ sum_{i=1..L} c_i s[n - i]; c_i s[n - i] = C bit i & rev bit (NB - 1 - n + i)
      uint64_t acc = 0;
      const int off = NB - 1 - n;
      const int words = (L >> 6) + 1;
      for (int k = 0; k < words; ++k) acc ^= C[k] & rev_word(off + 64 * k);
      int d = (int)(__builtin_popcountll(acc) & 1);  // includes c_0 s[n] (c_0 = 1)
      if (!d) {
        ++m;
        continue;
      }
      auto xor_shift = [&](std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, int sh) {
        const int q = sh >> 6, r = sh & 63;
        for (int k = kPW + 1; k >= q; --k) {
          uint64_t v = src[k - q] << r;
          if (r && k - q - 1 >= 0) v |= src[k - q - 1] >> (64 - r);
          dst[k] ^= v;
        }
      };
      if (2 * L <= n) {
        T = C;
        xor_shift(C, B, m);
        L = n + 1 - L;
        B = T;
        m = 1;
      } else {
        xor_shift(C, B, m);
        ++m;
      }
    }
    if (L != kDeg) throw std::runtime_error("mt19937 jump: characteristic polynomial of unexpected degree");
    // BM's C is the connection polynomial (c_0 = 1 ... c_L); the characteristic
    // polynomial is its reciprocal x^L C(1/x)
    for (int i = 0; i <= kDeg; ++i)
      if (C[i >> 6] >> (i & 63) & 1) {
        const int j = kDeg - i;
        P.w[j >> 6] |= 1ull << (j & 63);
      }
  });
  return P;
}

// g = x^D mod P
void mt_jump_poly(uint64_t D, MtPoly& g) {
  const MtPoly& P = mt_charpoly();
  // P shifted left by 0..63 bits (each XOR of the reduction word-aligned)
  static std::vector<uint64_t> Psh;
  static std::once_flag once;
  std::call_once(once, [&] {
    Psh.assign(64 * (kPW + 1), 0);
    for (int r = 0; r < 64; ++r)
      for (int k = 0; k <= kPW; ++k) {
        uint64_t v = k < kPW ? P.w[k] << r : 0;
        if (r && k > 0) v |= P.w[k - 1] >> (64 - r);
        Psh[64 * 0 + r * (kPW + 1) + k] = v;
      }
  });
  std::vector<uint64_t> sq(2 * kPW + 2);
  std::memset(g.w, 0, sizeof(g.w));
  g.w[0] = 1;
  int top = 63;
  while (top > 0 && !((D >> top) & 1)) --top;
  auto reduce = [&](uint64_t* a, int hi_bit) {  // a: bits up to hi_bit, reduced below 19937
    for (int i = hi_bit; i >= kDeg; --i) {
      if (!(a[i >> 6] >> (i & 63) & 1)) continue;
      const int sh = i - kDeg, q = sh >> 6, r = sh & 63;
      const uint64_t* ps = &Psh[r * (kPW + 1)];
      for (int k = 0; k <= kPW && q + k < 2 * kPW + 2; ++k) a[q + k] ^= ps[k];
    }
  };
  for (int b = top; b >= 0; --b) {
    // square: coefficient i -> 2i
    std::fill(sq.begin(), sq.end(), 0);
    for (int k = 0; k < kPW; ++k) {
      uint64_t v = g.w[k];
      if (!v) continue;
      uint64_t lo = 0, hi = 0;
      for (int j = 0; j < 32; ++j) {
        lo |= ((v >> j) & 1ull) << (2 * j);
        hi |= ((v >> (j + 32)) & 1ull) << (2 * j);
      }
      sq[2 * k] = lo;
      sq[2 * k + 1] = hi;
    }
    reduce(sq.data(), 2 * (kDeg - 1));
    std::memcpy(g.w, sq.data(), sizeof(g.w));
    if ((D >> b) & 1) {
      // times x
      uint64_t carry = 0;
      for (int k = 0; k < kPW; ++k) {
        const uint64_t v = g.w[k];
        g.w[k] = (v << 1) | carry;
        carry = v >> 63;
      }
      if (g.w[kDeg >> 6] >> (kDeg & 63) & 1)
        for (int k = 0; k < kPW; ++k) g.w[k] ^= P.w[k];
    }
  }
}

// the window s (x_k .. x_{k+623}, element 0 first) -> (x_{k+D} .. x_{k+D+623}), D >= 1
void mt_jump_window(uint32_t* s, uint64_t D) {
  MtPoly g;
  mt_jump_poly(D - 1, g);
  uint32_t acc[kN];
  std::memset(acc, 0, sizeof(acc));
  int h = 0;
  int deg = kDeg - 1;
  while (deg > 0 && !(g.w[deg >> 6] >> (deg & 63) & 1)) --deg;
  for (int i = deg; i >= 0; --i) {
    mt_step(acc, h);
    if (g.w[i >> 6] >> (i & 63) & 1) {
      // acc element j (at (h + j) % N) ^= s[j]
      const int n1 = kN - h;
      for (int j = 0; j < n1; ++j) acc[h + j] ^= s[j];
      for (int j = n1; j < kN; ++j) acc[j - n1] ^= s[j];
    }
  }
  mt_step(acc, h);  // one plain advance: the first word's low bits are valid again
  for (int j = 0; j < kN; ++j) s[j] = acc[(h + j) % kN];
}

// skips at least this many outputs go by jump-ahead (KP_MT_JUMP_MIN; 0 never)
uint64_t mt_jump_min() {
  static const uint64_t v = [] {
    const char* e = std::getenv("KP_MT_JUMP_MIN");
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)60000000;
  }();
  return v;
}

// ATen's mt19937 over the CPU-generator state blob of torch.get_rng_state():
//   { u64 seed; i32 left; i32 seeded; u64 next; u64 state[624]; ... }.
// operator(): if (--left == 0) twist (left = 624, next = 0); return temper(state[next++]).
struct TorchMt {
  int32_t left;
  uint64_t next;
  uint32_t s[kN];
  void load(const uint8_t* st) {
    std::memcpy(&left, st + 8, 4);
    std::memcpy(&next, st + 16, 8);
    for (int i = 0; i < kN; ++i) {
      uint64_t v;
      std::memcpy(&v, st + 24 + 8 * i, 8);
      s[i] = (uint32_t)v;
    }
  }
  void store(uint8_t* st) const {
    std::memcpy(st + 8, &left, 4);
    std::memcpy(st + 16, &next, 8);
    for (int i = 0; i < kN; ++i) {
      const uint64_t v = s[i];
      std::memcpy(st + 24 + 8 * i, &v, 8);
    }
  }
  // advance by n outputs (operator() semantics, nothing tempered)
  void skip(uint64_t n) {
    const uint64_t jmin = mt_jump_min();
    if (jmin && n >= jmin && n > (uint64_t)(left - 1) + kN) {
      // the rest of this block, then t whole twists by jump-ahead; c words of the last
      // block consumed (the twisting call takes its first word: left = kN, next = 1)
      const uint64_t rest = n - (uint64_t)(left - 1);
      const uint64_t t = (rest + kN - 1) / kN;
      const uint64_t c = rest - (uint64_t)kN * (t - 1);
      mt_jump_window(s, (uint64_t)kN * t);
      left = (int32_t)(kN - c + 1);
      next = c;
      return;
    }
    while (n > 0) {
      const uint64_t k = std::min<uint64_t>(n, (uint64_t)(left - 1));
      left -= (int32_t)k;
      next += k;
      n -= k;
      if (n > 0) {
        mt_twist(s);
        left = kN;
        next = 1;
        n -= 1;
      }
    }
  }
  // the next n outputs, in order, tempered as they are taken
  void fill(uint32_t* out, size_t n) {
    size_t k = 0;
    while (k < n) {
      if (left <= 1) {  // the next operator() call twists
        mt_twist(s);
        left = kN + 1;
        next = 0;
      }
      const size_t m = std::min<size_t>(n - k, (size_t)(left - 1));
      const uint32_t* src = s + next;
      for (size_t j = 0; j < m; ++j) out[k + j] = mt_temper(src[j]);
      k += m;
      next += m;
      left -= (int32_t)m;
    }
  }
};

// ---------------------------------------------------------------------------------
// torch.Tensor.normal_ on the CPU generator, float32, contiguous, n >= 16
// (aten/src/ATen/native/cpu/DistributionTemplates.h normal_fill / normal_fill_AVX2):
// n uniforms u = (random() & 0xFFFFFF) * 2^-24, Box-Muller over each block of 16
// (u1 = 1 - u[j], u2 = u[j + 8]), and when 16 does not divide n the last 16 values
// are redrawn (16 more uniforms) and transformed again.
//  * cap 1 -- torch built for AVX2 / AVX512 (torch.backends.cpu.get_cpu_capability()):
//    normal_fill_16_AVX2 with avx_mathfun's log256_ps / sincos256_ps (Cephes
//    polynomials), every multiply feeding an add contracted to an FMA as the build
//    does; pinned value for value against torch (tests/test_rng_protocol.py);
//  * cap 0 -- the scalar kernel: logf / cosf / sinf / sqrtf of libm, no contraction.
// This file is compiled with -ffp-contract=off: every fused operation below is an
// explicit fmadd.
// ---------------------------------------------------------------------------------
// v_log / v_sincos below are an altered restatement of log256_ps / sincos256_ps from
// avx_mathfun.h (the AVX port by Giovanni Garberoglio, 2012, of sse_mathfun.h by Julien
// Pommier, 2007; Cephes polynomials), which torch's CPU normal_ uses.  Their notice
// (the zlib license):
//   This software is provided 'as-is', without any express or implied warranty.  In no
//   event will the authors be held liable for any damages arising from the use of this
//   software.  Permission is granted to anyone to use this software for any purpose,
//   including commercial applications, and to alter it and redistribute it freely,
//   subject to the following restrictions:
//   1. The origin of this software must not be misrepresented; you must not claim that
//      you wrote the original software.  If you use this software in a product, an
//      acknowledgment in the product documentation would be appreciated but is not
//      required.
//   2. Altered source versions must be plainly marked as such, and must not be
//      misrepresented as being the original software.
//   3. This notice may not be removed or altered from any source distribution.
// Altered here: every multiply that feeds an add is an explicit fmadd, as torch's build
// contracts them.
// avx_mathfun's log256_ps and sincos256_ps as torch's AVX2 build runs them: each
// multiply that feeds an add fused (an explicit fmadd; the rest stay separate, and this
// file is built with -ffp-contract=off so nothing else is fused)
inline __m256 v_log(__m256 x) {
  const __m256 one = _mm256_set1_ps(1.0f);
  const __m256 invalid = _mm256_cmp_ps(x, _mm256_setzero_ps(), _CMP_LE_OS);
  x = _mm256_max_ps(x, _mm256_castsi256_ps(_mm256_set1_epi32(0x00800000)));
  __m256i imm0 = _mm256_srli_epi32(_mm256_castps_si256(x), 23);
  x = _mm256_and_ps(x, _mm256_castsi256_ps(_mm256_set1_epi32(~0x7f800000)));
  x = _mm256_or_ps(x, _mm256_set1_ps(0.5f));
  imm0 = _mm256_sub_epi32(imm0, _mm256_set1_epi32(0x7f));
  __m256 e = _mm256_add_ps(_mm256_cvtepi32_ps(imm0), one);
  const __m256 mask = _mm256_cmp_ps(x, _mm256_set1_ps(0.707106781186547524f), _CMP_LT_OS);
  const __m256 tmp = _mm256_and_ps(x, mask);
  x = _mm256_sub_ps(x, one);
  e = _mm256_sub_ps(e, _mm256_and_ps(one, mask));
  x = _mm256_add_ps(x, tmp);
  const __m256 z = _mm256_mul_ps(x, x);
  __m256 y = _mm256_set1_ps(7.0376836292E-2f);
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(-1.1514610310E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(1.1676998740E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(-1.2420140846E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(1.4249322787E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(-1.6668057665E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(2.0000714765E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(-2.4999993993E-1f));
  y = _mm256_fmadd_ps(y, x, _mm256_set1_ps(3.3333331174E-1f));
  y = _mm256_mul_ps(y, x);
  y = _mm256_fmadd_ps(y, z, _mm256_mul_ps(e, _mm256_set1_ps(-2.12194440e-4f)));
  y = _mm256_fmadd_ps(z, _mm256_set1_ps(-0.5f), y);
  x = _mm256_add_ps(x, y);
  x = _mm256_fmadd_ps(e, _mm256_set1_ps(0.693359375f), x);
  return _mm256_or_ps(x, invalid);
}
inline void v_sincos(__m256 x, __m256& s, __m256& c) {
  __m256 sign_sin = _mm256_and_ps(x, _mm256_castsi256_ps(_mm256_set1_epi32((int)0x80000000)));
  x = _mm256_and_ps(x, _mm256_castsi256_ps(_mm256_set1_epi32(0x7fffffff)));
  __m256 y = _mm256_mul_ps(x, _mm256_set1_ps(1.27323954473516f));
  __m256i imm2 = _mm256_cvttps_epi32(y);
  imm2 = _mm256_add_epi32(imm2, _mm256_set1_epi32(1));
  imm2 = _mm256_and_si256(imm2, _mm256_set1_epi32(~1));
  y = _mm256_cvtepi32_ps(imm2);
  __m256i imm4 = imm2;
  const __m256 swap_sign_sin = _mm256_castsi256_ps(_mm256_slli_epi32(_mm256_and_si256(imm2, _mm256_set1_epi32(4)), 29));
  const __m256 poly = _mm256_castsi256_ps(
      _mm256_cmpeq_epi32(_mm256_and_si256(imm2, _mm256_set1_epi32(2)), _mm256_setzero_si256()));
  x = _mm256_fmadd_ps(y, _mm256_set1_ps(-0.78515625f), x);
  x = _mm256_fmadd_ps(y, _mm256_set1_ps(-2.4187564849853515625e-4f), x);
  x = _mm256_fmadd_ps(y, _mm256_set1_ps(-3.77489497744594108e-8f), x);
  imm4 = _mm256_sub_epi32(imm4, _mm256_set1_epi32(2));
  imm4 = _mm256_andnot_si256(imm4, _mm256_set1_epi32(4));
  const __m256 sign_cos = _mm256_castsi256_ps(_mm256_slli_epi32(imm4, 29));
  sign_sin = _mm256_xor_ps(sign_sin, swap_sign_sin);
  const __m256 z = _mm256_mul_ps(x, x);
  __m256 yc = _mm256_set1_ps(2.443315711809948E-005f);
  yc = _mm256_fmadd_ps(yc, z, _mm256_set1_ps(-1.388731625493765E-003f));
  yc = _mm256_fmadd_ps(yc, z, _mm256_set1_ps(4.166664568298827E-002f));
  yc = _mm256_mul_ps(yc, z);
  yc = _mm256_fmadd_ps(yc, z, _mm256_sub_ps(_mm256_setzero_ps(), _mm256_mul_ps(z, _mm256_set1_ps(0.5f))));
  yc = _mm256_add_ps(yc, _mm256_set1_ps(1.0f));
  __m256 ys = _mm256_set1_ps(-1.9515295891E-4f);
  ys = _mm256_fmadd_ps(ys, z, _mm256_set1_ps(8.3321608736E-3f));
  ys = _mm256_fmadd_ps(ys, z, _mm256_set1_ps(-1.6666654611E-1f));
  ys = _mm256_mul_ps(ys, z);
  ys = _mm256_fmadd_ps(ys, x, x);
  const __m256 ysin2 = _mm256_and_ps(poly, ys), ysin1 = _mm256_andnot_ps(poly, yc);
  ys = _mm256_sub_ps(ys, ysin2);
  yc = _mm256_sub_ps(yc, ysin1);
  s = _mm256_xor_ps(_mm256_add_ps(ysin1, ysin2), sign_sin);
  c = _mm256_xor_ps(_mm256_add_ps(yc, ys), sign_cos);
}

inline void normal_fill16(float* d, float mean, float std_, int cap) {
  if (cap) {
    const __m256 u1 = _mm256_sub_ps(_mm256_set1_ps(1.0f), _mm256_loadu_ps(d));
    const __m256 u2 = _mm256_loadu_ps(d + 8);
    const __m256 radius = _mm256_sqrt_ps(_mm256_mul_ps(_mm256_set1_ps(-2.0f), v_log(u1)));
    const __m256 theta = _mm256_mul_ps(_mm256_set1_ps((float)(2.0f * 3.14159265358979323846)), u2);
    __m256 sn, cs;
    v_sincos(theta, sn, cs);
    _mm256_storeu_ps(d, _mm256_fmadd_ps(_mm256_mul_ps(radius, cs), _mm256_set1_ps(std_), _mm256_set1_ps(mean)));
    _mm256_storeu_ps(d + 8, _mm256_fmadd_ps(_mm256_mul_ps(radius, sn), _mm256_set1_ps(std_), _mm256_set1_ps(mean)));
    return;
  }
  for (int j = 0; j < 8; ++j) {
    const float u1 = 1.0f - d[j], u2 = d[j + 8];
    const float radius = std::sqrt(-2.0f * std::log(u1));
    const float theta = (float)(2.0f * 3.14159265358979323846 * (double)u2);
    d[j] = radius * std::cos(theta) * std_ + mean;
    d[j + 8] = radius * std::sin(theta) * std_ + mean;
  }
}

// torch.empty(n).normal_(mean, std) for n >= 16 (normal_fill): advances mt like torch
template <class Mt>
void normal_draw(Mt& mt, int64_t n, float mean, float std_, int cap, float* out) {
  std::vector<uint32_t> r((size_t)n);
  mt.fill(r.data(), (size_t)n);
  for (int64_t i = 0; i < n; ++i) out[i] = (float)(r[(size_t)i] & 0xFFFFFFu) * (1.0f / 16777216.0f);
  for (int64_t i = 0; i + 16 <= n; i += 16) normal_fill16(out + i, mean, std_, cap);
  if (n % 16) {
    uint32_t t[16];
    mt.fill(t, 16);
    float* d = out + n - 16;
    for (int i = 0; i < 16; ++i) d[i] = (float)(t[i] & 0xFFFFFFu) * (1.0f / 16777216.0f);
    normal_fill16(d, mean, std_, cap);
  }
}

// numpy's legacy MT19937 (numpy/random/src/mt19937/mt19937.h: {uint32 key[624]; int pos}):
// regenerate when pos reaches 624.  Works on a local copy; the current block is kept
// tempered (tb) so a draw is one load.
struct NumpyMt {
  uint32_t key[kN];
  uint32_t tb[kN];
  int pos;
  void temper_all() {
    for (int i = 0; i < kN; ++i) tb[i] = mt_temper(key[i]);
  }
  void load(const uint32_t* k, const int32_t* p) {
    std::memcpy(key, k, sizeof(key));
    pos = *p;
    temper_all();
  }
  void store(uint32_t* k, int32_t* p) const {
    std::memcpy(k, key, sizeof(key));
    *p = pos;
  }
  inline uint32_t next32() {
    if (pos >= kN) {
      mt_twist(key);
      temper_all();
      pos = 0;
    }
    return tb[pos++];
  }
  // numpy/random/src/distributions: random_interval(max), max < 2^32 (masked rejection)
  inline uint32_t interval(uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > max) {
    }
    return v;
  }
};

// a % d for 32-bit a, d >= 1 (Lemire, Kaser & Kurz 2019), fm = 2^64 / d rounded up
inline uint32_t fastmod_u32(uint32_t a, uint64_t fm, uint32_t d) {
  const uint64_t lowbits = fm * a;
  return (uint32_t)(((__uint128_t)lowbits * d) >> 64);
}

// One persistent helper thread that runs one task at a time for a caller that waits
// for it.  It spins briefly between tasks (a scheduling pass calls every few tens of
// microseconds) and then sleeps on a condition variable.  Re-created after a fork.
class Helper {
 public:
  static Helper& get() {
    static Helper* h = new Helper();  // never destroyed: no join at process exit
    return *h;
  }
  // run a() here and b() on the helper (inline if the helper is busy or unusable)
  void run2(const std::function<void()>& a, const std::function<void()>& b) {
    std::unique_lock<std::mutex> owner(own_, std::try_to_lock);
    if (!owner.owns_lock() || !ensure()) {
      b();
      a();
      return;
    }
    task_ = &b;
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_.store(1, std::memory_order_release);
    }
    cv_.notify_one();
    bool a_failed = false;
    try {
      a();
    } catch (...) {
      a_failed = true;  // b() still references the caller's frame: wait for it first
    }
    // if the helper has not claimed the task yet (descheduled on a busy host), take it back
    int posted = 1;
    const bool claimed = !state_.compare_exchange_strong(posted, 0, std::memory_order_acq_rel);
    if (!claimed) {
      try {
        b();
      } catch (...) {
        a_failed = true;
      }
    } else {
      while (state_.load(std::memory_order_acquire) != 2) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
      state_.store(0, std::memory_order_relaxed);
    }
    if (a_failed || (claimed && failed_)) throw std::bad_alloc();
  }

 private:
  bool ensure() {
    const pid_t me = getpid();
    if (pid_ == me) return true;
    try {
      state_.store(0);
      std::thread([this] { loop(); }).detach();
      pid_ = me;
      return true;
    } catch (...) {
      return false;
    }
  }
  // states: 0 idle, 1 posted, 3 claimed by the helper, 2 done
  void loop() {
    for (;;) {
      int spins = 0;
      for (;;) {
        int posted = 1;
        if (state_.compare_exchange_weak(posted, 3, std::memory_order_acq_rel)) break;
        if (++spins < 200000) {
#if defined(__x86_64__)
          __builtin_ia32_pause();
#endif
          continue;
        }
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return state_.load(std::memory_order_acquire) == 1; });
      }
      try {
        (*task_)();
        failed_ = false;
      } catch (...) {
        failed_ = true;
      }
      state_.store(2, std::memory_order_release);
    }
  }
  std::mutex own_, mu_;
  std::condition_variable cv_;
  std::atomic<int> state_{0};
  const std::function<void()>* task_ = nullptr;
  pid_t pid_ = 0;
  bool failed_ = false;
};

// ATen's bernoulli_(p) on a float tensor draws u = random64() * 2^-53 (hi word first)
// per element and keeps it when u < p.  u is exact, so u < p <=> m < ceil(p * 2^53)
// for the 53-bit integer m: the test runs on integers, block-wise over bulk draws.
void bernoulli_words(TorchMt& mt, uint64_t n, double p, uint32_t* out, std::vector<uint32_t>& buf) {
  const uint64_t mask53 = (1ULL << 53) - 1;
  const uint64_t thr = (uint64_t)std::ceil(std::ldexp(std::min(std::max(p, 0.0), 1.0), 53));
  constexpr uint64_t CH = 1u << 14;  // elements per chunk (multiple of 32)
  buf.resize(2 * CH);
  for (uint64_t i0 = 0; i0 < n; i0 += CH) {
    const uint64_t m = std::min<uint64_t>(CH, n - i0);
    mt.fill(buf.data(), 2 * m);
    const uint32_t* b = buf.data();
    uint32_t* o = out + (i0 >> 5);
    const uint64_t nw = (m + 31) / 32;
    for (uint64_t w = 0; w < nw; ++w) {
      uint32_t acc = 0;
      const uint64_t lim = std::min<uint64_t>(32, m - 32 * w);
      for (uint64_t j = 0; j < lim; ++j) {
        const uint64_t e = 32 * w + j;
        const uint64_t v = (((uint64_t)b[2 * e] << 32) | b[2 * e + 1]) & mask53;
        acc |= (uint32_t)(v < thr) << j;
      }
      o[w] = acc;
    }
  }
}

// Deferred TransE draws (kp_rng_transe_enqueue / kp_rng_wait).  The engine schedules
// a batch's slots one after another on the Python thread; with the synchronous entry
// point each slot waited for its own shuffles and randints.  Here the caller only
// snapshots the torch generator and advances it past the slot's randints (twisting,
// nothing tempered), and the draws are produced behind its back:
//   * one sequential worker runs the numpy shuffles of every queued slot in queue
//     order (numpy's consumption is data-dependent: rejection sampling), reading and
//     writing the live numpy state only between the caller's enqueue and its wait;
//   * a small pool fills each slot's randints from its own snapshot, in any order.
// Both write disjoint parts of the slot's output ([row order | entity | head_or_tail]
// per epoch).  kp_rng_wait() returns once every queued slot is complete.

// The shuffles of one slot come in two parts:
//  * te_draws (sequential, on the live numpy state): every epoch's random_interval(i)
//    draws, i = R - 1 .. 1 (masked rejection, numpy's consumption is data-dependent), the
//    draw for i left at out[e*3R + i] (its row-order slot, used as scratch);
//  * te_perms (any thread, after te_draws): the permutation chain -- epoch e shuffles the
//    order left by epoch e - 1 with those draws -- written over the same slots.
// Only te_draws is on the batch's sequential chain.
// ui - (v <= ui) as ui - 1 + borrow(ui - v): a two-instruction carried chain (cmp, adc)
inline uint32_t accept_step(uint32_t ui, uint32_t v) {
#if defined(__x86_64__)
  asm("cmpl %1, %0\n\tadcl $-1, %0" : "+r"(ui) : "r"(v) : "cc");
  return ui;
#else
  return ui - (uint32_t)(v <= ui);
#endif
}

void te_draws(uint32_t* np_key, int32_t* np_pos, int32_t R, int32_t epochs, int32_t* jv0, size_t stride, NumpyMt& np) {
  // validated here, on the thread that owns the live numpy state while draws are queued
  // (the enqueueing thread must not read it: the sequential worker may be writing it)
  if (*np_pos < 0 || *np_pos > kN) throw std::invalid_argument("numpy MT19937 pos out of range");
  np.load(np_key, np_pos);
  for (int e = 0; e < epochs; ++e) {
    int32_t* jv = jv0 ? jv0 + (size_t)e * stride : nullptr;  // null: advance only
    // for i in reversed(range(1, R)): j = random_interval(i).  The mask of i is fixed while
    // i stays above half of it, so the inner loop's carried chain is compare -> subtract; a
    // rejected draw leaves i unchanged and its jv[i] is overwritten by the next one
    uint32_t ui = (uint32_t)(R - 1);
    while (ui >= 1) {
      if (np.pos >= kN) {
        mt_twist(np.key);
        np.temper_all();
        np.pos = 0;
      }
      const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(ui), lo = mask >> 1;
      const uint32_t* tb = np.tb + np.pos;
      const int n = kN - np.pos;  // draws left in this block
      int k = 0;
      if (jv) {
        for (; k < n && ui > lo; ++k) {
          const uint32_t v = tb[k] & mask;
          jv[ui] = (int32_t)v;
          ui = accept_step(ui, v);
        }
      } else {
        for (; k < n && ui > lo; ++k) ui = accept_step(ui, tb[k] & mask);
      }
      np.pos += k;
    }
  }
  np.store(np_key, np_pos);
}

void te_perms(int32_t R, int32_t epochs, const int32_t* jv0, size_t stride, int32_t* out, std::vector<int32_t>& idx) {
  idx.resize((size_t)std::max(R, 1));
  int32_t* perm = idx.data();
  for (int i = 0; i < R; ++i) perm[i] = i;
  for (int e = 0; e < epochs; ++e) {
    const int32_t* jv = jv0 + (size_t)e * stride;
    for (int t = R - 1; t >= 1; --t) std::swap(perm[t], perm[jv[t]]);
    std::memcpy(out + (size_t)e * 3 * R, perm, sizeof(int32_t) * R);
  }
}

// both parts on one thread: the draws into a local scratch (cache-resident), then the chain
void te_shuffles(uint32_t* np_key, int32_t* np_pos, int32_t R, int32_t epochs, int32_t* out, NumpyMt& np,
                 std::vector<int32_t>& idx, std::vector<int32_t>& jv) {
  if (!out) {
    te_draws(np_key, np_pos, R, epochs, nullptr, 0, np);
    return;
  }
  jv.resize((size_t)std::max(R, 1) * std::max(epochs, 1));
  te_draws(np_key, np_pos, R, epochs, jv.data(), (size_t)R, np);
  te_perms(R, epochs, jv.data(), (size_t)R, out, idx);
}

// KP_RNG_PERMS_INLINE=1: the permutation chain stays on the sequential worker (A/B of
// where it runs; default: the pool)
const bool g_perms_inline = std::getenv("KP_RNG_PERMS_INLINE") && std::atoi(std::getenv("KP_RNG_PERMS_INLINE")) == 1;

// torch.randint(high=N) = random() % N and randint(high=2), ratio*R each per epoch;
// only the first R of each are stepped
void te_randints(TorchMt& mt, int32_t R, int32_t epochs, int32_t ratio, uint32_t nent, int32_t* out,
                 std::vector<uint32_t>& draw) {
  const uint64_t n = (uint64_t)ratio * (uint64_t)R;
  const uint64_t fm = UINT64_C(0xFFFFFFFFFFFFFFFF) / nent + 1;
  draw.resize(std::max(R, 1));
  for (int e = 0; e < epochs; ++e) {
    int32_t* o = out + (size_t)e * 3 * R;
    mt.fill(draw.data(), R);
    for (int k = 0; k < R; ++k) o[R + k] = (int32_t)fastmod_u32(draw[k], fm, nent);
    mt.skip(n - (uint64_t)R);
    mt.fill(draw.data(), R);
    for (int k = 0; k < R; ++k) o[2 * R + k] = (int32_t)(draw[k] & 1u);
    mt.skip(n - (uint64_t)R);
  }
}

// A queued task runs with the worker's scratch (numpy copy, index and draw buffers).
struct Scratch {
  NumpyMt np;
  std::vector<int32_t> idx, jv;
  std::vector<uint32_t> draw;
};
using Task = std::function<void(Scratch&)>;

// Batch tags of queued work (kp_rng_batch_close / kp_rng_batch_wait): every task carries
// the batch that was open when it was queued -- or, queued from inside a task (the walk
// queues shuffles, a shuffle queues its permutation chain), its parent's -- so a batch's
// draws can be waited for while later batches' tasks are already queued behind them.
std::atomic<int64_t> g_open_batch{1};
thread_local int64_t t_task_batch = 0;  // the batch of the task this thread is running
inline int64_t submit_tag() { return t_task_batch ? t_task_batch : g_open_batch.load(std::memory_order_acquire); }
// per-batch pending counts of one queue (guarded by the queue's mutex)
struct BatchPending {
  std::map<int64_t, int64_t> n;
  void add(int64_t tag) { ++n[tag]; }
  void done(int64_t tag) {
    auto it = n.find(tag);
    if (it != n.end() && --it->second == 0) n.erase(it);
  }
  bool clear_upto(int64_t id) const { return n.empty() || n.begin()->first > id; }
};

// KP_RNG_STATS=1: per batch (at each kp_rng_wait), the busy time of the walker, the
// sequential worker and the pool, and when the last task ended relative to the wait
// call, on stderr (a diagnostic of where a batch's draw time goes; off by default)
struct RngStats {
  const bool on = std::getenv("KP_RNG_STATS") != nullptr;
  std::atomic<int64_t> walk_ns{0}, seq_ns{0}, pool_ns{0}, seq_tasks{0}, pool_tasks{0}, last_end_ns{0},
      first_start_ns{0};
  static int64_t now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  void span(std::atomic<int64_t>& acc, int64_t t0) {
    const int64_t t1 = now();
    acc += t1 - t0;
    int64_t prev = last_end_ns.load();
    while (prev < t1 && !last_end_ns.compare_exchange_weak(prev, t1)) {
    }
    int64_t z = 0;
    first_start_ns.compare_exchange_strong(z, t0);
  }
  void report(int64_t t_wait) {
    std::fprintf(stderr,
                 "[kp_rng] walk %.2f ms | seq %.2f ms (%lld tasks) | pool %.2f ms (%lld tasks) | first task %.2f ms "
                 "before the wait, last ended %.2f ms after it\n",
                 walk_ns / 1e6, seq_ns / 1e6, (long long)seq_tasks.load(), pool_ns / 1e6, (long long)pool_tasks.load(),
                 (t_wait - first_start_ns) / 1e6, (last_end_ns - t_wait) / 1e6);
    walk_ns = seq_ns = pool_ns = seq_tasks = pool_tasks = last_end_ns = first_start_ns = 0;
  }
};
RngStats& rng_stats() {
  static RngStats* s = new RngStats();
  return *s;
}

class DrawQueue {
 public:
  static DrawQueue& get() {
    static DrawQueue* q = new DrawQueue();  // never destroyed: workers are detached
    return *q;
  }
  // seq: runs on the one sequential worker in queue order (may be empty); fill: on the
  // pool.  false: the workers could not be started (the caller then runs both inline
  // after a wait()).
  bool enqueue(Task seq, Task fill) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!ensure_locked()) return false;
    // one wake-up per queued task, on the queue's own condition variable (a notify_all on a
    // shared one woke every pool thread for each of a batch's ~600 tasks)
    const int64_t tag = submit_tag();
    if (seq) {
      seq_.push_back(Item{std::move(seq), tag});
      ++pending_;
      bp_.add(tag);
      cv_seq_.notify_one();
    }
    if (fill) {
      fills_.push_back(Item{std::move(fill), tag});
      ++pending_;
      bp_.add(tag);
      cv_fill_.notify_one();
    }
    return true;
  }
  int wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [this] { return pending_ == 0; });
    const int rc = fail_rc_;
    fail_rc_ = KP_OK;
    return rc;
  }
  // every task of the batches <= id done (later batches' tasks may still run); the
  // first failure of any task so far (not cleared: wait() reports and clears it)
  int wait_batch(int64_t id) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return bp_.clear_upto(id); });
    return fail_rc_;
  }

 private:
  bool ensure_locked() {
    const pid_t me = getpid();
    if (pid_ == me) return true;
    // first use, or a forked child (the parent's workers do not exist here)
    seq_.clear();
    fills_.clear();
    bp_ = BatchPending();
    pending_ = 0;
    int nfill = 4;
    if (const char* e = std::getenv("KP_RNG_THREADS")) nfill = std::max(1, std::min(16, std::atoi(e)));
    try {
      std::thread([this] { loop(true); }).detach();
      for (int i = 0; i < nfill; ++i) std::thread([this] { loop(false); }).detach();
    } catch (...) {
      return false;
    }
    pid_ = me;
    return true;
  }
  void loop(bool sequential) {
    Scratch sc;
    const pid_t me = getpid();
    for (;;) {
      Item t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        auto& q = sequential ? seq_ : fills_;
        (sequential ? cv_seq_ : cv_fill_).wait(lk, [&] { return !q.empty(); });
        if (pid_ != me) return;
        t = std::move(q.front());
        q.pop_front();
      }
      int rc = KP_OK;
      RngStats& st = rng_stats();
      const int64_t t0 = st.on ? RngStats::now() : 0;
      t_task_batch = t.tag;
      try {
        t.t(sc);
      } catch (const std::invalid_argument&) {
        rc = KP_EINVAL;
      } catch (...) {
        rc = KP_ENOMEM;
      }
      t_task_batch = 0;
      if (st.on) {
        st.span(sequential ? st.seq_ns : st.pool_ns, t0);
        ++(sequential ? st.seq_tasks : st.pool_tasks);
      }
      std::lock_guard<std::mutex> lk(mu_);
      if (rc != KP_OK && fail_rc_ == KP_OK) fail_rc_ = rc;
      bp_.done(t.tag);
      --pending_;
      cv_done_.notify_all();
    }
  }
  struct Item {
    Task t;
    int64_t tag = 0;
  };
  std::mutex mu_;
  std::condition_variable cv_seq_, cv_fill_, cv_done_;
  std::deque<Item> seq_, fills_;
  BatchPending bp_;
  int64_t pending_ = 0;
  int fail_rc_ = KP_OK;  // first failure of a queued task since the last wait()
  pid_t pid_ = 0;
};

// Queue one slot's TransE epoch draws (see the deferred protocol above) from the torch
// generator `mt`, which is advanced past the slot's randints.  out == nullptr: a slot
// another rank post-trains -- only the generators advance (the numpy shuffles still run:
// their consumption is data-dependent), nothing is written.
int te_enqueue(TorchMt& mt, uint32_t* np_key, int32_t* np_pos, int32_t R, int32_t epochs, int32_t ratio, uint32_t nent,
               int32_t* out) {
  if (R == 0 || epochs == 0) return KP_OK;  // np.random.shuffle of an empty array draws nothing
  const TorchMt snap = mt;
  mt.skip((uint64_t)epochs * 2u * (uint64_t)ratio * (uint64_t)R);
  Task seq = [=](Scratch& sc) {
    if (g_perms_inline || !out) {
      te_shuffles(np_key, np_pos, R, epochs, out, sc.np, sc.idx, sc.jv);
      return;
    }
    // The sequential worker only walks the chain (no stores: 2.4 vs 3.7-4.2 ms per bench
    // batch on the box, tools/rng_bench.cpp, profiles/r05/rng_bench_box.txt), from a
    // snapshot of the numpy state taken here; a pool task replays the same chain from the
    // snapshot with the draws stored (in ordinary memory: `out` may be page-locked, where
    // the scattered stores ran ~1.5x slower) and then runs the permutation chain into out
    auto snap = std::make_shared<std::vector<uint32_t>>(np_key, np_key + kN);
    const int32_t pos0 = *np_pos;
    te_draws(np_key, np_pos, R, epochs, nullptr, 0, sc.np);
    auto replay = [=](Scratch& s2) {
      int32_t p = pos0;
      s2.jv.resize((size_t)R * (size_t)epochs);
      te_draws(snap->data(), &p, R, epochs, s2.jv.data(), (size_t)R, s2.np);
      te_perms(R, epochs, s2.jv.data(), (size_t)R, out, s2.idx);
    };
    if (!DrawQueue::get().enqueue(Task(), replay)) replay(sc);
  };
  Task fill;
  if (out)
    fill = [=](Scratch& sc) {
      TorchMt m = snap;
      te_randints(m, R, epochs, ratio, nent, out, sc.draw);
    };
  if (!DrawQueue::get().enqueue(seq, fill)) {
    // no worker threads: finish every queued task first (numpy order), then this one
    const int rc = DrawQueue::get().wait();
    if (rc != KP_OK) return rc;
    Scratch sc;
    seq(sc);
    if (fill) fill(sc);
  }
  return KP_OK;
}

// The torch-stream walk of kp_rng_transe_calls_async on a thread of its own: tasks run in
// submission order on one TorchMt carried from task to task (loaded from the caller's
// state by the first task after a kp_rng_torch_take, handed back by the next take), so the
// scheduling thread only queues.  The walk itself queues the numpy shuffles and randint
// fills on the DrawQueue, in order.
class TorchWalker {
 public:
  static TorchWalker& get() {
    static TorchWalker* w = new TorchWalker();  // never destroyed: the thread is detached
    return *w;
  }
  // false: no thread (the caller runs the task inline on the carried / loaded state)
  bool submit(const uint8_t* ts, std::function<int(TorchMt&)> task) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!ensure_locked()) return false;
    if (!carried_) {
      mt_.load(ts);
      carried_ = true;
    }
    const int64_t tag = submit_tag();
    q_.push_back(std::make_pair(std::move(task), tag));
    ++pending_;
    bp_.add(tag);
    cv_work_.notify_all();
    return true;
  }
  // every walk of the batches <= id done (see DrawQueue::wait_batch); the carried stream
  // stays with the walker
  int wait_batch(int64_t id) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return bp_.clear_upto(id); });
    return fail_rc_;
  }
  // wait for every queued walk; then, if a walk carries the stream, store it into ts and
  // release it (*taken = 1)
  int take(uint8_t* ts, int32_t* taken) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [this] { return pending_ == 0; });
    if (taken) *taken = 0;
    if (carried_ && ts) {
      mt_.store(ts);
      carried_ = false;
      if (taken) *taken = 1;
    }
    const int rc = fail_rc_;
    fail_rc_ = KP_OK;
    if (rc != KP_OK) carried_ = false;  // a failed walk leaves a partial stream: nothing continues it
    return rc;
  }
  int wait() { return take(nullptr, nullptr); }

 private:
  bool ensure_locked() {
    const pid_t me = getpid();
    if (pid_ == me) return true;
    q_.clear();
    bp_ = BatchPending();
    pending_ = 0;
    carried_ = false;
    try {
      std::thread([this] { loop(); }).detach();
    } catch (...) {
      return false;
    }
    pid_ = me;
    return true;
  }
  void loop() {
    const pid_t me = getpid();
    for (;;) {
      std::pair<std::function<int(TorchMt&)>, int64_t> t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_work_.wait(lk, [&] { return !q_.empty(); });
        if (pid_ != me) return;
        t = std::move(q_.front());
        q_.pop_front();
      }
      int rc;
      RngStats& st = rng_stats();
      const int64_t t0 = st.on ? RngStats::now() : 0;
      t_task_batch = t.second;  // the shuffles it queues belong to the same batch
      try {
        rc = t.first(mt_);  // mt_ is only touched here and under mu_ with the queue empty
      } catch (const std::invalid_argument&) {
        rc = KP_EINVAL;
      } catch (...) {
        rc = KP_ENOMEM;
      }
      t_task_batch = 0;
      if (st.on) st.span(st.walk_ns, t0);
      std::lock_guard<std::mutex> lk(mu_);
      if (rc != KP_OK && fail_rc_ == KP_OK) fail_rc_ = rc;
      bp_.done(t.second);
      --pending_;
      cv_done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::deque<std::pair<std::function<int(TorchMt&)>, int64_t>> q_;
  BatchPending bp_;
  int64_t pending_ = 0;
  int fail_rc_ = KP_OK;
  bool carried_ = false;
  TorchMt mt_;
  pid_t pid_ = 0;
};

// every draw of n TransE compute_relevance calls from the torch stream `mt` (see
// kp_rng_transe_calls)
int transe_calls_walk(TorchMt& mt, uint32_t* np_key, int32_t* np_pos, int32_t cap, int32_t D, int32_t d,
                      float xavier_std, int32_t n, const int32_t* R_base, const int32_t* R_pt, const uint8_t* want,
                      int32_t epochs, int32_t ratio, uint32_t nent, float* x_base, float* x_pt, int32_t* out) {
  int32_t* o = out;
  for (int32_t i = 0; i < n; ++i) {
    mt.skip((uint64_t)D);  // torch.rand(1, D): one output per element, values unused
    const int w = want ? want[i] : 3;  // bit 0: base draws wanted here, bit 1: the pt draws
    normal_draw(mt, d, 0.0f, xavier_std, cap, x_base + (size_t)i * d);  // base KelpieTransE's xavier_normal_
    if (R_base[i] >= 0) {
      const int rc = te_enqueue(mt, np_key, np_pos, R_base[i], epochs, ratio, nent, (w & 1) ? o : nullptr);
      if (rc != KP_OK) return rc;
      if (w & 1) o += (size_t)epochs * 3 * R_base[i];
    }
    normal_draw(mt, d, 0.0f, xavier_std, cap, x_pt + (size_t)i * d);  // the post-trained one's
    if (R_pt[i] >= 0) {
      const int rc = te_enqueue(mt, np_key, np_pos, R_pt[i], epochs, ratio, nent, (w & 2) ? o : nullptr);
      if (rc != KP_OK) return rc;
      if (w & 2) o += (size_t)epochs * 3 * R_pt[i];
    }
  }
  return KP_OK;
}

int transe_calls_check(size_t tlen, uint32_t* np_key, int32_t* np_pos, int32_t cap, int32_t D, int32_t d, int32_t n,
                       const int32_t* R_base, const int32_t* R_pt, const uint8_t* want, int32_t epochs, int32_t ratio,
                       int64_t n_entities, float* x_base, float* x_pt, int32_t* out) {
  if (tlen < 24 + kN * 8 || !np_key || !np_pos || (cap != 0 && cap != 1) || D < 0 || d < 16 || n < 0 ||
      (n > 0 && (!R_base || !R_pt || !x_base || !x_pt)) || epochs < 0 || ratio < 1 || n_entities < 1 ||
      n_entities >= (1LL << 32))
    return KP_EINVAL;
  int64_t words = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (R_base[i] < -1 || R_pt[i] < -1) return KP_EINVAL;
    const int w = want ? want[i] : 3;
    words += (int64_t)epochs * 3 * ((w & 1 ? std::max(R_base[i], 0) : 0) + (w & 2 ? std::max(R_pt[i], 0) : 0));
  }
  if (words > 0 && !out) return KP_EINVAL;
  return KP_OK;
}

}  // namespace

extern "C" {

int kp_rng_transe_epochs(uint8_t* ts, size_t tlen, uint32_t* np_key, int32_t* np_pos, int32_t R, int32_t epochs,
                         int32_t ratio, int64_t n_entities, int32_t* out) {
  if (!ts || tlen < 24 + kN * 8 || !np_key || !np_pos || R < 0 || epochs < 0 || ratio < 1 || n_entities < 1 ||
      n_entities >= (1LL << 32) || (R > 0 && epochs > 0 && !out))
    return KP_EINVAL;
  if (*np_pos < 0 || *np_pos > kN) return KP_EINVAL;
  try {
    auto shuffles = [&] {
      NumpyMt np;
      std::vector<int32_t> idx, jv;
      te_shuffles(np_key, np_pos, R, epochs, out, np, idx, jv);
    };
    auto randints = [&] {
      TorchMt mt;
      mt.load(ts);
      std::vector<uint32_t> draw;
      te_randints(mt, R, epochs, ratio, (uint32_t)n_entities, out, draw);
      mt.store(ts);
    };
    if (R >= 16 && epochs >= 4) {
      const std::function<void()> a = randints, b = shuffles;
      Helper::get().run2(a, b);
    } else {
      shuffles();
      randints();
    }
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_transe_enqueue(uint8_t* ts, size_t tlen, uint32_t* np_key, int32_t* np_pos, int32_t R, int32_t epochs,
                          int32_t ratio, int64_t n_entities, int32_t* out) {
  if (!ts || tlen < 24 + kN * 8 || !np_key || !np_pos || R < 0 || epochs < 0 || ratio < 1 || n_entities < 1 ||
      n_entities >= (1LL << 32) || (R > 0 && epochs > 0 && !out))
    return KP_EINVAL;
  if (R == 0 || epochs == 0) return KP_OK;  // np.random.shuffle of an empty array draws nothing
  try {
    TorchMt mt;
    mt.load(ts);
    const int rc = te_enqueue(mt, np_key, np_pos, R, epochs, ratio, (uint32_t)n_entities, out);
    if (rc != KP_OK) return rc;
    mt.store(ts);
  } catch (const std::invalid_argument&) {
    return KP_EINVAL;
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_transe_calls(uint8_t* ts, size_t tlen, uint32_t* np_key, int32_t* np_pos, int32_t cap, int32_t D,
                        int32_t d, float xavier_std, int32_t n, const int32_t* R_base, const int32_t* R_pt,
                        const uint8_t* want, int32_t epochs, int32_t ratio, int64_t n_entities, float* x_base,
                        float* x_pt, int32_t* out) {
  if (!ts) return KP_EINVAL;
  int rc = transe_calls_check(tlen, np_key, np_pos, cap, D, d, n, R_base, R_pt, want, epochs, ratio, n_entities,
                              x_base, x_pt, out);
  if (rc != KP_OK) return rc;
  try {
    // a stream still carried by an asynchronous walk continues from where it ends
    int32_t taken = 0;
    rc = TorchWalker::get().take(ts, &taken);
    if (rc != KP_OK) return rc;
    TorchMt mt;
    mt.load(ts);
    rc = transe_calls_walk(mt, np_key, np_pos, cap, D, d, xavier_std, n, R_base, R_pt, want, epochs, ratio,
                           (uint32_t)n_entities, x_base, x_pt, out);
    if (rc != KP_OK) return rc;
    mt.store(ts);
  } catch (const std::invalid_argument&) {
    return KP_EINVAL;
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_transe_calls_async(const uint8_t* ts, size_t tlen, uint32_t* np_key, int32_t* np_pos, int32_t cap,
                              int32_t D, int32_t d, float xavier_std, int32_t n, const int32_t* R_base,
                              const int32_t* R_pt, const uint8_t* want, int32_t epochs, int32_t ratio,
                              int64_t n_entities, float* x_base, float* x_pt, int32_t* out) {
  if (!ts) return KP_EINVAL;
  const int rc = transe_calls_check(tlen, np_key, np_pos, cap, D, d, n, R_base, R_pt, want, epochs, ratio,
                                    n_entities, x_base, x_pt, out);
  if (rc != KP_OK) return rc;
  try {
    std::vector<int32_t> rb(R_base, R_base + n), rp(R_pt, R_pt + n);
    std::vector<uint8_t> wv;
    if (want) wv.assign(want, want + n);
    const uint32_t nent = (uint32_t)n_entities;
    auto task = [=](TorchMt& mt) {
      return transe_calls_walk(mt, np_key, np_pos, cap, D, d, xavier_std, n, rb.data(), rp.data(),
                               wv.empty() ? nullptr : wv.data(), epochs, ratio, nent, x_base, x_pt, out);
    };
    if (!TorchWalker::get().submit(ts, task)) {
      // no walker thread (nothing is carried then: a failed start drops the carried
      // state): walk here on the caller's state and say so, so that the caller keeps the
      // stream itself instead of expecting a walk to carry it
      TorchMt mt;
      mt.load(ts);
      const int r2 = task(mt);
      if (r2 != KP_OK) return r2;
      mt.store(const_cast<uint8_t*>(ts));
      return KP_INLINE;
    }
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_torch_take(uint8_t* ts, size_t tlen, int32_t* taken) {
  if (!ts || tlen < 24 + kN * 8 || !taken) return KP_EINVAL;
  return TorchWalker::get().take(ts, taken);
}

// the word layout of kp_rng_conve_masks: per step, one word-aligned run per segment
static int conve_mask_plan(int32_t n_steps, const int32_t* rows, int32_t n_seg, const int32_t* seg_elems,
                           const double* seg_keep, uint64_t* draws) {
  if (n_steps < 0 || n_seg < 0 || n_seg > 8 || (n_steps > 0 && !rows) || (n_seg > 0 && (!seg_elems || !seg_keep)))
    return KP_EINVAL;
  uint64_t total = 0;
  for (int j = 0; j < n_seg; ++j)
    if (seg_elems[j] <= 0 || !(seg_keep[j] >= 0.0 && seg_keep[j] <= 1.0)) return KP_EINVAL;
  for (int st = 0; st < n_steps; ++st) {
    if (rows[st] < 0) return KP_EINVAL;
    for (int j = 0; j < n_seg; ++j)
      if (seg_keep[j] > 0.0) total += (uint64_t)rows[st] * (uint64_t)seg_elems[j];
  }
  *draws = total;
  return KP_OK;
}

static void conve_mask_fill(TorchMt& m, int32_t n_steps, const int32_t* rows, int32_t n_seg,
                            const int32_t* seg_elems, const double* seg_keep, uint32_t* out,
                            std::vector<uint32_t>& buf) {
  size_t w0 = 0;
  for (int st = 0; st < n_steps; ++st)
    for (int j = 0; j < n_seg; ++j) {
      const uint64_t n = (uint64_t)rows[st] * (uint64_t)seg_elems[j];
      const size_t nw = (size_t)((n + 31) / 32);
      if (seg_keep[j] > 0.0)
        bernoulli_words(m, n, seg_keep[j], out + w0, buf);  // one random64 (two outputs) per element
      else
        std::memset(out + w0, 0, sizeof(uint32_t) * nw);  // rate 1: zeros, nothing drawn
      w0 += nw;
    }
}

int kp_rng_conve_masks_enqueue(uint8_t* ts, size_t tlen, int32_t n_steps, const int32_t* rows, int32_t n_seg,
                               const int32_t* seg_elems, const double* seg_keep, uint32_t* out) {
  if (!ts || tlen < 24 + kN * 8 || (n_steps > 0 && n_seg > 0 && !out)) return KP_EINVAL;
  uint64_t total = 0;
  int rc = conve_mask_plan(n_steps, rows, n_seg, seg_elems, seg_keep, &total);
  if (rc != KP_OK) return rc;
  try {
    TorchMt mt;
    mt.load(ts);
    std::vector<int32_t> rv(rows, rows + n_steps);
    std::vector<int32_t> ev(seg_elems, seg_elems + n_seg);
    std::vector<double> kv(seg_keep, seg_keep + n_seg);
    TorchMt adv = mt;
    adv.skip(2 * total);
    Task fill = [=](Scratch& sc) {
      TorchMt m = mt;
      conve_mask_fill(m, n_steps, rv.data(), n_seg, ev.data(), kv.data(), out, sc.draw);
    };
    if (!DrawQueue::get().enqueue(Task(), fill)) {
      rc = DrawQueue::get().wait();
      if (rc != KP_OK) return rc;
      Scratch sc;
      fill(sc);
    }
    adv.store(ts);
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_batch_close(int64_t* id) {
  if (!id) return KP_EINVAL;
  *id = g_open_batch.fetch_add(1, std::memory_order_acq_rel);
  return KP_OK;
}

int kp_rng_batch_wait(int64_t id) {
  // the walks first: they queue the batch's shuffles and fills
  const int rw = TorchWalker::get().wait_batch(id);
  const int rd = DrawQueue::get().wait_batch(id);
  return rw != KP_OK ? rw : rd;
}

int kp_rng_wait(void) {
  const int64_t t_wait = rng_stats().on ? RngStats::now() : 0;
  // the torch walks queue draws: they finish first
  const int rw = TorchWalker::get().wait();
  const int rd = DrawQueue::get().wait();
  if (rng_stats().on) rng_stats().report(t_wait);
  return rw != KP_OK ? rw : rd;
}

int kp_rng_conve_masks(uint8_t* ts, size_t tlen, int32_t n_steps, const int32_t* rows, int32_t n_seg,
                       const int32_t* seg_elems, const double* seg_keep, uint32_t* out) {
  if (!ts || tlen < 24 + kN * 8 || (n_steps > 0 && n_seg > 0 && !out)) return KP_EINVAL;
  uint64_t total = 0;
  const int rc = conve_mask_plan(n_steps, rows, n_seg, seg_elems, seg_keep, &total);
  if (rc != KP_OK) return rc;
  try {
    TorchMt mt;
    mt.load(ts);
    std::vector<uint32_t> buf;
    conve_mask_fill(mt, n_steps, rows, n_seg, seg_elems, seg_keep, out, buf);
    mt.store(ts);
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_bernoulli_bits(uint8_t* st, size_t len, uint64_t n, double p, uint32_t* out) {
  if (!st || len < 24 + kN * 8 || (n > 0 && !out)) return KP_EINVAL;
  try {
    TorchMt mt;
    mt.load(st);
    std::vector<uint32_t> buf;
    bernoulli_words(mt, n, p, out, buf);
    mt.store(st);
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_rng_normal(uint8_t* ts, size_t tlen, int64_t n, float mean, float std_, int32_t cap, float* out) {
  if (!ts || tlen < 24 + kN * 8 || n < 16 || !out || (cap != 0 && cap != 1)) return KP_EINVAL;
  TorchMt mt;
  mt.load(ts);
  normal_draw(mt, n, mean, std_, cap, out);
  mt.store(ts);
  return KP_OK;
}

int kp_mt19937_discard(uint8_t* st, size_t len, uint64_t n) {
  if (!st || len < 24 + kN * 8) return KP_EINVAL;
  // the jump-ahead (mt_charpoly / mt_jump_poly) can throw; no exception crosses the C ABI,
  // and the caller's state blob is written only after a successful skip
  try {
    TorchMt mt;
    mt.load(st);
    mt.skip(n);
    mt.store(st);
  } catch (const std::bad_alloc&) {
    return KP_ENOMEM;
  } catch (...) {
    return KP_EINVAL;
  }
  return KP_OK;
}

}  // extern "C"
