// kp_attn.hpp -- the flash-attention-shaped pass over the frozen entity table
// shared by the ComplEx (softmax cross-entropy) and ConvE (sigmoid BCE)
// post-training steps.
#pragma once
#if (defined(KP_ATTN_NODMA) || defined(KP_DIAG_M0SAVE)) && !defined(KP_DIAGNOSTIC_BUILD)
#error "KP_ATTN_NODMA is a timing-only diagnostic (wrong results): build it with make diag"
#endif
#include <algorithm>

#include "kp_common.hpp"

namespace kpattn {

#ifdef KP_ATTN_STAMPS
// diagnostic build only (make stamps): per-phase issue cycles of kp_attn, summed
// over waves: [S phase, softmax, O phase, tile end (DMA wait + barrier), tiles]
__device__ unsigned long long g_attn_stamps[8];
#define KP_STAMP(v) v = __builtin_amdgcn_s_memtime()
#else
#define KP_STAMP(v) (void)0
#endif

constexpr float kNegInf = -__builtin_huge_valf();

// ----------------------------------------------------------------------------
// q = lhs o rel  (complex.py:65-72): [a c - b e | a e + b c], no fp contraction
// ----------------------------------------------------------------------------
__device__ __forceinline__ float cx_q(const float* __restrict__ lhs, const float* __restrict__ rel, int d,
                                      int half) {
  if (d < half) {
    float ac = __fmul_rn(lhs[d], rel[d]);
    float be = __fmul_rn(lhs[d + half], rel[d + half]);
    return __fsub_rn(ac, be);
  } else if (d < 2 * half) {
    int i = d - half;
    float ae = __fmul_rn(lhs[i], rel[d]);
    float bc = __fmul_rn(lhs[d], rel[i]);
    return __fadd_rn(ae, bc);
  }
  return 0.f;
}

// ----------------------------------------------------------------------------
// LDS-DMA: one wave-instruction copies 64 lanes x 16 B from per-lane global
// addresses to the wave-uniform LDS byte address `lds_base` (+16 B per lane).  Two
// forms (template flag BUILTIN):
//  - __builtin_amdgcn_global_load_lds: hipcc sets M0 itself and counts the copy, and
//    waits for it (vmcnt(0)) before any later LDS read the compiler can see.  Used
//    where every LDS read is inline asm (kp_attn, the asm read form of kp_attn3): the
//    compiler sees no read to serialise, so the copy streams under the MFMAs.
//  - inline asm (M0 written inside the statement): for the compiler-visible read form
//    of kp_attn3 (ConvE), where the builtin's waits would drain every copy before the
//    next O-phase read (4.18 vs 2.05 ms per launch measured with the spread schedule).
// Either way the kernel owns the hand-off: `s_waitcnt vmcnt(0)` before the barrier
// that gives the buffer to the readers.
// ----------------------------------------------------------------------------
template <bool BUILTIN>
__device__ __forceinline__ void glds16(const float* gp, uint32_t lds_base) {
  if constexpr (BUILTIN) {
    __builtin_amdgcn_global_load_lds(gp, (__attribute__((address_space(3))) void*)(uintptr_t)lds_base, 16, 0, 0);
  } else {
    // M0 is reserved to the compiler (a clobber of it is not honoured), so the DMA saves
    // it and puts it back: any M0 the compiler set stays valid across the statement
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds_base), "v"(gp)
                 : "memory");
  }
}

// LDS reads issued through inline asm, so their placement is the source order:
// each k-step's operands are read one k-step ahead, and the kernel waits with a
// counted lgkmcnt (LDS returns in order).  tied() makes the consumer depend on the
// wait, so no MFMA is scheduled above it.
__device__ __forceinline__ f32x4 lds_rd128(uint32_t addr) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ float lds_rd32(uint32_t addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N));
}
__device__ __forceinline__ f32x4 tied(f32x4 v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ float tied(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

// ----------------------------------------------------------------------------
// kp_attn: per query q (row of Qpre), over frozen entities [key_begin, key_end):
//   m = max_e s_e,  l = sum_e exp(s_e - m),  O = sum_e exp(s_e - m) E_e
// with s_e = q . E_e.  4 waves x 16 queries per workgroup share a 32-entity E
// tile in LDS (double buffered, staged by LDS-DMA while the previous tile is
// consumed).  fp32 MFMA 16x16x4 in the swapped form S^T = E . Q^T (key on the C
// row), so P already sits in the B-operand layout of O^T += E^T . P.
//   lane l: g = l>>4, c = l&15.  Q fragment qv[j][i] = Q[c][16j+4g+i] stays in
//   VGPRs; O^T accumulators O[j][r] = O[d = od(j, 4g+r)][q = c] with the
//   dimension map od(j, i) = 64(j/4) + 4i + j%4 for j < 4(DB/4), else
//   64(DB/4) + 16(j%4) + i, so a lane's A operands for four blocks are one
//   16-byte LDS read.
// Softmax reference: instead of the online max (whose rescaling of O under a
// branch makes the compiler copy the whole AGPR-resident O block every tile),
// weights are exp(s - m_ref) with m_ref = the first tile's max.  fp32 is scale
// invariant, so this is as accurate as long as s - m_ref <= kMargin; the running
// max is tracked on the side and, in the rare case a later score exceeds
// m_ref + kMargin, the workgroup recomputes the split with m_ref = the exact max.
// MODE ATT_SOFTMAX_O (ComplEx step) / ATT_SOFTMAX (pairs: statistics only) /
// ATT_BCE_O (ConvE): instead of the softmax the BCELoss-through-sigmoid gradient
//   G(s) = ((p - y)/max(p(1-p),1e-12) * gs) * p(1-p)
//   (p = sigmoid(s), y = the smoothed non-target label, gs = 1/(b*N) per query,
//   bce_optimizer.py:35,98-112) weights O = sum_e G(s_e) E_e.
// ----------------------------------------------------------------------------
enum { ATT_SOFTMAX_O = 0, ATT_SOFTMAX = 1, ATT_BCE_O = 2 };
constexpr float kMargin = 40.0f;  // max exponent s - m_ref of a pass-1 weight (e^40 * N * |E| << FLT_MAX)

// Work partition (stream-K style): the (64-query tile, 32-entity key tile) iterations
// of all query tiles, in query-tile-major order, are cut into equal contiguous
// ranges of per_wg iterations, one per workgroup, with exactly as many workgroups
// as the GPU holds at once.  A workgroup's range covers key-tile segments of one or
// more query tiles; each segment writes a partial (m, l, O) into slot `part` of its
// query tile, and the owner of a tile's last segment fills the unused slots up to
// n_parts with empty partials (m = -inf, l = 0, O = 0).  Consumers merge n_parts
// partials per query exactly as they merged N-split partials.
struct AttnWork {
  int ktq;      // key tiles per query tile, ceil(n_ent / 32)
  int per_wg;   // iterations per workgroup (stream-K)
  int n_parts;  // partial slots per query
  int ranges;   // > 0: XCD-grouped aligned key ranges (kp_attn3 only; attn_plan_ranges)
};

template <int DB, int MODE>
__global__ __launch_bounds__(256, 1) void kp_attn(const float* __restrict__ E, int n_ent,
                                                  const float* __restrict__ Qpre, int nq, AttnWork wk,
                                                  float* __restrict__ out_m, float* __restrict__ out_l,
                                                  float* __restrict__ out_O, const float* __restrict__ qscale,
                                                  float ylo) {
  constexpr bool WITH_O = MODE != ATT_SOFTMAX;
  constexpr int DP = 16 * DB;
  // entities per LDS tile: NSUB 16-entity MFMA sub-tiles.  32, not 64: a 64-entity
  // double buffer of narrow rows (ConvE, 133 KB) leaves room for one workgroup per CU
  // instead of two, and two co-resident workgroups measured faster (4.26 vs 4.63 ms).
  constexpr int NSUB = 2;
  constexpr int KT = 16 * NSUB;
  constexpr int F4_ROW = DP / 4;
  constexpr int SEGS = (F4_ROW + 63) / 64;  // 1-KiB LDS-DMA pieces per row (no piece crosses a row)
  // LDS row stride: whole pieces plus 4 floats (S = 4 mod 64 banks: conflict-free
  // ds_read_b128 across the 16 rows of an S read and along the row of an O read).
  // Lanes past the row's end load a clamped duplicate into the padding, so every
  // LDS-DMA instruction runs with all 64 lanes and no branch.
  constexpr int S = 256 * SEGS + 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][KT][S]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  int key_begin = 0, key_end = 0;  // the current segment's keys (captured by the DMA lambdas)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;

  // LDS-DMA staging: piece (row, seg) = 64 lanes x 16 B of one entity row, landing at
  // row*S + seg*256.  Rows past the table are clamped to a valid row; their scores
  // are masked, so they add 0.
  // Wave w issues pieces ins = w + 4p, p < PIECES; with SEGS in {1, 2} the piece's
  // segment (ins % SEGS) is fixed per wave, so the lane mask is too.
  static_assert(SEGS == 1 || SEGS == 2, "rows wider than 512 floats need more LDS-DMA pieces");
  constexpr int PIECES = KT * SEGS / 4;
  const int my_seg = w % SEGS;
  const float* lane_src = E + 4 * min(my_seg * 64 + lane, F4_ROW - 1);
  auto issue_piece = [&](int tile, int buf, int p) {
    const int row = (w + 4 * p) / SEGS;
    const int grow = min(key_begin + tile * KT + row, n_ent - 1);
    const uint32_t dst = lds0 + 4u * (uint32_t)(buf * (KT * S) + row * S + my_seg * 256);
    glds16<true>(lane_src + (size_t)grow * DP, __builtin_amdgcn_readfirstlane(dst));
  };
  auto issue = [&](int tile, int buf) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) issue_piece(tile, buf, p);
  };
  const int QT = (nq + 63) / 64;
  const long long total = (long long)QT * wk.ktq;
  long long it = (long long)blockIdx.x * wk.per_wg;
  const long long it_end = min(total, it + (long long)wk.per_wg);
  while (it < it_end) {  // the segments of this workgroup's range (uniform across waves)
  const int qt = (int)(it / wk.ktq);
  const int kt0 = (int)(it - (long long)qt * wk.ktq);
  const int kt1 = (int)min((long long)wk.ktq, (long long)kt0 + (it_end - it));
  const int part = (int)blockIdx.x - (int)(((long long)qt * wk.ktq) / wk.per_wg);
  key_begin = kt0 * KT;
  key_end = min(n_ent, kt1 * KT);
  const int ntiles = kt1 - kt0;
  const int q = qt * 64 + 16 * w + c;
  const bool valid = q < nq;
  // ---- Q fragment -> registers
  float qv[DB][4];
  float gsc = 0.f;
  if (MODE == ATT_BCE_O) gsc = valid ? qscale[q] : 0.f;
  {
    const float* qp = Qpre + (size_t)(valid ? q : 0) * DP;
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      float4 v = *reinterpret_cast<const float4*>(qp + 16 * j + 4 * g);
      qv[j][0] = valid ? v.x : 0.f;
      qv[j][1] = valid ? v.y : 0.f;
      qv[j][2] = valid ? v.z : 0.f;
      qv[j][3] = valid ? v.w : 0.f;
    }
  }
  f32x4 O[WITH_O ? DB : 1];
  float m_ref = kNegInf, l_run = 0.f;

  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int j = 0; j < (WITH_O ? DB : 1); ++j) O[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    l_run = 0.f;
    float m_seen = kNegInf;  // running max of this lane's scores
    if (ntiles > 0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

#ifdef KP_ATTN_STAMPS
    unsigned long long st_acc[4] = {0, 0, 0, 0};
#endif
    for (int t = 0; t < ntiles; ++t) {
#ifdef KP_ATTN_STAMPS
      unsigned long long ts0, ts1, ts2, ts3, ts4;
#endif
      KP_STAMP(ts0);
      const int k0 = key_begin + t * KT;
      // ---- S^T per 16-entity sub-tile u: sc[u][r] = q_c . E[k0 + 16u + 4g + r]
      const uint32_t sbase = lds0 + 4u * (uint32_t)((t & 1) * (KT * S) + c * S + 4 * g);
      f32x4 sc[NSUB];
      f32x4 ra[2][NSUB];
#pragma unroll
      for (int u = 0; u < NSUB; ++u) {
        sc[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        ra[0][u] = lds_rd128(sbase + 4u * 16u * S * u);
      }
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        if (j + 1 < DB) {
#pragma unroll
          for (int u = 0; u < NSUB; ++u) ra[(j + 1) & 1][u] = lds_rd128(sbase + 4u * 16u * S * u + 64u * (j + 1));
          lgkm_wait<NSUB>();
        } else {
          lgkm_wait<0>();
        }
        f32x4 a[NSUB];
#pragma unroll
        for (int u = 0; u < NSUB; ++u) a[u] = tied(ra[j & 1][u]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int u = 0; u < NSUB; ++u) sc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][i], qv[j][i], sc[u], 0, 0, 0);
      }
      // next tile's LDS-DMA, issued while the last S MFMAs drain (after the last tile
      // it reloads clamped rows into the idle buffer: harmless and branch-free)
#ifndef KP_ATTN_NODMA  // diagnostic: isolates the DMA issue cost (wrong results)
      issue(t + 1, (t + 1) & 1);
#endif
      KP_STAMP(ts1);
      float pw[NSUB][4];
      if (MODE == ATT_BCE_O) {
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // reference op order, with the two divisions as hardware reciprocals
            // (v_rcp_f32, 1 ulp): the IEEE division sequences were 30 % of the tile
            const float x0 = __builtin_amdgcn_rcpf(1.0f + __expf(-sc[u][r]));
            const float w0 = (1.0f - x0) * x0;
            pw[u][r] = (k0 + 16 * u + 4 * g + r < key_end)
                           ? (((x0 - ylo) * __builtin_amdgcn_rcpf(fmaxf(w0, 1e-12f))) * gsc) * w0
                           : 0.f;
          }
      } else {
        float v[NSUB][4];
        float tmax = kNegInf;
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[u][r] = (k0 + 16 * u + 4 * g + r < key_end) ? sc[u][r] : kNegInf;
            tmax = fmaxf(tmax, v[u][r]);
          }
        m_seen = fmaxf(m_seen, tmax);
        if (pass == 0 && t == 0) {  // the reference max of pass 1: the first tile's
          float mq = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
          m_ref = fmaxf(mq, __shfl_xor(mq, 32, 64));
        }
        float lt = 0.f;
#pragma unroll
        for (int u = 0; u < NSUB; ++u) {
#pragma unroll
          for (int r = 0; r < 4; ++r) pw[u][r] = __expf(v[u][r] - m_ref);
          lt += (pw[u][0] + pw[u][1]) + (pw[u][2] + pw[u][3]);
        }
        l_run += lt;
      }
      KP_STAMP(ts2);
      if (WITH_O) {
        // O^T += E^T P over the KT entities: k-step rr takes entity 16(rr/4) + 4g + rr%4.
        // A-operand lane (i = c, k = g) of block j is E[entity][od(j, c)]: 4 consecutive
        // blocks share one 16-B LDS read; the DB % 4 remaining blocks take one 4-B read each.
        constexpr int NB4 = DB / 4, REM = DB % 4, NR = NB4 + REM, NK = 4 * NSUB;
        f32x4 ob[2][NB4 > 0 ? NB4 : 1];
        float os[2][REM > 0 ? REM : 1];
        auto load_k = [&](int rr, int b) {
          const int row = 16 * (rr >> 2) + 4 * g + (rr & 3);
          const uint32_t base = lds0 + 4u * (uint32_t)((t & 1) * (KT * S) + row * S);
#pragma unroll
          for (int m = 0; m < NB4; ++m) ob[b][m] = lds_rd128(base + 4u * (64 * m + 4 * c));
#pragma unroll
          for (int k = 0; k < REM; ++k) os[b][k] = lds_rd32(base + 4u * (64 * NB4 + 16 * k + c));
        };
        load_k(0, 0);
#pragma unroll
        for (int rr = 0; rr < NK; ++rr) {
          const int b = rr & 1;
          if (rr + 1 < NK) {
            load_k(rr + 1, b ^ 1);
            lgkm_wait<NR>();
          } else {
            lgkm_wait<0>();
          }
          const float pv = pw[rr >> 2][rr & 3];
#pragma unroll
          for (int m = 0; m < NB4; ++m) {
            const f32x4 vv = tied(ob[b][m]);
            O[4 * m + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv.x, pv, O[4 * m + 0], 0, 0, 0);
            O[4 * m + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv.y, pv, O[4 * m + 1], 0, 0, 0);
            O[4 * m + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv.z, pv, O[4 * m + 2], 0, 0, 0);
            O[4 * m + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv.w, pv, O[4 * m + 3], 0, 0, 0);
          }
#pragma unroll
          for (int k = 0; k < REM; ++k) {
            const float vv = tied(os[b][k]);
            O[4 * NB4 + k] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv, pv, O[4 * NB4 + k], 0, 0, 0);
          }
        }
      }
      KP_STAMP(ts3);
      // tile t+1 landed (each wave waits for its own DMA) and every wave is done with buffer t&1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      KP_STAMP(ts4);
#ifdef KP_ATTN_STAMPS
      st_acc[0] += ts1 - ts0;
      st_acc[1] += ts2 - ts1;
      st_acc[2] += ts3 - ts2;
      st_acc[3] += ts4 - ts3;
#endif
    }
#ifdef KP_ATTN_STAMPS
    if (lane == 0) {
      for (int k = 0; k < 4; ++k) atomicAdd(&g_attn_stamps[k], st_acc[k]);
      atomicAdd(&g_attn_stamps[4], (unsigned long long)ntiles);
    }
#endif
    if (MODE == ATT_BCE_O) break;
    // exact max of the query; a second pass only if some weight exceeded e^kMargin
    float mq = fmaxf(m_seen, __shfl_xor(m_seen, 16, 64));
    mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
    if (pass == 1 || !__syncthreads_or(mq > m_ref + kMargin)) break;
    m_ref = mq;
  }

  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (valid) {
    const size_t o = (size_t)part * nq + q;
    if (g == 0 && MODE != ATT_BCE_O) {
      out_m[o] = m_ref;
      out_l[o] = l_tot;
    }
    if (WITH_O) {
      // O^T row i = 4g+r of block j holds dimension od(j, i)
      float* dst = out_O + o * DP;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * g + r;
#pragma unroll
        for (int m = 0; m < DB / 4; ++m)
          *reinterpret_cast<float4*>(dst + 64 * m + 4 * i) =
              make_float4(O[4 * m][r], O[4 * m + 1][r], O[4 * m + 2][r], O[4 * m + 3][r]);
#pragma unroll
        for (int k = 0; k < DB % 4; ++k) dst[64 * (DB / 4) + 16 * k + i] = O[4 * (DB / 4) + k][r];
      }
    }
  }
  // the owner of a query tile's last segment marks the unused partial slots empty
  if (kt1 == wk.ktq && valid) {
    for (int pp = part + 1; pp < wk.n_parts; ++pp) {
      const size_t o = (size_t)pp * nq + q;
      if (g == 0 && MODE != ATT_BCE_O) {
        out_m[o] = kNegInf;
        out_l[o] = 0.f;
      }
      if (WITH_O) {
        float* dst = out_O + o * DP;
        for (int d = 4 * g; d < DP; d += 16) *reinterpret_cast<float4*>(dst + d) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  it += kt1 - kt0;
  }
}

// Host: the stream-K partition for nq queries over n_ent keys on `slots` co-resident
// workgroups.  A workgroup takes at least ktq/15 key tiles, so a query tile is cut
// into at most 16 partials (the consumers' merge limit).
struct AttnPlan {
  AttnWork wk;
  int n_wg;
};
inline AttnPlan attn_plan(int nq, int n_ent, int slots) {
  const int QT = (nq + 63) / 64, ktq = (n_ent + 31) / 32;
  const long long total = (long long)QT * ktq;
  long long per = (total + slots - 1) / slots;
  per = std::max<long long>(per, (ktq + 14) / 15);
  per = std::max<long long>(per, 1);
  AttnPlan p{};
  p.n_wg = (int)((total + per - 1) / per);
  p.wk.ktq = ktq;
  p.wk.per_wg = (int)per;
  int parts = 1;
  for (int qt = 0; qt < QT; ++qt) {
    const long long w0 = ((long long)qt * ktq) / per, w1 = ((long long)(qt + 1) * ktq - 1) / per;
    parts = std::max(parts, (int)(w1 - w0 + 1));
  }
  p.wk.n_parts = parts;
  return p;
}

// Host: the XCD-grouped partition of kp_attn3.  The key tiles are cut into S aligned
// ranges; a unit is (query tile, range), numbered range-major, so consecutive units
// read the same keys.  Workgroup b (placed on XCD b % 8 by the dispatcher; used for
// speed only) takes logical id L = (b % 8) * (n_wg / 8) + b / 8 and units L, L + n_wg,
// ...: the workgroups of one XCD run consecutive units at the same time, so one key
// range streams into that XCD's L2 once and serves up to 32 query tiles, where the
// stream-K ranges of different workgroups are unrelated and every query tile re-reads
// the table from the Infinity Cache.  S minimises rounds x (range length + a per-unit
// overhead), at most 16 (the consumers' merge limit); every (query, range) partial is
// written.
inline AttnPlan attn_plan_ranges(int nq, int n_ent, int slots) {
  const int QT = (nq + 63) / 64, ktq = (n_ent + 31) / 32;
  const int n_wg = std::max(8, slots / 8 * 8);
  int best_s = 1;
  long long best = -1;
  for (int S = 1; S <= std::min(16, ktq); ++S) {
    const long long rounds = ((long long)QT * S + n_wg - 1) / n_wg;
    const long long cost = rounds * ((ktq + S - 1) / S + 2);
    if (best < 0 || cost < best) {
      best = cost;
      best_s = S;
    }
  }
  AttnPlan p{};
  p.wk.ktq = ktq;
  p.wk.per_wg = 0;
  p.wk.n_parts = best_s;
  p.wk.ranges = best_s;
  p.n_wg = (int)std::min<long long>(n_wg, ((long long)QT * best_s + 7) / 8 * 8);
  return p;
}

// LDS bytes of kp_attn<DB, *>
constexpr size_t attn_lds_bytes(int DB) {
  return 2u * 32u * (256u * ((4u * DB + 63u) / 64u) + 4u) * sizeof(float);
}

}  // namespace kpattn
