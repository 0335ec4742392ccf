// kp_attn4.hpp -- the ComplEx step attention (kp_attn3<DB, ATT_SOFTMAX_O>'s contract) as a
// cross-tile software pipeline.  EXPERIMENT, not part of the library: built only into the
// micro-benchmark (tools/attn_micro.hip with -Itools/attn4).  Correct (the micro's fp64
// check and output hash equal kp_attn3's on every shape) but no faster: 0.351-0.353 vs
// 0.353-0.358 ms (FB15k-237 shape), 1.300-1.303 vs 1.311-1.341 ms (DB100K shape), best
// variant KP_A4_SAHEAD=2 (profiles/r03k_attn4_micro.jsonl).
//
// kp_attn3 runs each 32-entity key tile as a dependent chain per wave: S = E . Q^T on
// the MFMA pipe, then the softmax weights and their three-piece split on the VALU, then
// O^T += E^T . P on the MFMA pipe, then a barrier.  With one wave per SIMD (the D = 400
// fragments take 448 registers) nothing covers the VALU part or the phase changes:
// measured per tile S 2.97k + weights/split 0.65k + O 2.72k + tile end 0.34k cycles
// against 4.8k of MFMA work.  Here the S MFMAs of tile t + 1 are
// interleaved with the O MFMAs of tile t, and the weights of tile t + 1 are computed in
// the issue gaps of the last O blocks of tile t, so the MFMA pipe always has independent
// work queued.
//
// That needs three tiles' worth of LDS at once (O of t, S of t + 1, the DMA of t + 2):
// 3 x 75 KiB does not fit.  The image is therefore laid out block-major inside a tile,
//   byte (entity e, dim d, piece p) = (e / 32) TILE_B + ((d / 16) 3 + p) 1024 + (e % 32) 32 + (d % 16) 2,
// so the 1-KiB DMA pieces are (16-dim block, piece) columns of the tile, and a block's
// LDS bytes are free as soon as the O MFMAs of that block have read them.  Per tile
// iteration (two LDS buffers, tile t in buf t & 1):
//   H1: O(t) blocks [0, OH1) with S(t+1) steps [0, SH1)  (S step j reads blocks 2j, 2j+1;
//       OH1 = 2 SH1), while the DMA brings tile t+1's blocks [OH1, DB) into buf (t+1) & 1
//       (whose tile t-1 is finished);                                      -- barrier
//   H2: O(t) blocks [OH1, DB) with S(t+1) steps [SH1, NS), while the DMA brings tile
//       t+2's blocks [0, OH1) into buf t & 1 (freed by H1); the weights and split of tile
//       t+1 ride in the last OSM O blocks;                                  -- barrier.
// Every wave issues the same MFMA groups in the same order; each group (an S step of 12
// MFMAs or an O block of 6) has exactly 6 LDS reads, issued two groups ahead one per
// MFMA issue gap (sched_barrier pins the order), so one counted lgkmcnt(6) before each
// group waits for exactly its operands.  S reads are never issued across a barrier that
// guards their DMA: each half starts with two O groups.
//
// Both read layouts are conflict-free under gfx950's lane groups without padding
// (S: ds_read_b128 of lanes (g, c) at c*32 + (g&1)*16 within a 1-KiB column; O:
// ds_read_b64_tr_b16, 32 lanes covering 256 contiguous bytes).  Arithmetic (bf16x3
// products in mfma3's order, centred weights, fp64 prefix sums of the shift, the
// exact-max second pass) is kp_attn3's; only the order of the O accumulation over key
// tiles is the same, the l sum is taken per element (not bitwise equal to kp_attn3).
#pragma once
#include <type_traits>

#include "kp_attn3.hpp"

namespace kpattn {

#if (defined(KP_A4_NODMA) || defined(KP_A4_NOSM) || defined(KP_A4_NOREAD)) && !defined(KP_DIAGNOSTIC_BUILD)
#error "kp_attn4 timing-only diagnostics (wrong results) need KP_DIAGNOSTIC_BUILD"
#endif
#ifndef KP_A4_DMA_PER_GROUP
#define KP_A4_DMA_PER_GROUP 2  // LDS-DMA pieces per wave issued with each MFMA group
#endif

__host__ __device__ constexpr int attn4_tile_bytes(int DB) { return DB * 3 * 1024; }
constexpr size_t attn4_lds_bytes(int DB) { return 2u * (size_t)attn4_tile_bytes(DB); }
// the pipelined form exists for the ComplEx d = 200 step (DB = 25: 13 S steps, 25 O blocks)
__host__ __device__ constexpr bool attn4_supported(int DB) { return DB == 25; }

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// Blocked split image of the fp32 table E [n_ent][DP] (zeroed by the caller): one thread
// per (entity, 2 dims).
template <int DP>
__global__ void kp_split3_blocked(const float* __restrict__ E, int n_ent, uint8_t* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n_ent * (DP / 2)) return;
  const int e = (int)(i / (DP / 2)), d = 2 * (int)(i % (DP / 2));
  __bf16 h[2], m[2], l[2];
  split3(E[(size_t)e * DP + d], h[0], m[0], l[0]);
  split3(E[(size_t)e * DP + d + 1], h[1], m[1], l[1]);
  const size_t base = (size_t)(e / 32) * attn4_tile_bytes(DP / 16) + (size_t)((d / 16) * 3) * 1024 +
                      (size_t)(e % 32) * 32 + (size_t)(d % 16) * 2;
  __bf16* p0 = reinterpret_cast<__bf16*>(out + base);
  __bf16* p1 = reinterpret_cast<__bf16*>(out + base + 1024);
  __bf16* p2 = reinterpret_cast<__bf16*>(out + base + 2048);
  p0[0] = h[0];
  p0[1] = h[1];
  p1[0] = m[0];
  p1[1] = m[1];
  p2[0] = l[0];
  p2[1] = l[1];
}

// asm LDS reads with the offset split over two bases (base, base + 32 KiB): the tile is
// 75 KiB and the instruction's offset field 16 bits
template <int OFF>
__device__ __forceinline__ bf16x8 rd8(uint32_t lo, uint32_t hi) {
  static_assert(OFF >= 0 && OFF < 32768 + 65536, "offset");
  if constexpr (OFF < 32768)
    return lds_rd_bf8<true>(lo, OFF);
  else
    return lds_rd_bf8<true>(hi, OFF - 32768);
}
template <int OFF>
__device__ __forceinline__ bf16x4 rd4(uint32_t lo, uint32_t hi) {
  if constexpr (OFF < 32768)
    return lds_rd_bf4<true>(lo, OFF);
  else
    return lds_rd_bf4<true>(hi, OFF - 32768);
}
template <int OFF>
__device__ __forceinline__ bf16x4 rdt(uint32_t lo, uint32_t hi) {
  if constexpr (OFF < 32768)
    return lds_rd_tr<true>(lo, OFF);
  else
    return lds_rd_tr<true>(hi, OFF - 32768);
}

// The group stream of one steady iteration.  Position p in [0, NPOS): H1 = [0, 3 SH1),
// H2 = [3 SH1, NPOS).  kind 0 = O block, 1 = S step; idx = block / step.
#ifndef KP_A4_SAHEAD
#define KP_A4_SAHEAD 1  // groups ahead that an S step's operands are read (1: one S operand slot)
#endif
#ifndef KP_A4_OAHEAD
#define KP_A4_OAHEAD 2  // groups ahead that an O block's operands are read
#endif
static_assert(KP_A4_SAHEAD >= 1 && KP_A4_SAHEAD <= 2 && KP_A4_OAHEAD >= 2 && KP_A4_OAHEAD <= 3, "read-ahead");

template <int DB>
struct Attn4Plan {
  static constexpr int DP = 16 * DB;
  static constexpr int NK = DP / 32, TAIL = (DP % 32) / 16, NS = NK + TAIL;
  static constexpr int SH1 = 5, OH1 = 2 * SH1;
  static constexpr int NS2 = NS - SH1;
  static constexpr int OSM = DB - OH1 - 2 - (NS2 - 1);  // O blocks after the last S step
  static constexpr int NH1 = 3 * SH1;
  static constexpr int NH2 = 2 + 2 * NS2 - 1 + OSM;
  static constexpr int NPOS = NH1 + NH2;
  static_assert(NS2 >= 1 && OSM >= 4, "kp_attn4: plan needs at least 4 O blocks after the last S step");
  static_assert(2 * NK + TAIL == DB, "kp_attn4: 16-dim blocks");
  static constexpr int kind(int p) {
    if (p < NH1) return (p % 3 == 2) ? 1 : 0;
    const int q = p - NH1;
    if (q < 2) return 0;
    if (q < 2 + 2 * NS2 - 1) return ((q - 2) % 2 == 0) ? 1 : 0;
    return 0;
  }
  static constexpr int idx(int p) {
    if (p < NH1) return (p % 3 == 2) ? p / 3 : 2 * (p / 3) + p % 3;
    const int q = p - NH1;
    if (q < 2) return OH1 + q;
    if (q < 2 + 2 * NS2 - 1) return ((q - 2) % 2 == 0) ? SH1 + (q - 2) / 2 : OH1 + 2 + (q - 3) / 2;
    return OH1 + 2 + (NS2 - 1) + (q - (2 + 2 * NS2 - 1));
  }
  // first position of the weights' O blocks (H2's tail)
  static constexpr int SM0 = NH1 + 2 + 2 * NS2 - 1;
  // Read schedule.  Group q (q >= NPOS: the next iteration's group q - NPOS, always an O
  // block) has its 6 operand reads issued during position issue(q) = q - ahead(kind).
  static constexpr int kind_x(int q) { return q < NPOS ? kind(q) : 0; }
  static constexpr int ahead(int q) { return kind_x(q) == 1 ? KP_A4_SAHEAD : KP_A4_OAHEAD; }
  static constexpr int issue(int q) { return q - ahead(q); }
  // groups whose reads are issued during position p, in order (at most 2)
  static constexpr int MAXA = KP_A4_OAHEAD > KP_A4_SAHEAD ? KP_A4_OAHEAD : KP_A4_SAHEAD;
  static constexpr int n_issued(int p) {
    int n = 0;
    for (int q = p + 1; q <= p + MAXA; ++q)
      if (issue(q) == p) ++n;
    return n;
  }
  static constexpr int issued(int p, int i) {
    int n = 0;
    for (int q = p + 1; q <= p + MAXA; ++q)
      if (issue(q) == p) {
        if (n == i) return q;
        ++n;
      }
    return -1;
  }
  // lgkmcnt before group p's MFMAs: reads issued before position p that come after p's
  // own in issue order (those of later groups)
  static constexpr int wait(int p) {
    int n = 0;
    for (int r = p + 1; r <= p + MAXA; ++r)
      if (issue(r) < p && (issue(r) > issue(p) || (issue(r) == issue(p) && r > p))) n += 6;
    return n;
  }
  static_assert(NPOS >= 4, "plan");
};

// O-operand slot of block m (see kp_attn4's operand slots)
template <int DB>
__host__ __device__ constexpr int attn4_oslot(int m) {
  constexpr int R = KP_A4_OAHEAD + 1;  // ring: the block in use plus OAHEAD in flight
  return (m == DB - 1 && DB % R == 1) ? R : m % R;
}

template <int DB>
__global__ __launch_bounds__(256, 1) void kp_attn4(const uint8_t* __restrict__ E4, int n_ent,
                                                   const float* __restrict__ Qpre, int nq, AttnWork wk,
                                                   float* __restrict__ out_m, float* __restrict__ out_l,
                                                   float* __restrict__ out_O, const double* __restrict__ colpre) {
  using PL = Attn4Plan<DB>;
  constexpr int DP = PL::DP, NK = PL::NK, TAIL = PL::TAIL, NS = PL::NS;
  constexpr int KT = 32;
  constexpr int TILE_B = attn4_tile_bytes(DB);
  constexpr int NPC = 3 * DB;  // 1-KiB pieces per tile
  constexpr int OH1 = PL::OH1;
  constexpr int NH1 = PL::NH1, NPOS = PL::NPOS;
  constexpr int P1 = NPC - 3 * OH1;  // H1's pieces (tile t+1, blocks [OH1, DB))
  constexpr int P2 = 3 * OH1;        // H2's pieces (tile t+2, blocks [0, OH1))
  constexpr int K1 = (P1 + 3) / 4, K2 = (P2 + 3) / 4;  // per wave, at most
  extern __shared__ __attribute__((aligned(16))) uint8_t lds4[];  // [2][TILE_B]
  constexpr auto oslot = [](int m) constexpr { return attn4_oslot<DB>(m); };
  static_assert(DB % (KP_A4_OAHEAD + 1) <= 1, "kp_attn4: the O-operand ring needs DB % (OAHEAD + 1) <= 1");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds4;
  int kt_base = 0, key_begin = 0, key_end = 0;
#ifdef KP_ATTN3_STAMPS
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0};
#endif

  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(E4), (short)0, (int)((n_ent + 31) / 32 * TILE_B + 1024), 0x00020000);
  // piece `pc` of the unit's tile `tile` -> LDS buffer `buf`
  auto dma = [&](int tile, int buf, int pc) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds0 + (uint32_t)(buf * TILE_B + 1024 * pc)), 16,
        16 * lane, (kt_base + tile) * TILE_B + 1024 * pc, 0, 0);
  };
  // this wave's k-th piece of H1 (tile t+1, blocks [OH1, DB)) / H2 (tile t+2, blocks [0, OH1)).
  // Branch-free: a wave past the last piece re-issues the half's last piece (the same
  // bytes to the same LDS bytes, which nobody reads during that half), so every wave issues
  // the same number of pieces and the loop body stays one basic block.
  auto dma_h1 = [&](int tile, int k) { dma(tile, tile & 1, min(3 * OH1 + 4 * k + w, NPC - 1)); };
  auto dma_h2 = [&](int tile, int k) { dma(tile, tile & 1, min(4 * k + w, P2 - 1)); };

  const int QT = (nq + 63) / 64;
  const long long total = (long long)QT * wk.ktq;
  long long it = wk.ranges ? 0 : (long long)blockIdx.x * wk.per_wg;
  const long long it_end = wk.ranges ? 0 : min(total, it + (long long)wk.per_wg);
  const int n_units = QT * wk.ranges;
  int unit = ((int)gridDim.x % 8 == 0) ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8)
                                       : (int)blockIdx.x;
  for (;;) {
    int qt, kt0, kt1, part;
    bool fill_rest;
    if (wk.ranges) {
      if (unit >= n_units) break;
      qt = unit % QT;
      part = unit / QT;
      kt0 = (int)((long long)part * wk.ktq / wk.ranges);
      kt1 = (int)((long long)(part + 1) * wk.ktq / wk.ranges);
      fill_rest = false;
      unit += (int)gridDim.x;
    } else {
      if (it >= it_end) break;
      qt = (int)(it / wk.ktq);
      kt0 = (int)(it - (long long)qt * wk.ktq);
      kt1 = (int)min((long long)wk.ktq, (long long)kt0 + (it_end - it));
      part = (int)blockIdx.x - (int)(((long long)qt * wk.ktq) / wk.per_wg);
      fill_rest = kt1 == wk.ktq;
      it += kt1 - kt0;
    }
    kt_base = kt0;
    key_begin = kt0 * KT;
    key_end = min(n_ent, kt1 * KT);
    const int ntiles = kt1 - kt0;
    const int q = qt * 64 + 16 * w + c;
    const bool valid = q < nq;
    // ---- query pieces -> VGPRs: B operand of S step s is q[32 s + 8 g + j]
    bf16x8 qb[NK][3];
    bf16x4 qt4[3];
    {
      const float* qp = Qpre + (size_t)(valid ? q : 0) * DP;
#pragma unroll
      for (int s = 0; s < NK; ++s) {
        const float4 v0 = *reinterpret_cast<const float4*>(qp + 32 * s + 8 * g);
        const float4 v1 = *reinterpret_cast<const float4*>(qp + 32 * s + 8 * g + 4);
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 h, m, l;
          split3(valid ? f[j] : 0.f, h, m, l);
          qb[s][0][j] = h;
          qb[s][1][j] = m;
          qb[s][2][j] = l;
        }
      }
      if (TAIL) {
        const float4 v0 = *reinterpret_cast<const float4*>(qp + 32 * NK + 4 * g);
        const float f[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 h, m, l;
          split3(valid ? f[j] : 0.f, h, m, l);
          qt4[0][j] = h;
          qt4[1][j] = m;
          qt4[2][j] = l;
        }
      }
    }
    f32x4 O[DB];
    float m_ref = kNegInf, l_run = 0.f, m_seen = kNegInf, csh = 0.f;

    // per-lane LDS bases of a buffer (lo / lo + 32 KiB)
    auto sbase = [&](int buf) { return lds0 + (uint32_t)(buf * TILE_B + (g >> 1) * 3072 + c * 32 + (g & 1) * 16); };
    auto tbase = [&](int buf) { return lds0 + (uint32_t)(buf * TILE_B + c * 32 + 8 * g); };
    auto obase = [&](int buf) { return lds0 + (uint32_t)(buf * TILE_B + (4 * g + (c >> 2)) * 32 + 8 * (c & 3)); };

    // operand slots: S reads by step parity, O reads by oslot(block) -- a ring of three
    // (reads run two groups ahead) plus a fourth for the last block when DB % 3 == 1, so
    // the ring continues into the next tile's blocks 0 and 1 (read during blocks DB-2, DB-1)
    constexpr int NSS = KP_A4_SAHEAD;  // S operand slots
    bf16x8 sa[NSS][2][3];  // [slot][sub-tile][piece]
    bf16x4 ta[2][3];     // tail step
    bf16x4 ol[KP_A4_OAHEAD + 2][3], oh[KP_A4_OAHEAD + 2][3];
    // reads of S step J (6) from the buffer at bases (lo, hi)
    auto read_s = [&](auto J, uint32_t lo, uint32_t hi, uint32_t tlo, uint32_t thi) {
      constexpr int j = decltype(J)::value;
      if constexpr (j < NK) {
        static_for<0, 6>([&](auto K) {
          constexpr int k = decltype(K)::value, u = k & 1, p = k >> 1;
          sa[j % NSS][u][p] = rd8<(2 * j * 3 + p) * 1024 + u * 512>(lo, hi);
        });
      } else {
        static_for<0, 6>([&](auto K) {
          constexpr int k = decltype(K)::value, u = k & 1, p = k >> 1;
          ta[u][p] = rd4<(2 * NK * 3 + p) * 1024 + u * 512>(tlo, thi);
        });
      }
    };
    // one read (k of 6) of S step J, for spreading over MFMA gaps
    auto read_s1 = [&](auto J, auto K, uint32_t lo, uint32_t hi, uint32_t tlo, uint32_t thi) {
      constexpr int j = decltype(J)::value, k = decltype(K)::value, u = k & 1, p = k >> 1;
      if constexpr (j < NK)
        sa[j % NSS][u][p] = rd8<(2 * j * 3 + p) * 1024 + u * 512>(lo, hi);
      else
        ta[u][p] = rd4<(2 * NK * 3 + p) * 1024 + u * 512>(tlo, thi);
    };
    auto read_o1 = [&](auto M, auto K, uint32_t lo, uint32_t hi) {
      constexpr int m = decltype(M)::value, k = decltype(K)::value, p = k >> 1;
      if constexpr (k & 1)
        oh[oslot(m)][p] = rdt<(3 * m + p) * 1024 + 512>(lo, hi);
      else
        ol[oslot(m)][p] = rdt<(3 * m + p) * 1024>(lo, hi);
    };
    f32x4 sc[2];
    // the twelve MFMAs of S step J (sub-tiles alternating, mfma3's product order), with
    // callback after(k) after MFMA k
    auto mfma_s = [&](auto J, auto&& after) {
      constexpr int j = decltype(J)::value;
      static_for<0, 12>([&](auto K) {
        constexpr int k = decltype(K)::value, u = k & 1, pr = k >> 1;
        if constexpr (j < NK)
          sc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa[j % NSS][u][kPA[pr]], qb[j < NK ? j : 0][kPB[pr]], sc[u],
                                                          0, 0, 0);
        else
          sc[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, ta[u][kPA[pr]]),
                                                            __builtin_bit_cast(s16x4, qt4[kPB[pr]]), sc[u], 0, 0, 0);
        after(K);
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    bf16x8 pb[3], pbn[3];
    auto mfma_o = [&](auto M, auto&& after) {
      constexpr int m = decltype(M)::value;
      bf16x8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const bf16x4 x = ol[oslot(m)][p], y = oh[oslot(m)][p];
        a[p] = (bf16x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      }
      static_for<0, 6>([&](auto K) {
        constexpr int k = decltype(K)::value;
        O[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kPA[k]], pb[kPB[k]], O[m], 0, 0, 0);
        after(K);
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    // weights of a tile whose S accumulators are in sc: element jj = (u, r) = entity
    // 16 u + 4 g + r; pw = exp(s - m_ref) - csh (centred), summed into l, split into pbn
    float lt = 0.f;
    auto weight1 = [&](int k0, auto JJ) {
      constexpr int jj = decltype(JJ)::value, u = jj >> 2, r = jj & 3;
      // branch-free (selects, no exec-masked region inside the MFMA stream)
      const bool ok = k0 + 16 * u + 4 * g + r < key_end;
      const float s = sc[u][r];
      m_seen = fmaxf(m_seen, ok ? s : kNegInf);
      const float e = __expf((ok ? s : m_ref) - m_ref);
      const float pw = ok ? __fsub_rn(e, csh) : 0.f;
      lt += pw;
      __bf16 h, mm, l;
      split3(pw, h, mm, l);
      pbn[0][jj] = h;
      pbn[1][jj] = mm;
      pbn[2][jj] = l;
    };

    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < DB; ++j) O[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      l_run = 0.f;
      m_seen = kNegInf;
      // ---- prologue: tile 0 whole into buf 0, tile 1's blocks [0, OH1) into buf 1
      for (int k = 0; k < (NPC + 3) / 4; ++k)
        if (4 * k + w < NPC) dma(0, 0, 4 * k + w);
      if (ntiles > 1)
        for (int k = 0; k < K2; ++k) dma_h2(1, k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      {
        // S(0), one step of reads ahead
        const uint32_t lo = sbase(0), hi = lo + 32768, tlo = tbase(0), thi = tlo + 32768;
        sc[0] = sc[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (NSS >= 2) {
          read_s(std::integral_constant<int, 0>{}, lo, hi, tlo, thi);
          static_for<0, NS>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if constexpr (j + 1 < NS) {
              read_s(std::integral_constant<int, j + 1>{}, lo, hi, tlo, thi);
              lgkm_wait<6>();
            } else {
              lgkm_wait<0>();
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_s(J, [](auto) {});
          });
        } else {
          // one S slot: step j + 1's reads ride in step j's MFMA gaps (after its operands
          // are in registers: the A pieces are copied into the MFMA operands first)
          read_s(std::integral_constant<int, 0>{}, lo, hi, tlo, thi);
          static_for<0, NS>([&](auto J) {
            constexpr int j = decltype(J)::value;
            lgkm_wait<0>();
            __builtin_amdgcn_sched_barrier(0);
            mfma_s(J, [](auto) {});
            if constexpr (j + 1 < NS) read_s(std::integral_constant<int, j + 1>{}, lo, hi, tlo, thi);
          });
        }
        // weights of tile 0: the reference max (pass 0) and the centring shift
        if (pass == 0) {
          float tmax = kNegInf;
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (key_begin + 16 * u + 4 * g + r < key_end) tmax = fmaxf(tmax, sc[u][r]);
          float mq = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
          m_ref = fmaxf(mq, __shfl_xor(mq, 32, 64));
        }
        float mn = kPosInf;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (key_begin + 16 * u + 4 * g + r < key_end) mn = fminf(mn, __expf(sc[u][r] - m_ref));
        mn = fminf(mn, __shfl_xor(mn, 16, 64));
        mn = fminf(mn, __shfl_xor(mn, 32, 64));
        csh = (mn < kPosInf) ? mn : 0.f;
        lt = 0.f;
        static_for<0, 8>([&](auto JJ) { weight1(key_begin, JJ); });
        l_run += lt;
#pragma unroll
        for (int p = 0; p < 3; ++p) pb[p] = pbn[p];
        // the first OAHEAD groups' reads (O blocks of tile 0)
        const uint32_t olo = obase(0), ohi = olo + 32768;
        static_for<0, KP_A4_OAHEAD>([&](auto M) {
          static_for<0, 6>([&](auto K) { read_o1(M, K, olo, ohi); });
        });
      }

      // ---- steady iterations: O(t) with S(t+1)
#ifdef KP_ATTN3_STAMPS
      // diagnostic build: [H1 groups, mid barrier, H2 groups, end barrier, iterations]
      unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, st4 = 0;
#endif
      for (int t = 0; t + 1 < ntiles; ++t) {
        KP3_STAMP(st0);
        const int bo = t & 1, bs = bo ^ 1;
        const uint32_t olo = obase(bo), ohi = olo + 32768;
        const uint32_t slo = sbase(bs), shi = slo + 32768, tlo = tbase(bs), thi = tlo + 32768;
        // next iteration's O reads come from buffer bs (tile t+1)
        const uint32_t nlo = obase(bs), nhi = nlo + 32768;
        // tile t+2's first part: past the unit's last tile this loads whatever follows it in
        // the image (zeros past its end: buffer loads out of range return 0) into blocks
        // that nobody reads again in this unit
        const int k1 = key_begin + (t + 1) * KT;
        sc[0] = sc[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        lt = 0.f;
        static_for<0, NPOS>([&](auto P) {
          constexpr int p = decltype(P)::value;
          constexpr int kind = PL::kind(p), ix = PL::idx(p);
          if constexpr (p == NH1) {
            // mid barrier: this half's DMA (tile t+1, blocks [OH1, DB)) has landed everywhere,
            // and every wave is past O(t) blocks [0, OH1)
            KP3_STAMP(st1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            KP3_STAMP(st2);
          }
          lgkm_wait<PL::wait(p)>();
          __builtin_amdgcn_sched_barrier(0);
          // DMA pieces of this position: KP_A4_DMA_PER_GROUP per group from the start of each
          // half, so the last piece has most of the half to land before the barrier that
          // waits for it (spread evenly over the half, the last pieces' fetch latency was
          // exposed at the barriers)
#ifdef KP_A4_NODMA
          if constexpr (false) {
#else
          if constexpr (p < NH1) {
#endif
#pragma unroll
            for (int k = 0; k < K1; ++k)
              if (k / KP_A4_DMA_PER_GROUP == p) dma_h1(t + 1, k);
          } else if constexpr (p >= NH1
#ifdef KP_A4_NODMA
                               && false
#endif
          ) {
#pragma unroll
            for (int k = 0; k < K2; ++k)
              if (k / KP_A4_DMA_PER_GROUP == p - NH1) dma_h2(t + 2, k);
          }
          __builtin_amdgcn_sched_barrier(0);
          // read r (0 .. 6 n_issued - 1) of the groups whose operands are read during p (the
          // next iteration's first O blocks at the end of the stream)
          constexpr int NR = 6 * PL::n_issued(p);
          auto rd_next = [&](auto R) {
            constexpr int r = decltype(R)::value;
#ifdef KP_A4_NOREAD
            return;
#endif
            if constexpr (r < NR) {
              constexpr int q = PL::issued(p, r / 6);
              constexpr auto K = std::integral_constant<int, r % 6>{};
              if constexpr (q < NPOS) {
                constexpr int kn = PL::kind(q), in = PL::idx(q);
                if constexpr (kn == 1)
                  read_s1(std::integral_constant<int, in>{}, K, slo, shi, tlo, thi);
                else
                  read_o1(std::integral_constant<int, in>{}, K, olo, ohi);
              } else {
                read_o1(std::integral_constant<int, q - NPOS>{}, K, nlo, nhi);
              }
            }
          };
          if constexpr (kind == 1) {
            // 12 MFMAs: one read after each of the first NR
            mfma_s(std::integral_constant<int, ix>{}, [&](auto K) { rd_next(K); });
          } else {
            // 6 MFMAs: NR / 6 reads after each
            mfma_o(std::integral_constant<int, ix>{}, [&](auto K) {
              constexpr int k = decltype(K)::value;
              if constexpr (NR > 6) {
                rd_next(std::integral_constant<int, 2 * k>{});
                rd_next(std::integral_constant<int, 2 * k + 1>{});
              } else {
                rd_next(K);
              }
              // the weights of tile t+1 in the issue gaps of the last O blocks
              if constexpr (p >= PL::SM0) {
                constexpr int slot = (p - PL::SM0) * 6 + k;  // 0 .. 6 OSM - 1
#ifndef KP_A4_NOSM
                if constexpr (slot % 3 == 1 && slot / 3 < 8) weight1(k1, std::integral_constant<int, slot / 3>{});
#endif
              }
            });
          }
        });
        l_run += lt;
        KP3_STAMP(st3);
        // end barrier: tile t+2's first part has landed; every wave is done with buffer bo
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        KP3_STAMP(st4);
#ifdef KP_ATTN3_STAMPS
        st_acc[0] += st1 - st0;
        st_acc[1] += st2 - st1;
        st_acc[2] += st3 - st2;
        st_acc[3] += st4 - st3;
        st_acc[4] += 1;
#endif
#pragma unroll
        for (int p = 0; p < 3; ++p) pb[p] = pbn[p];
      }

      // ---- the last tile: O only (its reads of blocks 0 and 1 are in flight)
      {
        const int bo = (ntiles - 1) & 1;
        const uint32_t olo = obase(bo), ohi = olo + 32768;
        static_for<0, DB>([&](auto M) {
          constexpr int m = decltype(M)::value;
          // in flight: blocks m .. min(m + OAHEAD - 1, DB - 1)
          constexpr int later = (m + KP_A4_OAHEAD - 1 < DB ? KP_A4_OAHEAD - 1 : DB - 1 - m);
          lgkm_wait<6 * later>();
          __builtin_amdgcn_sched_barrier(0);
          mfma_o(M, [&](auto K) {
            if constexpr (m + KP_A4_OAHEAD < DB)
              read_o1(std::integral_constant<int, m + KP_A4_OAHEAD>{}, K, olo, ohi);
          });
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      float mq = fmaxf(m_seen, __shfl_xor(m_seen, 16, 64));
      mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
      if (pass == 1 || !__syncthreads_or(mq > m_ref + kMargin)) break;
      m_ref = mq;
    }

    float l_tot = l_run + __shfl_xor(l_run, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (ntiles > 0) {
      l_tot = __fmaf_rn(csh, (float)(key_end - key_begin), l_tot);
      const double* p0 = colpre + (size_t)kt0 * DP;
      const double* p1 = colpre + (size_t)kt1 * DP;
#pragma unroll
      for (int m = 0; m < DB; ++m) {
        const int d = 16 * m + 4 * g;
        const double2 a0 = *reinterpret_cast<const double2*>(p0 + d), a1 = *reinterpret_cast<const double2*>(p0 + d + 2);
        const double2 b0 = *reinterpret_cast<const double2*>(p1 + d), b1 = *reinterpret_cast<const double2*>(p1 + d + 2);
        O[m][0] = __fmaf_rn(csh, (float)(b0.x - a0.x), O[m][0]);
        O[m][1] = __fmaf_rn(csh, (float)(b0.y - a0.y), O[m][1]);
        O[m][2] = __fmaf_rn(csh, (float)(b1.x - a1.x), O[m][2]);
        O[m][3] = __fmaf_rn(csh, (float)(b1.y - a1.y), O[m][3]);
      }
    }
    if (valid) {
      const size_t o = (size_t)part * nq + q;
      if (g == 0) {
        out_m[o] = m_ref;
        out_l[o] = l_tot;
      }
      float* dst = out_O + o * DP;
#pragma unroll
      for (int m = 0; m < DB; ++m)
        *reinterpret_cast<float4*>(dst + 16 * m + 4 * g) = make_float4(O[m][0], O[m][1], O[m][2], O[m][3]);
    }
    if (fill_rest && valid) {
      for (int pp = part + 1; pp < wk.n_parts; ++pp) {
        const size_t o = (size_t)pp * nq + q;
        if (g == 0) {
          out_m[o] = kNegInf;
          out_l[o] = 0.f;
        }
        float* dst = out_O + o * DP;
        for (int d = 4 * g; d < DP; d += 16) *reinterpret_cast<float4*>(dst + d) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
#ifdef KP_ATTN3_STAMPS
  if (lane == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&g_attn3_stamps[i], st_acc[i]);
#endif
}

// (diagnostic stamps flushed at the end of kp_attn4, see below)
// Host: the blocked split image of c->dE, built once per context.
template <int DB>
const uint8_t* split3_blocked_image(kp_ctx* c) {
  constexpr int DP = 16 * DB;
  KP_REQUIRE(c->dp == DP, "attn4: table stride mismatch");
  if (!c->e4_ready) {
    const size_t n_tiles = (size_t)(c->n_ent + 31) / 32;
    const size_t bytes = n_tiles * attn4_tile_bytes(DB) + 1024;
    uint8_t* d = reinterpret_cast<uint8_t*>(c->e4.ensure(bytes));
    KP_HIP(hipMemsetAsync(d, 0, bytes, c->stream));
    const long long n = (long long)c->n_ent * (DP / 2);
    hipLaunchKernelGGL((kp_split3_blocked<DP>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->dE,
                       c->n_ent, d);
    KP_HIP(hipGetLastError());
    c->e4_ready = true;
  }
  return c->e4.as<uint8_t>();
}

template <int DB>
void launch_attn4(kp_ctx* c, int n_ent, const float* Q, int nq, const AttnPlan& plan, float* m, float* l, float* O) {
  KP_REQUIRE(n_ent == c->n_ent, "attn4: key count differs from the table's (tile prefix sums)");
  KP_REQUIRE((long long)(n_ent + 31) / 32 * attn4_tile_bytes(DB) + 1024 < (1LL << 31),
             "attn4: table too large for the 32-bit buffer descriptor of the blocked image");
  const uint8_t* E4 = split3_blocked_image<DB>(c);
  const double* pre = tile_prefix<DB>(c);
  hipLaunchKernelGGL((kp_attn4<DB>), dim3(plan.n_wg), dim3(256), attn4_lds_bytes(DB), c->stream, E4, n_ent, Q, nq,
                     plan.wk, m, l, O, pre);
  KP_HIP(hipGetLastError());
}

}  // namespace kpattn
