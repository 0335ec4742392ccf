// kp_attn5.hpp -- kp_attn3 for the ComplEx D = 400 rows with the dimensions split over a
// wave pair, so that two waves share each SIMD.
//
// kp_attn3<25> holds, per wave, the three bf16 pieces of its 16 queries over all 400
// dimensions (150 VGPRs) and their 400-dimension O accumulators (100): with its operand
// buffers ~448 registers, one wave per SIMD, and per tile the S MFMAs, the softmax and
// split of P, and the O MFMAs form one dependent chain that nothing else fills (MFMA busy
// 0.62, SQ_WAIT_INST_ANY 44 %: DESIGN.md section 5).  Here a workgroup is 8 waves: wave
// w and its partner w ^ 4 take the same 16 queries (pair w & 3), half 0 the dimensions
// of k-steps 0..5 plus the 16-deep tail (dims 0..191, 384..399) in the S phase and O
// blocks 0..11 (dims 0..191), half 1 k-steps 6..11 (dims 192..383) and O blocks 12..24
// (dims 192..399): 150 MFMAs per wave per tile either way, and about half the registers,
// so two waves per SIMD.
//
// Per 32-entity tile (both sub-tiles u = 0, 1 of 16 entities):
//   1. S: each wave's partial S^T of both sub-tiles over its dimensions (ILV schedule of
//      kp_attn3: reads two k-steps ahead in the MFMA issue gaps, sched_barrier pinned);
//   2. exchange: half h owns sub-tile h; it writes its partial of sub-tile 1 - h to its
//      LDS slot, and after a barrier adds the partner's partial of sub-tile h;
//   3. softmax of its own sub-tile (the first tile of a pass exchanges the column max and
//      min: m_ref and the centring shift csh = e^{min - m_ref} = the smallest weight);
//   4. exchange: its sub-tile's weights into the partner's slot (the slot it just read),
//      a barrier, the partner's from its own slot; P of the whole tile split into
//      pieces as kp_attn3 does;
//   5. O over its dimensions (ILV reads two blocks ahead), one LDS-DMA piece of the next
//      tile per O block; vmcnt(0) and the tile barrier.
// The table image, the tile DMA (buffer descriptor, scalar offsets), the work partition,
// the fixed reference max with the kMargin rerun, the centred accumulation with its fp64
// prefix-sum correction and the outputs are kp_attn3's.  Results agree with kp_attn3 to
// fp32 rounding (S is the sum of two half-dimension MFMA chains), not bitwise.
#pragma once
#include "kp_attn3.hpp"

namespace kpattn {

constexpr int A5_DP = 400;
constexpr int A5_ROW_B = split3_row_bytes(A5_DP);  // 2,400 B (odd number of 16-dim blocks: no pad)
constexpr int A5_PIECES = split3_pieces(A5_DP);    // 75 whole 1-KiB pieces per tile
constexpr int A5_BUF_B = 1024 * A5_PIECES;         // 76,800 B per tile buffer
constexpr int A5_X_OFF = 2 * A5_BUF_B;             // exchange slots: 8 waves x 1 KiB
constexpr int A5_XS_OFF = A5_X_OFF + 8 * 1024;     // per-wave column scalars: 8 x 32 floats
constexpr size_t attn5_lds_bytes() { return (size_t)A5_XS_OFF + 8 * 32 * sizeof(float); }
static_assert(attn5_lds_bytes() <= 160 * 1024, "kp_attn5: LDS over the 160 KiB of a CU");
static_assert(split3_tile_bytes(A5_DP) == A5_BUF_B, "kp_attn5: a tile is a whole number of DMA pieces");

template <int H, int G, int MODE>
__device__ __forceinline__ void attn5_half(const uint8_t* __restrict__ E3, int n_ent, const float* __restrict__ Qpre,
                                           int nq, const AttnWork& wk, float* __restrict__ out_m,
                                           float* __restrict__ out_l, float* __restrict__ out_O,
                                           const double* __restrict__ colpre, int w, int lane, uint32_t lds0,
                                           float* __restrict__ xf) {
  static_assert(MODE != ATT_BCE_O, "kp_attn5: the ComplEx softmax modes only");
  constexpr bool WITH_O = MODE != ATT_SOFTMAX;
  constexpr int DP = A5_DP, KT = 32, NK = DP / 32;  // 12 full k-steps + a 16-deep tail
  constexpr int NSF = 6;                            // full k-steps of this half
  constexpr int KS0 = H ? 6 : 0;                    // its first full k-step
  constexpr int TL = H ? 0 : 1;                     // the tail k-step (dims 384..399): half 0
  constexpr int LAST = NSF + TL - 1;                // index of this half's last S step
  constexpr int MB0 = H ? 12 : 0, NB = H ? 13 : 12;  // O blocks [MB0, MB0 + NB)
  constexpr int ROW_B = A5_ROW_B, PART_B = 2 * DP, BUF_B = A5_BUF_B;
  constexpr uint32_t SUB_B = 16u * ROW_B;           // the second sub-tile's rows
  static_assert(SUB_B + 3 * PART_B + 64 * NK < 65536, "LDS read offsets exceed the 16-bit offset field");
  const int g = lane >> 4, c = lane & 15;
  const int pr = w >> 1;   // the pair: queries 16 pr .. 16 pr + 15 of the query tile
  const int wp = w ^ 1;    // the partner wave (the other half)
  // exchange slots (floats): slot[w] = lanes x 4; column scalars xs[w][32]
  float* my_slot = xf + w * 256 + 4 * lane;
  float* pa_slot = xf + wp * 256 + 4 * lane;
  float* my_xs = xf + 8 * 256 + w * 32;
  const float* pa_xs = xf + 8 * 256 + wp * 32;
  int key_begin = 0, key_end = 0;

  // the next tile's LDS-DMA: wave w copies pieces w, w + 8, ... (10 pieces for w < 3, else
  // 9), one per O block (ATT_SOFTMAX: a burst after the S exchange)
  const __amdgpu_buffer_rsrc_t e3rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(E3), (short)0, (int)((n_ent + 31) / 32 * 32 * ROW_B + 1024), 0x00020000);
  const int npw = (A5_PIECES - w + 7) / 8;  // wave-uniform
  auto bdma = [&](int tile, int buf, int k) {
    const int p = w + 8 * k;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        e3rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds0 + (uint32_t)(buf * BUF_B + 1024 * p)), 16,
        16 * lane, (key_begin + tile * KT) * ROW_B + 1024 * p, 0, 0);
  };
  auto issue = [&](int tile, int buf) {
    for (int k = 0; k < npw; ++k) bdma(tile, buf, k);
  };

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
    key_begin = kt0 * KT;
    key_end = min(n_ent, kt1 * KT);
    const int ntiles = kt1 - kt0;
    const int q = qt * 64 + 16 * pr + c;
    const bool valid = q < nq;
    // ---- this half's query pieces -> VGPRs: B operand of local step s is q[32 (KS0 + s) + 8 g + j]
    bf16x8 qb[NSF][3];
    bf16x4 qt4[3];
    {
      const float* qp = Qpre + (size_t)(valid ? q : 0) * DP;
#pragma unroll
      for (int s = 0; s < NSF; ++s) {
        const float4 v0 = *reinterpret_cast<const float4*>(qp + 32 * (KS0 + s) + 8 * g);
        const float4 v1 = *reinterpret_cast<const float4*>(qp + 32 * (KS0 + s) + 8 * g + 4);
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
      if (TL) {
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
    f32x4 O[WITH_O ? NB : 1];
    float m_ref = kNegInf, l_run = 0.f;
    float csh = 0.f;

    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < (WITH_O ? NB : 1); ++j) O[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      l_run = 0.f;
      float m_seen = kNegInf;
      if (ntiles > 0) issue(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();

      // per-tile state carried from one phase (interval) to the next
      f32x4 sc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
      bf16x8 pb[3];
      bf16x4 ol[3][3], oh[3][3];
      auto tile_base = [&](int t) { return lds0 + (uint32_t)((t & 1) * BUF_B); };
      auto o_base = [&](int t) { return tile_base(t) + (uint32_t)((4 * g + (c >> 2)) * ROW_B + 8 * (c & 3)); };
      auto read_o = [&](uint32_t ob, int m, int k) {  // read k of local block m (piece k / 2, rows 4g / 16 + 4g)
        const int mm = MB0 + m, pp = k >> 1;
        if (k & 1)
          oh[m % 3][pp] = lds_rd_tr<true>(ob, 16 * ROW_B + pp * PART_B + 32 * mm);
        else
          ol[m % 3][pp] = lds_rd_tr<true>(ob, pp * PART_B + 32 * mm);
      };
      // ---- S: partial S^T of both sub-tiles over this half's dimensions, then the
      // partial of the sub-tile the partner keeps into this wave's slot
      auto phase_s = [&](int t) {
        sc[0] = sc[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const uint32_t rb = tile_base(t) + (uint32_t)(c * ROW_B + 16 * g);
        const uint32_t rbt = rb - 8u * g;  // tail reads: 8 bytes per lane group
        bf16x8 ra[3][2][3];
        bf16x4 rt[2][3];
        auto read_k = [&](int s, int k) {  // read k (sub-tile k % 2, piece k / 2) of local step s
          const int uu = k & 1, pp = k >> 1;
          if (s < NSF)
            ra[s % 3][uu][pp] = lds_rd_bf8<true>(rb, (int)(uu * SUB_B) + pp * PART_B + 64 * (KS0 + s));
          else
            rt[uu][pp] = lds_rd_bf4<true>(rbt, (int)(uu * SUB_B) + pp * PART_B + 64 * NK);
        };
#pragma unroll
        for (int k = 0; k < 6; ++k) read_k(0, k);
        if (LAST >= 1)
#pragma unroll
          for (int k = 0; k < 6; ++k) read_k(1, k);
#pragma unroll
        for (int s = 0; s <= LAST; ++s) {
          if (s < LAST)
            lgkm_wait<6>();
          else
            lgkm_wait<0>();
          __builtin_amdgcn_sched_barrier(0);
          const int b = s % 3;
#pragma unroll
          for (int k = 0; k < 6; ++k) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              if (s < NSF)
                sc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[b][u][kPA[k]], qb[s < NSF ? s : 0][kPB[k]], sc[u],
                                                                0, 0, 0);
              else
                sc[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, rt[u][kPA[k]]),
                                                                  __builtin_bit_cast(s16x4, qt4[kPB[k]]), sc[u], 0, 0,
                                                                  0);
              if (u == 0 && s + 2 <= LAST) read_k(s + 2, k);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        *reinterpret_cast<f32x4*>(my_slot) = sc[1 - H];
      };
      // ---- softmax of sub-tile H (this half's): the partner's partial added, the next
      // tile's LDS-DMA issued (its buffer was released by the lagging group's O phase of
      // tile t - 1, the interval before), the weights into the partner's slot, and the O
      // phase's first two blocks read ahead.  The first tile of a pass exchanges the
      // column max and min (a barrier inside the interval; the other group meets it)
      auto phase_soft = [&](int t) {
        f32x4 S = sc[H];
        {
          const f32x4 v = *reinterpret_cast<const f32x4*>(pa_slot);
          S += v;
        }
        if (t + 1 < ntiles) issue(t + 1, (t + 1) & 1);
        const int e0 = key_begin + t * KT + 16 * H + 4 * g;  // entity e0 + r for query c
        float v[4];
        float tmax = kNegInf, tmin = kPosInf;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool in = e0 + r < key_end;
          v[r] = in ? S[r] : kNegInf;
          tmax = fmaxf(tmax, v[r]);
          tmin = in ? fminf(tmin, S[r]) : tmin;
        }
        m_seen = fmaxf(m_seen, tmax);
        if (t == 0) {
          // the pass's reference max (pass 0) and its centring shift, the smallest weight
          // e^{min - m_ref}, over both sub-tiles of the first tile
          float mq = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
          mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
          float mn = fminf(tmin, __shfl_xor(tmin, 16, 64));
          mn = fminf(mn, __shfl_xor(mn, 32, 64));
          if (g == 0) {
            my_xs[c] = mq;
            my_xs[16 + c] = mn;
          }
          __syncthreads();
          mq = fmaxf(mq, pa_xs[c]);
          mn = fminf(mn, pa_xs[16 + c]);
          if (pass == 0) m_ref = mq;
          csh = (mn < kPosInf) ? __expf(mn - m_ref) : 0.f;
        }
        float pw[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[r] = (e0 + r < key_end) ? __fsub_rn(__expf(v[r] - m_ref), csh) : 0.f;
        l_run += (pw[0] + pw[1]) + (pw[2] + pw[3]);
        if (WITH_O) {
          *reinterpret_cast<f32x4*>(pa_slot) = (f32x4){pw[0], pw[1], pw[2], pw[3]};
          // P pieces of this half's sub-tile in the B layout (element j of lane group g:
          // entity 4 g + j of sub-tile 0 for j < 4, 4 g + j - 4 of sub-tile 1)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            __bf16 h, m, l;
            split3(pw[r], h, m, l);
            pb[0][4 * H + r] = h;
            pb[1][4 * H + r] = m;
            pb[2][4 * H + r] = l;
          }
          const uint32_t ob = o_base(t);
#pragma unroll
          for (int k = 0; k < 6; ++k) read_o(ob, 0, k);
#pragma unroll
          for (int k = 0; k < 6; ++k) read_o(ob, 1, k);
        }
      };
      // ---- the partner's weights, then O^T += E^T . P over this half's blocks; block
      // m + 2's reads ride in block m's MFMA issue gaps
      auto phase_o = [&](int t) {
        if (!WITH_O) return;
        {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(my_slot);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            __bf16 h, m, l;
            split3(pv[r], h, m, l);
            pb[0][4 * (1 - H) + r] = h;
            pb[1][4 * (1 - H) + r] = m;
            pb[2][4 * (1 - H) + r] = l;
          }
        }
        const uint32_t ob = o_base(t);
#pragma unroll
        for (int m = 0; m < NB; ++m) {
          if (m + 1 < NB)
            lgkm_wait<6>();
          else
            lgkm_wait<0>();
          __builtin_amdgcn_sched_barrier(0);
          bf16x8 a[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const bf16x4 x = ol[m % 3][p], y = oh[m % 3][p];
            a[p] = (bf16x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
          }
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            O[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kPA[k]], pb[kPB[k]], O[m], 0, 0, 0);
            if (m + 2 < NB) read_o(ob, m + 2, k);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      };
      // Intervals between workgroup barriers, 3 per tile: group 0 runs S_t | softmax_t |
      // O_t, group 1 one interval later (O_{t-1} | S_t | softmax_t), so on every SIMD one
      // wave's softmax sits beside the other's MFMAs.  Both groups pass the same barriers:
      // 3 per tile, 2 more on the first tile (the max / min exchange), 1 for the lag.
      // The next tile's copies, issued in the softmax intervals, land before the barrier
      // that closes each tile's third interval.
      if (G == 0) {
        for (int t = 0; t < ntiles; ++t) {
          phase_s(t);
          __syncthreads();
          phase_soft(t);
          __syncthreads();
          if (t == 0) __syncthreads();  // group 1's max / min exchange
          phase_o(t);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
        }
        __syncthreads();  // group 1's last O phase
      } else {
        __syncthreads();  // group 0's first S phase
        for (int t = 0; t < ntiles; ++t) {
          if (t == 0) __syncthreads();  // group 0's max / min exchange
          phase_s(t);
          __syncthreads();
          phase_soft(t);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          phase_o(t);
          __syncthreads();
        }
      }
      float mq = fmaxf(m_seen, __shfl_xor(m_seen, 16, 64));
      mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
      if (pass == 1 || !__syncthreads_or(mq > m_ref + kMargin)) break;
      // rerun with the exact max of both halves
      if (g == 0) my_xs[c] = mq;
      __syncthreads();
      m_ref = fmaxf(mq, pa_xs[c]);
      __syncthreads();
    }

    // the column sums of the weights over both halves (half 0's + half 1's on both)
    float l_tot = l_run + __shfl_xor(l_run, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (g == 0) my_xs[c] = l_tot;
    __syncthreads();
    {
      const float lp = pa_xs[c];
      l_tot = H == 0 ? l_tot + lp : lp + l_tot;
    }
    if (ntiles > 0) {
      // the shifted-out part: csh * (number of keys) and csh * (sum of the keys' rows),
      // the latter from the fp64 prefix sums of the table over tiles
      l_tot = __fmaf_rn(csh, (float)(key_end - key_begin), l_tot);
      if (WITH_O) {
        const double* p0 = colpre + (size_t)kt0 * DP;
        const double* p1 = colpre + (size_t)kt1 * DP;
#pragma unroll
        for (int m = 0; m < NB; ++m) {
          const int d = 16 * (MB0 + m) + 4 * g;  // 32-byte aligned quad of dims
          const double2 a0 = *reinterpret_cast<const double2*>(p0 + d), a1 = *reinterpret_cast<const double2*>(p0 + d + 2);
          const double2 b0 = *reinterpret_cast<const double2*>(p1 + d), b1 = *reinterpret_cast<const double2*>(p1 + d + 2);
          O[m][0] = __fmaf_rn(csh, (float)(b0.x - a0.x), O[m][0]);
          O[m][1] = __fmaf_rn(csh, (float)(b0.y - a0.y), O[m][1]);
          O[m][2] = __fmaf_rn(csh, (float)(b1.x - a1.x), O[m][2]);
          O[m][3] = __fmaf_rn(csh, (float)(b1.y - a1.y), O[m][3]);
        }
      }
    }
    if (valid) {
      const size_t o = (size_t)part * nq + q;
      if (H == 0 && g == 0) {
        out_m[o] = m_ref;
        out_l[o] = l_tot;
      }
      if (WITH_O) {
        // O^T block m: lane (g, c) holds dims 16 m + 4 g + r of query c
        float* dst = out_O + o * DP;
#pragma unroll
        for (int m = 0; m < NB; ++m)
          *reinterpret_cast<float4*>(dst + 16 * (MB0 + m) + 4 * g) = make_float4(O[m][0], O[m][1], O[m][2], O[m][3]);
      }
    }
    if (fill_rest && valid) {
      for (int pp = part + 1; pp < wk.n_parts; ++pp) {
        const size_t o = (size_t)pp * nq + q;
        if (H == 0 && g == 0) {
          out_m[o] = kNegInf;
          out_l[o] = 0.f;
        }
        if (WITH_O) {
          float* dst = out_O + o * DP;
          for (int m = 0; m < NB; ++m)
            *reinterpret_cast<float4*>(dst + 16 * (MB0 + m) + 4 * g) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }
}

// 8 waves: pairs (w, w ^ 1), even w the first half of the dimensions; waves 4..7 (the
// second group, sharing the SIMDs of waves 0..3) one interval behind
template <int MODE>
__global__ __launch_bounds__(512, 1) void kp_attn5(const uint8_t* __restrict__ E3, int n_ent,
                                                   const float* __restrict__ Qpre, int nq, AttnWork wk,
                                                   float* __restrict__ out_m, float* __restrict__ out_l,
                                                   float* __restrict__ out_O, const double* __restrict__ colpre) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds5[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds5;
  float* xf = reinterpret_cast<float*>(lds5 + A5_X_OFF);
  switch ((w & 1) | (w >> 2) << 1) {  // (half, group)
    case 0: attn5_half<0, 0, MODE>(E3, n_ent, Qpre, nq, wk, out_m, out_l, out_O, colpre, w, lane, lds0, xf); break;
    case 1: attn5_half<1, 0, MODE>(E3, n_ent, Qpre, nq, wk, out_m, out_l, out_O, colpre, w, lane, lds0, xf); break;
    case 2: attn5_half<0, 1, MODE>(E3, n_ent, Qpre, nq, wk, out_m, out_l, out_O, colpre, w, lane, lds0, xf); break;
    default: attn5_half<1, 1, MODE>(E3, n_ent, Qpre, nq, wk, out_m, out_l, out_O, colpre, w, lane, lds0, xf); break;
  }
}

// Host: co-resident kp_attn5 workgroups per CU (one: the LDS), cached per context.
inline int attn5_wpc(kp_ctx* c) {
  if (c->attn5_wpc <= 0) {
    int n = 0, n2 = 0;
    KP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kp_attn5<ATT_SOFTMAX_O>, 512, attn5_lds_bytes()));
    KP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n2, kp_attn5<ATT_SOFTMAX>, 512, attn5_lds_bytes()));
    c->attn5_wpc = std::max(1, std::min(n, n2));
  }
  return c->attn5_wpc;
}

template <int MODE>
void launch_attn5(kp_ctx* c, int n_ent, const float* Q, int nq, const AttnPlan& plan, float* m, float* l, float* O) {
  KP_REQUIRE(c->dp == A5_DP, "attn5: the D = 400 ComplEx table only");
  KP_REQUIRE(n_ent == c->n_ent, "attn5: key count differs from the table's (tile prefix sums)");
  KP_REQUIRE((long long)(n_ent + 31) / 32 * 32 * A5_ROW_B + 1024 < (1LL << 31),
             "attn5: table too large for the 32-bit buffer descriptor of the split image");
  const uint8_t* E3 = split3_image<25>(c);
  const double* pre = tile_prefix<25>(c);
  hipLaunchKernelGGL((kp_attn5<MODE>), dim3(plan.n_wg), dim3(512), attn5_lds_bytes(), c->stream, E3, n_ent, Q, nq,
                     plan.wk, m, l, O, pre);
  KP_HIP(hipGetLastError());
}

}  // namespace kpattn
