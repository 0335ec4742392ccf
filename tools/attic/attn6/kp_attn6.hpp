// kp_attn6.hpp -- the ComplEx step attention (ATT_SOFTMAX_O, D = 400) of kp_attn3 with
// the O phase shared across a wave pair.
//
// kp_attn3 gives each of a workgroup's four waves its own 16 queries for both phases, so
// every wave reads the whole 32-entity key tile twice per tile: the rows for the S phase
// (ds_read_b128) and E^T for the O phase (two ds_read_b64_tr_b16 per piece and 16-dim
// block).  Its counters (profiles/r05a: settled clock, FB15k-237 shape) put 13 % of the
// wave cycles into LDS-issue stalls (SQ_WAIT_INST_LDS) at 228 LDS instructions per wave
// and tile, 150 of them the O phase's transposed reads.
//
// Here the waves w and w ^ 1 form a pair over their 32 queries:
//   * S phase, softmax and centring exactly as kp_attn3, each wave for its own 16 queries
//     over all 400 dims (its three-piece Q stays in VGPRs);
//   * the pair swaps its fp32 weights through LDS (2 KiB per wave, the 8 KiB beside the
//     two 76-KiB tile buffers) and each wave splits its partner's into the three bf16
//     pieces itself;
//   * O phase: member h accumulates O^T for BOTH queries groups over its half of the
//     dims (16-dim blocks 13 h .. 13 h + 12; member 1's 13th block lies past D = 400 and
//     is skipped), so each E^T operand read feeds 12 MFMAs instead of 6: 78 transposed
//     reads per wave and tile instead of 150, and the same 300 MFMAs.
// The MFMA sequences per (query, block) are kp_attn3's (same operands, same order), so
// the partials are bitwise those of kp_attn3 (tools/attn_micro.hip prints the output
// hash; the GPU parity tests compare both).
#pragma once
#include "kp_attn3.hpp"

namespace kpattn {

// O blocks per pair member and the LDS bytes: two tile buffers + four 2-KiB weight slots
template <int DB>
__host__ __device__ constexpr int attn6_ob() { return (DB + 1) / 2; }
template <int DB>
constexpr size_t attn6_lds_bytes() { return attn3_lds_bytes(DB) + 4u * 2048u; }

template <int DB>
__global__ __launch_bounds__(256, 1) void kp_attn6(const uint8_t* __restrict__ E3, int n_ent,
                                                   const float* __restrict__ Qpre, int nq, AttnWork wk,
                                                   float* __restrict__ out_m, float* __restrict__ out_l,
                                                   float* __restrict__ out_O, const double* __restrict__ colpre) {
  constexpr int DP = 16 * DB;
  static_assert(attn3_asm(DB) && attn3_bufdma(DB), "kp_attn6: the asm read form with buffer LDS-DMA only");
  constexpr int NK = DP / 32;
  constexpr int TAIL = (DP % 32) / 16;
  constexpr int KT = 32;
  constexpr int PART_B = 2 * DP;
  constexpr int ROW_B = split3_row_bytes(DP);
  constexpr int PIECES = attn3_buf_pieces(DB);
  constexpr int BUF_B = 1024 * PIECES;
  constexpr int OB = attn6_ob<DB>();
  constexpr int NPW = PIECES / 4;  // LDS-DMA pieces per wave and tile
  extern __shared__ __attribute__((aligned(16))) uint8_t lds6[];  // [2][BUF_B] tiles, [4][2048] weight slots

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hm = w & 1;          // pair member: O blocks [OB hm, OB hm + OB)
  const int mb = OB * hm;
  const int g = lane >> 4, c = lane & 15;
  int key_begin = 0, key_end = 0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds6;
  const uint32_t xs_own = lds0 + 2u * BUF_B + (uint32_t)(w * 2048 + 16 * lane);
  const uint32_t xs_par = lds0 + 2u * BUF_B + (uint32_t)((w ^ 1) * 2048 + 16 * lane);

  const __amdgpu_buffer_rsrc_t e3rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(E3), (short)0, (int)((n_ent + 31) / 32 * 32 * ROW_B + 1024), 0x00020000);
  auto bdma = [&](int tile, int buf, int p) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        e3rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds0 + (uint32_t)(buf * BUF_B + 1024 * p)), 16,
        16 * lane, (key_begin + tile * KT) * ROW_B + 1024 * p, 0, 0);
  };
  auto issue = [&](int tile, int buf) {
#pragma unroll
    for (int p0 = 0; p0 < PIECES; p0 += 4) bdma(tile, buf, p0 + w);
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
    const int q = qt * 64 + 16 * w + c;         // own query
    const int qp = qt * 64 + 16 * (w ^ 1) + c;  // the partner's
    const bool valid = q < nq, validp = qp < nq;
    // ---- own query pieces -> VGPRs (kp_attn3's B operand of the S phase)
    bf16x8 qb[NK][3];
    bf16x4 qt4[3];
    {
      const float* qpp = Qpre + (size_t)(valid ? q : 0) * DP;
#pragma unroll
      for (int s = 0; s < NK; ++s) {
        const float4 v0 = *reinterpret_cast<const float4*>(qpp + 32 * s + 8 * g);
        const float4 v1 = *reinterpret_cast<const float4*>(qpp + 32 * s + 8 * g + 4);
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hh, mm, ll;
          split3(valid ? f[j] : 0.f, hh, mm, ll);
          qb[s][0][j] = hh;
          qb[s][1][j] = mm;
          qb[s][2][j] = ll;
        }
      }
      if (TAIL) {
        const float4 v0 = *reinterpret_cast<const float4*>(qpp + 32 * NK + 4 * g);
        const float f[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 hh, mm, ll;
          split3(valid ? f[j] : 0.f, hh, mm, ll);
          qt4[0][j] = hh;
          qt4[1][j] = mm;
          qt4[2][j] = ll;
        }
      }
    }
    f32x4 O0[OB], O1[OB];  // O^T of the own / the partner's queries over this member's blocks
    float m_ref = kNegInf, l_run = 0.f;
    float csh = 0.f;

    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < OB; ++j) O0[j] = O1[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      l_run = 0.f;
      float m_seen = kNegInf;
      if (ntiles > 0) issue(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();

      for (int t = 0; t < ntiles; ++t) {
        const int k0 = key_begin + t * KT;
        const int tn = t + 1 < ntiles ? t + 1 : t;  // the last tile re-reads its own rows
        const uint32_t tb = lds0 + (uint32_t)((t & 1) * BUF_B);
        // ---- S phase: kp_attn3's interleaved schedule, unchanged
        f32x4 sc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
        const uint32_t rb = tb + (uint32_t)(c * ROW_B + 16 * g);
        const uint32_t rbt = rb - 8u * g;
        constexpr uint32_t SUB_B = 16u * ROW_B;
        static_assert(SUB_B + 3 * PART_B + 64 * NK < 65536, "LDS read offsets exceed the 16-bit offset field");
        constexpr int LAST = NK + TAIL - 1;
        bf16x8 ra[3][2][3];
        bf16x4 rt[2][3];
        auto load_step = [&](int j) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              if (j < NK)
                ra[j % 3][u][p] = lds_rd_bf8<true>(rb, (int)(u * SUB_B) + p * PART_B + 64 * j);
              else
                rt[u][p] = lds_rd_bf4<true>(rbt, (int)(u * SUB_B) + p * PART_B + 64 * NK);
            }
        };
        load_step(0);
        if (LAST >= 1) load_step(1);
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
              if (s < NK)
                sc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[b][u][kPA[k]], qb[s < NK ? s : 0][kPB[k]], sc[u],
                                                                0, 0, 0);
              else
                sc[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, rt[u][kPA[k]]),
                                                                  __builtin_bit_cast(s16x4, qt4[kPB[k]]), sc[u], 0, 0,
                                                                  0);
              if (u == 0 && s + 2 <= LAST) {
                const int j = s + 2, uu = k & 1, pp = k >> 1;
                if (j < NK)
                  ra[j % 3][uu][pp] = lds_rd_bf8<true>(rb, (int)(uu * SUB_B) + pp * PART_B + 64 * j);
                else
                  rt[uu][pp] = lds_rd_bf4<true>(rbt, (int)(uu * SUB_B) + pp * PART_B + 64 * NK);
              }
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        // ---- O-phase operands of this member's blocks: block m = global block mb + m;
        // blocks 0 and 1 are read before the softmax, block m + 2 during block m
        const uint32_t ob = tb + (uint32_t)((4 * g + (c >> 2)) * ROW_B + 8 * (c & 3) + 32 * mb);
        bf16x4 ol[3][3], oh[3][3];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            ol[m][p] = lds_rd_tr<true>(ob, p * PART_B + 32 * m);
            oh[m][p] = lds_rd_tr<true>(ob, 16 * ROW_B + p * PART_B + 32 * m);
          }
        // ---- softmax weights of the own queries (kp_attn3, ATT_SOFTMAX_O)
        float pw[2][4];
        {
          float v[2][4];
          float tmax = kNegInf;
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[u][r] = (k0 + 16 * u + 4 * g + r < key_end) ? sc[u][r] : kNegInf;
              tmax = fmaxf(tmax, v[u][r]);
            }
          m_seen = fmaxf(m_seen, tmax);
          if (pass == 0 && t == 0) {
            float mq = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
            m_ref = fmaxf(mq, __shfl_xor(mq, 32, 64));
          }
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) pw[u][r] = __expf(v[u][r] - m_ref);
        }
        {
          if (t == 0) {
            float mn = kPosInf;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (k0 + 16 * u + 4 * g + r < key_end) mn = fminf(mn, pw[u][r]);
            mn = fminf(mn, __shfl_xor(mn, 16, 64));
            mn = fminf(mn, __shfl_xor(mn, 32, 64));
            csh = (mn < kPosInf) ? mn : 0.f;
          }
          float lt = 0.f;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              pw[u][r] = (k0 + 16 * u + 4 * g + r < key_end) ? __fsub_rn(pw[u][r], csh) : 0.f;
            lt += (pw[u][0] + pw[u][1]) + (pw[u][2] + pw[u][3]);
          }
          l_run += lt;
        }
        // ---- the pair swaps its weights: own fp32 weights out (same lane layout, so the
        // partner's lane (g, c) gets the weights of this wave's query c), barrier, the
        // partner's in; both sets split into three bf16 pieces in the B layout
        {
          const f32x4 w0 = {pw[0][0], pw[0][1], pw[0][2], pw[0][3]};
          const f32x4 w1 = {pw[1][0], pw[1][1], pw[1][2], pw[1][3]};
          asm volatile("ds_write_b128 %0, %1\n\tds_write_b128 %0, %2 offset:1024" ::"v"(xs_own), "v"(w0), "v"(w1)
                       : "memory");
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        f32x4 x0, x1;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024" : "=v"(x0), "=v"(x1) : "v"(xs_par)
                     : "memory");
        bf16x8 pb[3], pq[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hh, mm, ll;
          split3(pw[j >> 2][j & 3], hh, mm, ll);
          pb[0][j] = hh;
          pb[1][j] = mm;
          pb[2][j] = ll;
        }
        lgkm_wait<0>();
        asm volatile("" : "+v"(x0), "+v"(x1));  // the partner's weights are used only after the wait
        __builtin_amdgcn_sched_barrier(0);
        {
          const float pv[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            __bf16 hh, mm, ll;
            split3(pv[j], hh, mm, ll);
            pq[0][j] = hh;
            pq[1][j] = mm;
            pq[2][j] = ll;
          }
        }
        // ---- O phase: per block, six MFMAs for the own queries and six for the partner's
        // on the same A operand (each chain in kp_attn3's smallest-first order); block
        // m + 2's six reads ride one per two MFMAs, this wave's DMA pieces of the next tile
        // spread over the blocks
#pragma unroll
        for (int m = 0; m < OB; ++m) {
          if (m + 1 < OB)
            lgkm_wait<6>();
          else
            lgkm_wait<0>();
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < NPW; ++k)
            if ((k * OB) / NPW == m) bdma(tn, (t + 1) & 1, 4 * k + w);
          __builtin_amdgcn_sched_barrier(0);
          bf16x8 a[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const bf16x4 x = ol[m % 3][p], y = oh[m % 3][p];
            a[p] = (bf16x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
          }
          const bool live = (DB % 2 == 0) || m + 1 < OB || hm == 0;  // member 1's last block: past D
#pragma unroll
          for (int k = 0; k < 12; ++k) {
            if (live) {
              if (k < 6)
                O0[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kPA[k]], pb[kPB[k]], O0[m], 0, 0, 0);
              else
                O1[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kPA[k - 6]], pq[kPB[k - 6]], O1[m], 0, 0, 0);
            }
            if (m + 2 < OB && (k & 1) == 0) {
              const int mm = m + 2, pp = k >> 2, hi = (k >> 1) & 1;
              if (hi)
                oh[mm % 3][pp] = lds_rd_tr<true>(ob, 16 * ROW_B + pp * PART_B + 32 * mm);
              else
                ol[mm % 3][pp] = lds_rd_tr<true>(ob, pp * PART_B + 32 * mm);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      float mq = fmaxf(m_seen, __shfl_xor(m_seen, 16, 64));
      mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
      if (pass == 1) break;
      // workgroup-wide "some weight exceeded e^kMargin" (kp_attn3's __syncthreads_or, here
      // through the weight slots: its static LDS word would not fit beside 160 KiB)
      int redo = 0;
      {
        const int any = __builtin_amdgcn_ballot_w64(mq > m_ref + kMargin) != 0;
        const uint32_t fa = lds0 + 2u * BUF_B + (uint32_t)(w * 2048 + 1024);
        if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(fa), "v"(any) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t fi = lds0 + 2u * BUF_B + (uint32_t)(i * 2048 + 1024);
          asm volatile("ds_read_b32 %0, %1" : "=v"(f[i]) : "v"(fi) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
        redo = __builtin_amdgcn_readfirstlane((f[0] | f[1]) | (f[2] | f[3]));
        asm volatile("s_barrier" ::: "memory");  // every wave has read the flags
      }
      if (!redo) break;
      m_ref = mq;
    }

    float l_tot = l_run + __shfl_xor(l_run, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    // the partner's centring shift per query (the weight slots are free after the last
    // tile's closing barrier)
    float cshp = 0.f;
    {
      const uint32_t a_own = lds0 + 2u * BUF_B + (uint32_t)(w * 2048 + 4 * c);
      const uint32_t a_par = lds0 + 2u * BUF_B + (uint32_t)((w ^ 1) * 2048 + 4 * c);
      if (g == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(a_own), "v"(csh) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(cshp) : "v"(a_par) : "memory");
      asm volatile("s_barrier" ::: "memory");  // the slots are free again for the next unit
    }
    if (ntiles > 0) {
      l_tot = __fmaf_rn(csh, (float)(key_end - key_begin), l_tot);
      const double* p0 = colpre + (size_t)kt0 * DP;
      const double* p1 = colpre + (size_t)kt1 * DP;
#pragma unroll
      for (int m = 0; m < OB; ++m) {
        if (mb + m >= DB) continue;
        const int d = 16 * (mb + m) + 4 * g;
        const double2 a0 = *reinterpret_cast<const double2*>(p0 + d), a1 = *reinterpret_cast<const double2*>(p0 + d + 2);
        const double2 b0 = *reinterpret_cast<const double2*>(p1 + d), b1 = *reinterpret_cast<const double2*>(p1 + d + 2);
        const float e0 = (float)(b0.x - a0.x), e1 = (float)(b0.y - a0.y), e2 = (float)(b1.x - a1.x),
                    e3 = (float)(b1.y - a1.y);
        O0[m][0] = __fmaf_rn(csh, e0, O0[m][0]);
        O0[m][1] = __fmaf_rn(csh, e1, O0[m][1]);
        O0[m][2] = __fmaf_rn(csh, e2, O0[m][2]);
        O0[m][3] = __fmaf_rn(csh, e3, O0[m][3]);
        O1[m][0] = __fmaf_rn(cshp, e0, O1[m][0]);
        O1[m][1] = __fmaf_rn(cshp, e1, O1[m][1]);
        O1[m][2] = __fmaf_rn(cshp, e2, O1[m][2]);
        O1[m][3] = __fmaf_rn(cshp, e3, O1[m][3]);
      }
    }
    if (valid && g == 0) {
      const size_t o = (size_t)part * nq + q;
      out_m[o] = m_ref;
      out_l[o] = l_tot;
    }
#pragma unroll
    for (int m = 0; m < OB; ++m) {
      if (mb + m >= DB) continue;
      const int d = 16 * (mb + m) + 4 * g;
      if (valid)
        *reinterpret_cast<float4*>(out_O + ((size_t)part * nq + q) * DP + d) =
            make_float4(O0[m][0], O0[m][1], O0[m][2], O0[m][3]);
      if (validp)
        *reinterpret_cast<float4*>(out_O + ((size_t)part * nq + qp) * DP + d) =
            make_float4(O1[m][0], O1[m][1], O1[m][2], O1[m][3]);
    }
    if (fill_rest) {
      for (int pp = part + 1; pp < wk.n_parts; ++pp) {
        if (valid && g == 0) {
          out_m[(size_t)pp * nq + q] = kNegInf;
          out_l[(size_t)pp * nq + q] = 0.f;
        }
        for (int m = 0; m < OB; ++m) {
          if (mb + m >= DB) continue;
          const int d = 16 * (mb + m) + 4 * g;
          if (valid)
            *reinterpret_cast<float4*>(out_O + ((size_t)pp * nq + q) * DP + d) = make_float4(0.f, 0.f, 0.f, 0.f);
          if (validp)
            *reinterpret_cast<float4*>(out_O + ((size_t)pp * nq + qp) * DP + d) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }
}

template <int DB>
int attn6_wpc(kp_ctx* c) {
  int n = 0;
  KP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kp_attn6<DB>, 256, attn6_lds_bytes<DB>()));
  return std::max(1, n);
}

template <int DB>
void launch_attn6(kp_ctx* c, int n_ent, const float* Q, int nq, const AttnPlan& plan, float* m, float* l, float* O) {
  KP_REQUIRE(n_ent == c->n_ent, "attn6: key count differs from the table's (tile prefix sums)");
  KP_REQUIRE((long long)(n_ent + 31) / 32 * 32 * split3_row_bytes(16 * DB) + 1024 < (1LL << 31),
             "attn6: table too large for the 32-bit buffer descriptor of the split image");
  const uint8_t* E3 = split3_image<DB>(c);
  const double* pre = tile_prefix<DB>(c);
  hipLaunchKernelGGL((kp_attn6<DB>), dim3(plan.n_wg), dim3(256), attn6_lds_bytes<DB>(), c->stream, E3, n_ent, Q, nq,
                     plan.wk, m, l, O, pre);
  KP_HIP(hipGetLastError());
}

}  // namespace kpattn
