// kp_attn.hpp -- the flash-attention-shaped pass over the frozen entity table
// shared by the ComplEx (softmax cross-entropy) and ConvE (sigmoid BCE)
// post-training steps.
#pragma once
#include "kp_common.hpp"

namespace kpattn {

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
// kp_cx_attn: per query q, over frozen entities [key_begin, key_end):
//   m = max_e s_e,  l = sum_e exp(s_e - m),  O = sum_e exp(s_e - m) E_e
// with s_e = q . E_e.  4 waves x 16 queries per workgroup share a 16-entity
// E tile in LDS (double buffered, register prefetch).  fp32 MFMA 16x16x4 in the
// swapped form: S^T = E . Q^T (key on the C row), so P already sits in the
// B-operand layout of O^T += E^T . P (no LDS round trip for P).
//   lane l: g = l>>4, c = l&15.  Q fragment qv[j][i] = Q[c][16j+4g+i] stays in
//   VGPRs; O^T accumulators O[j][r] = O[d = 16j+4g+r][q = c].
// MODE 0 (ComplEx step):  queries q = x_slot o R_rel built from qdesc, softmax + O.
// MODE 1 (ComplEx pairs):  queries read from Qpre, softmax statistics only.
// MODE 2 (ConvE BCE):      queries read from Qpre; instead of the softmax the
//   BCELoss-through-sigmoid gradient G(s) = ((p - y)/max(p(1-p),1e-12) * gs) * p(1-p)
//   (p = sigmoid(s), y = the smoothed non-target label, gs = 1/(b*N) per query,
//   bce_optimizer.py:35,98-112) weights O = sum_e G(s_e) E_e.
// ----------------------------------------------------------------------------
enum { ATT_SOFTMAX_O = 0, ATT_SOFTMAX = 1, ATT_BCE_O = 2 };

template <int DB, int MODE>
__global__ __launch_bounds__(256, 1) void kp_attn(const float* __restrict__ E, int n_ent, int half,
                                                  const int4* __restrict__ qdesc,
                                                  const float* __restrict__ X,
                                                  const float* __restrict__ R,
                                                  const float* __restrict__ Qpre, int nq,
                                                  int keys_per_split, float* __restrict__ out_m,
                                                  float* __restrict__ out_l, float* __restrict__ out_O,
                                                  const float* __restrict__ qscale, float ylo) {
  constexpr bool WITH_O = MODE != ATT_SOFTMAX;
  constexpr int DP = 16 * DB;
  constexpr int S = DP + 4;  // LDS row stride: 2-way b128 / conflict-free b32
  constexpr int KT = 16;
  constexpr int F4_ROW = DP / 4;
  constexpr int NF4 = KT * F4_ROW;
  constexpr int PF = (NF4 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][KT][S]

  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int q = blockIdx.x * 64 + 16 * w + c;
  const bool valid = q < nq;
  const int split = blockIdx.y;
  const int key_begin = split * keys_per_split;
  const int key_end = min(n_ent, key_begin + keys_per_split);

  // ---- Q fragment -> registers
  float qv[DB][4];
  float gsc = 0.f;
  if (MODE == ATT_BCE_O) gsc = valid ? qscale[q] : 0.f;
  if (MODE == ATT_SOFTMAX_O) {
    const int4 sr = valid ? qdesc[q] : make_int4(0, 0, 0, 0);
    const float* x = X + (size_t)sr.x * DP;
    const float* r = R + (size_t)sr.y * DP;
#pragma unroll
    for (int j = 0; j < DB; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[j][i] = valid ? cx_q(x, r, 16 * j + 4 * g + i, half) : 0.f;
  } else {
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
#pragma unroll
  for (int j = 0; j < (WITH_O ? DB : 1); ++j) O[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = kNegInf, l_run = 0.f;

  const int nkeys = max(0, key_end - key_begin);
  const int ntiles = (nkeys + KT - 1) / KT;
  float4 pf[PF];

  auto gload = [&](int tile) {
    const int k0 = key_begin + tile * KT;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      int f = tid + 256 * u;
      int row = f / F4_ROW, c4 = f - row * F4_ROW;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < NF4 && k0 + row < key_end) v = *reinterpret_cast<const float4*>(E + (size_t)(k0 + row) * DP + 4 * c4);
      pf[u] = v;
    }
  };
  auto lstore = [&](int buf) {
    float* base = lds + buf * (KT * S);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      int f = tid + 256 * u;
      if (f < NF4) {
        int row = f / F4_ROW, c4 = f - row * F4_ROW;
        *reinterpret_cast<float4*>(base + row * S + 4 * c4) = pf[u];
      }
    }
  };

  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) gload(t + 1);
    const float* Es = lds + (t & 1) * (KT * S);
    const int k0 = key_begin + t * KT;
    // ---- S^T tile: s[r] = q_c . E[k0 + 4g + r]
    // two independent accumulation chains (dependent-issue latency 40 > 32 cycles)
    f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f}, s2 = s;
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      float4 a = *reinterpret_cast<const float4*>(Es + c * S + 16 * j + 4 * g);
      s = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, qv[j][0], s, 0, 0, 0);
      s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, qv[j][1], s2, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, qv[j][2], s, 0, 0, 0);
      s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, qv[j][3], s2, 0, 0, 0);
    }
    s += s2;
    if (MODE == ATT_BCE_O) {
      float p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = 1.0f / (1.0f + __expf(-s[r]));
        const float w = (1.0f - pr) * pr;
        const float gr = ((pr - ylo) / fmaxf(w, 1e-12f) * gsc) * w;
        p[r] = (k0 + 4 * g + r < key_end) ? gr : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int j = 0; j < DB; ++j) {
          float a = Es[(4 * g + r) * S + 16 * j + c];
          O[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, p[r], O[j], 0, 0, 0);
        }
      }
      if (t + 1 < ntiles) lstore((t + 1) & 1);
      __syncthreads();
      continue;
    }
    float sv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sv[r] = (k0 + 4 * g + r < key_end) ? s[r] : kNegInf;
    float tmax = fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float scale = __expf(m_run - m_new);
    float p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = __expf(sv[r] - m_new);
    l_run = l_run * scale + ((p[0] + p[1]) + (p[2] + p[3]));
    m_run = m_new;
    if (WITH_O) {
      if (__any(scale != 1.0f)) {
#pragma unroll
        for (int j = 0; j < DB; ++j) O[j] *= scale;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int j = 0; j < DB; ++j) {
          float a = Es[(4 * g + r) * S + 16 * j + c];
          O[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, p[r], O[j], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) lstore((t + 1) & 1);
    __syncthreads();
  }

  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (valid) {
    const size_t o = (size_t)split * nq + q;
    if (g == 0 && MODE != ATT_BCE_O) {
      out_m[o] = m_run;
      out_l[o] = l_tot;
    }
    if (WITH_O) {
      float* dst = out_O + o * DP;
#pragma unroll
      for (int j = 0; j < DB; ++j)
        *reinterpret_cast<float4*>(dst + 16 * j + 4 * g) = make_float4(O[j][0], O[j][1], O[j][2], O[j][3]);
    }
  }
}


}  // namespace kpattn
