// kp_conve.hip -- ConvE batched post-training (KelpieConvE + KelpieBCEOptimizer)
// and ranking, for gfx950.
//
// Reference semantics (src/link_prediction/models/conve.py:133-158,193-237,
// src/link_prediction/optimization/bce_optimizer.py:92-112,161-208):
//   rows = kelpie triples + inverses -> er_vocab (h, r) -> tails, insertion
//   order, NOT shuffled; minibatches of batch_size pairs; targets one-hot over
//   N = |E|+1 entities, smoothed (1-ls) y + 1/N; BCELoss(sigmoid(x . E_all^T));
//   encoder: BN1 -> input dropout -> conv 3x3 (32) -> BN2 -> ReLU -> feature-map
//   Dropout2d -> FC -> hidden dropout -> BN3 -> ReLU, with every layer frozen and BN in
//   eval mode, but the three dropouts in TRAIN mode (model.py:114-125): their masks are
//   drawn on the host (RNG as input, packed keep bits: per slot and step one word-aligned
//   run per dropout, in the forward's draw order); Adam(lr = 1e-3) on the kelpie row.
//   With an input or feature-map dropout the frozen-head pairs' encodings change every
//   step, so they are encoded per step with the kelpie pairs (else once per batch).
//
// Per step, for the pairs whose head is the kelpie ("kelpie pairs"):
//   conv forward (kp_cv_conv_fwd) -> FC (fp32 MFMA GEMM, split-K) -> dropout/BN3/ReLU
//   (kp_cv_post_fc) -> O = sum_e G(x . E_e) E_e over the frozen entities
//   (kpattn::kp_attn<.., ATT_BCE_O>, the same MFMA pass as ComplEx) -> target and
//   kelpie-column corrections and the encoder backward (kp_cv_dx, FC^T GEMM,
//   kp_cv_conv_bwd) -> kp_cv_update (+ the kelpie-column gradient of every pair;
//   pairs with a frozen head reuse their precomputed FC output) -> Adam.
#include <chrono>
#include <cstdio>
#include <cmath>
#include <unordered_map>

#include "kp_attn.hpp"
#include "kp_attn3.hpp"
#include "kp_cv_fused.hpp"

int cx_pick_db(int dim);

namespace {
using namespace kpattn;

using kpcvf::CvBits;
struct CvInst {  // one kelpie pair in one step
  int slot, rel, b, pos;
  CvBits mb;
  int tail_begin, tail_count;
};
struct CvFInst {  // one frozen-head pair in one step
  int slot, fp, b, pos;  // fp: its FC row (per batch), or its encoded row in the step's Q (fr_step)
  CvBits mb;
};
struct CvAct {
  int slot, k_begin, k_count, f_begin, f_count, pad0, pad1, pad2;
};
struct CvConst {
  int n_ent, dim, dp, H, hid;
  float scale;  // hidden dropout: 1/(1-p) as float32 (the noise value of a kept element)
  float ylo, yhi;
  int has_mask;             // hidden dropout drawn
  int has_in, has_fm;       // input / feature-map dropout drawn
  float scale_in, scale_fm;
  int fr_step;              // frozen-head pairs encoded every step (has_in || has_fm)
};

__device__ __forceinline__ float bce_g(float s, float y, float gs) {
  // BCELoss backward (grad = gs) followed by sigmoid backward, torch op order
#if KP_CV_EXACT_BCE & 1
  const float p = 1.0f / (1.0f + expf(-s));
#else
  const float p = 1.0f / (1.0f + __expf(-s));
#endif
  const float w = (1.0f - p) * p;
#if KP_CV_EXACT_BCE & 2
  if (w >= 1e-12f) return (p - y) * gs;
#endif
  return ((p - y) / fmaxf(w, 1e-12f) * gs) * w;
}

// the dropout multiplier of element idx of a pair's run starting at bit base (ATen's
// noise: bernoulli(keep) / keep, i.e. 1/(1-p) or 0); 1 when that dropout is not drawn
__device__ __forceinline__ float noise_at(const int32_t* __restrict__ bits, long long base, int idx, float scale) {
  if (base < 0) return 1.0f;
  const long long b = base + idx;
  const uint32_t w = (uint32_t)bits[b >> 5];
  return ((w >> (b & 31)) & 1u) ? scale : 0.0f;
}

// image (BN1) -> conv 3x3 + bias -> BN2 -> ReLU -> flat (conve.py:134-146).
// src[i] = (lhs, rel): lhs >= 0 a frozen entity row, lhs < 0 the kelpie row X[-lhs-1].
// W2C > 0: the feature-map width H - 2 as a compile-time constant (d = 200: 8), so the
// per-output index divisions become multiplies; 0: read from k.H
template <int W2C>
__global__ __launch_bounds__(256) void kp_cv_conv_fwd(int M, const int2* __restrict__ src,
                                                      const float* __restrict__ E, const float* __restrict__ X,
                                                      const float* __restrict__ R, CvConst k,
                                                      const float* __restrict__ cw, const float* __restrict__ cb,
                                                      const float* __restrict__ bna, const float* __restrict__ bnb,
                                                      const CvBits* __restrict__ mb, const int32_t* __restrict__ bits,
                                                      float* __restrict__ flat) {
  __shared__ float img[40 * 32];
  __shared__ float w[288], bias[32], a2[32], b2[32];
  const int i = blockIdx.x;
  if (i >= M) return;
  const int tid = threadIdx.x;
  const int2 sr = src[i];
  const float* lhs = sr.x >= 0 ? E + (size_t)sr.x * k.dp : X + (size_t)(-sr.x - 1) * k.dp;
  const float* rel = R + (size_t)sr.y * k.dp;
  const float a1 = bna[0], b1 = bnb[0];
  const long long in_b = mb ? mb[i].in : -1, fm_b = mb ? mb[i].fm : -1;
  for (int j = tid; j < 20 * k.H; j += 256) {
    img[j] = lhs[j] * a1 + b1;
    img[20 * k.H + j] = rel[j] * a1 + b1;
    if (in_b >= 0) {  // input dropout on the BN1 image (conve.py:141-142)
      img[j] *= noise_at(bits, in_b, j, k.scale_in);
      img[20 * k.H + j] *= noise_at(bits, in_b, 20 * k.H + j, k.scale_in);
    }
  }
  for (int j = tid; j < 288; j += 256) w[j] = cw[j];
  if (tid < 32) {
    bias[tid] = cb[tid];
    a2[tid] = bna[1 + tid];
    b2[tid] = bnb[1 + tid];
  }
  __syncthreads();
  const int W2 = W2C > 0 ? W2C : k.H - 2;
  const int per_c = 38 * W2;
  for (int o = tid; o < k.hid; o += 256) {
    const int c = o / per_c, rem = o - c * per_c;
    const int y = rem / W2, xx = rem - y * W2;
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) acc += w[c * 9 + ky * 3 + kx] * img[(y + ky) * k.H + xx + kx];
    acc += bias[c];
    const float v = acc * a2[c] + b2[c];
    float f = fmaxf(v, 0.f);
    if (fm_b >= 0) f *= noise_at(bits, fm_b, c, k.scale_fm);  // feature-map Dropout2d (conve.py:147)
    flat[(size_t)i * k.hid + o] = f;
  }
}

// x = ReLU(BN3(dropout(FC))) from the split-K FC slabs; writes dp-padded rows
__global__ void kp_cv_post_fc(int M, const float* __restrict__ slabs, int ksplit, CvConst k,
                              const CvBits* __restrict__ mb, const int32_t* __restrict__ bits,
                              const float* __restrict__ bna, const float* __restrict__ bnb, float* __restrict__ Q) {
  const int i = blockIdx.x;
  if (i >= M) return;
  const float* a3 = bna + 33;
  const float* b3 = bnb + 33;
  for (int d = threadIdx.x; d < k.dp; d += blockDim.x) {
    float v = 0.f;
    if (d < k.dim) {
      float fc = 0.f;
      for (int z = 0; z < ksplit; ++z) fc += slabs[((size_t)z * M + i) * k.dim + d];
      float nz = 1.0f;
      if (mb && k.has_mask) nz = noise_at(bits, mb[i].hid, d, k.scale);
      const float dr = (mb && k.has_mask) ? fc * nz : fc;
      v = fmaxf(dr * a3[d] + b3[d], 0.f);
    }
    Q[(size_t)i * k.dp + d] = v;
  }
}

// the shared-encoder path (kp_cv_fused.hpp): fc_i = (the kelpie row's band slabs, FC bias
// in band 0) + (the pair's map-row-18-19 slabs) + trel[relation], then as kp_cv_post_fc
__global__ void kp_cv_post_fc3(int M, const float* __restrict__ sl, int nzl, int nl, const float* __restrict__ sm,
                               int nzm, const float* __restrict__ trel, const int2* __restrict__ src,
                               const int2* __restrict__ psr, CvConst k, const CvBits* __restrict__ mb,
                               const int32_t* __restrict__ bits, const float* __restrict__ bna,
                               const float* __restrict__ bnb, float* __restrict__ Q) {
  const int i = blockIdx.x;
  if (i >= M) return;
  const int kr = psr[i].x, rel = src[i].y;
  const float* a3 = bna + 33;
  const float* b3 = bnb + 33;
  for (int d = threadIdx.x; d < k.dp; d += blockDim.x) {
    float v = 0.f;
    if (d < k.dim) {
      float fl = 0.f, fm = 0.f;
      for (int z = 0; z < nzl; ++z) fl += sl[((size_t)z * nl + kr) * k.dim + d];
      for (int z = 0; z < nzm; ++z) fm += sm[((size_t)z * M + i) * k.dim + d];
      const float fc = (fl + fm) + trel[(size_t)rel * k.dim + d];
      float nz = 1.0f;
      if (mb && k.has_mask) nz = noise_at(bits, mb[i].hid, d, k.scale);
      const float dr = (mb && k.has_mask) ? fc * nz : fc;
      v = fmaxf(dr * a3[d] + b3[d], 0.f);
    }
    Q[(size_t)i * k.dp + d] = v;
  }
}

// block-wide sum (256 threads)
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

// kp_cv_dx's dot products in its summation order: a 256-thread block_sum of per-thread
// partials over d = tid + 256 m, i.e. four wave sums (old wave w: d mod 256 in [64 w,
// 64 w + 64)) added in wave order.  One wave holding d = l + 64 j (lane l) keeps one
// partial per j mod 4 -- partial w is old wave w's lane l, accumulated in the same m
// order -- and adds the four wave sums in old-wave order: bitwise the block's result,
// with no LDS.
template <int NJ>
__device__ __forceinline__ float dot256_order1(const float* a, const float* b) {
  float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NJ; ++j) p[j & 3] += a[j] * b[j];
  return ((wave_sum(p[0]) + wave_sum(p[1])) + wave_sum(p[2])) + wave_sum(p[3]);
}

// kp_cv_dx on one wave per pair (NJ = ceil(dp / 64) row values per lane, in registers),
// bitwise the same as the 256-thread form below.  No LDS and <= 32 VGPRs, so it runs beside
// the other batch's attention workgroups: two kp_attn3<13> workgroups (asm form, 80 KiB
// each) fill a CU's LDS, and the round-5 two-wave form's 16 bytes of LDS then kept it off
// every CU they held (354 us per launch against 65 us, profiles/r06/r06y)
template <int NJ>
__global__ __launch_bounds__(64) void kp_cv_dx1(int M, CvConst k, const CvInst* __restrict__ inst,
                                                const float* __restrict__ Q, const float* __restrict__ O, int n_split,
                                                const int32_t* __restrict__ tails, const float* __restrict__ E,
                                                const float* __restrict__ X, const int32_t* __restrict__ bits,
                                                const float* __restrict__ bna, float* __restrict__ dfc,
                                                float* __restrict__ gk, __bf16* __restrict__ g3) {
  const int i = blockIdx.x;
  if (i >= M) return;
  const int t = threadIdx.x;
  const CvInst I = inst[i];
  float xi[NJ], xk[NJ], dx[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int d = t + 64 * j;
    const bool in = d < k.dim;
    xi[j] = in ? Q[(size_t)i * k.dp + d] : 0.f;
    xk[j] = in ? X[(size_t)I.slot * k.dp + d] : 0.f;
  }
  const float gs = 1.0f / (float)((long long)I.b * (long long)(k.n_ent + 1));
  const float sk = dot256_order1<NJ>(xi, xk);  // kelpie column
  bool k_is_tail = false;
  for (int u = 0; u < I.tail_count; ++u) k_is_tail |= (tails[I.tail_begin + u] == k.n_ent);
  const float Gk = bce_g(sk, k_is_tail ? k.yhi : k.ylo, gs);
  if (t == 0) gk[i] = Gk;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int d = t + 64 * j;
    float v = 0.f;
    if (d < k.dim)
      for (int sp = 0; sp < n_split; ++sp) v += O[((size_t)sp * M + i) * k.dp + d];
    dx[j] = v + Gk * xk[j];
  }
  // target corrections: G(s, yhi) - G(s, ylo) for the frozen tails
  for (int u = 0; u < I.tail_count; ++u) {
    const int e = tails[I.tail_begin + u];
    if (e == k.n_ent) continue;
    float er[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int d = t + 64 * j;
      er[j] = d < k.dim ? E[(size_t)e * k.dp + d] : 0.f;
    }
    const float st = dot256_order1<NJ>(xi, er);
    const float corr = bce_g(st, k.yhi, gs) - bce_g(st, k.ylo, gs);
#pragma unroll
    for (int j = 0; j < NJ; ++j) dx[j] += corr * er[j];
  }
  const float* a3 = bna + 33;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int d = t + 64 * j;
    if (d < k.dim) {
      const float nz = k.has_mask ? noise_at(bits, I.mb.hid, d, k.scale) : 1.0f;
      const float relu = xi[j] > 0.f ? 1.0f : 0.0f;
      const float v = dx[j] * relu * a3[d] * nz;
      dfc[(size_t)i * k.dim + d] = v;
      if (g3) {  // kp_cv_bwd_fused's A operand: [3][M][KB] bf16 pieces
        __bf16 h, m, l;
        split3(v, h, m, l);
        const size_t o = (size_t)i * kpcvf::KB + d, ps = (size_t)M * kpcvf::KB;
        g3[o] = h;
        g3[ps + o] = m;
        g3[2 * ps + o] = l;
      }
    }
  }
  if (g3)
    for (int d = k.dim + t; d < kpcvf::KB; d += 64) {
      const size_t o = (size_t)i * kpcvf::KB + d, ps = (size_t)M * kpcvf::KB;
      g3[o] = g3[ps + o] = g3[2 * ps + o] = (__bf16)0.f;
    }
}

// dL/dx_i (encoder output) -> dL/dfc_i; also G at the kelpie column
__global__ __launch_bounds__(256) void kp_cv_dx(int M, CvConst k, const CvInst* __restrict__ inst,
                                                const float* __restrict__ Q, const float* __restrict__ O, int n_split,
                                                const int32_t* __restrict__ tails, const float* __restrict__ E,
                                                const float* __restrict__ X, const int32_t* __restrict__ bits,
                                                const float* __restrict__ bna, float* __restrict__ dfc,
                                                float* __restrict__ gk, __bf16* __restrict__ g3) {
  __shared__ float red[4];
  __shared__ float xi[640], xk[640];
  const int i = blockIdx.x;
  if (i >= M) return;
  const int tid = threadIdx.x;
  const CvInst I = inst[i];
  for (int d = tid; d < k.dp; d += 256) {
    xi[d] = Q[(size_t)i * k.dp + d];
    xk[d] = X[(size_t)I.slot * k.dp + d];
  }
  __syncthreads();
  const float gs = 1.0f / (float)((long long)I.b * (long long)(k.n_ent + 1));
  // kelpie column
  float part = 0.f;
  for (int d = tid; d < k.dim; d += 256) part += xi[d] * xk[d];
  const float sk = block_sum(part, red);
  bool k_is_tail = false;
  for (int t = 0; t < I.tail_count; ++t) k_is_tail |= (tails[I.tail_begin + t] == k.n_ent);
  const float Gk = bce_g(sk, k_is_tail ? k.yhi : k.ylo, gs);
  if (tid == 0) gk[i] = Gk;
  const float* a3 = bna + 33;
  for (int d0 = 0; d0 < k.dim; d0 += 256) {
    const int d = d0 + tid;
    float dx = 0.f;
    if (d < k.dim) {
      for (int sp = 0; sp < n_split; ++sp) dx += O[((size_t)sp * M + i) * k.dp + d];
      dx += Gk * xk[d];
    }
    // target corrections: G(s, yhi) - G(s, ylo) for the frozen tails
    for (int t = 0; t < I.tail_count; ++t) {
      const int e = tails[I.tail_begin + t];
      if (e == k.n_ent) continue;
      float pp = 0.f;
      for (int dd = tid; dd < k.dim; dd += 256) pp += xi[dd] * E[(size_t)e * k.dp + dd];
      const float st = block_sum(pp, red);
      const float corr = bce_g(st, k.yhi, gs) - bce_g(st, k.ylo, gs);
      if (d < k.dim) dx += corr * E[(size_t)e * k.dp + d];
    }
    if (d < k.dim) {
      const float nz = k.has_mask ? noise_at(bits, I.mb.hid, d, k.scale) : 1.0f;
      const float relu = xi[d] > 0.f ? 1.0f : 0.0f;
      const float v = dx * relu * a3[d] * nz;
      dfc[(size_t)i * k.dim + d] = v;
      if (g3) {  // kp_cv_bwd_fused's A operand: [3][M][KB] bf16 pieces
        __bf16 h, m, l;
        split3(v, h, m, l);
        const size_t o = (size_t)i * kpcvf::KB + d, ps = (size_t)M * kpcvf::KB;
        g3[o] = h;
        g3[ps + o] = m;
        g3[2 * ps + o] = l;
      }
    }
  }
  if (g3)
    for (int d = k.dim + tid; d < kpcvf::KB; d += 256) {
      const size_t o = (size_t)i * kpcvf::KB + d, ps = (size_t)M * kpcvf::KB;
      g3[o] = g3[ps + o] = g3[2 * ps + o] = (__bf16)0.f;
    }
}

// dL/dflat -> ReLU / BN2 -> transposed 3x3 conv -> BN1 -> the lhs half of the image
// (feature-map dropout: flat holds the dropped map, so flat > 0 is the ReLU mask of a
// kept channel, and a kept channel's gradient carries its 1/(1-p); input dropout: the
// image gradient times the input mask)
__global__ __launch_bounds__(256) void kp_cv_conv_bwd(int M, CvConst k, const float* __restrict__ dflat,
                                                      const float* __restrict__ flat,
                                                      const float* __restrict__ cw, const float* __restrict__ bna,
                                                      const CvBits* __restrict__ mb,
                                                      const int32_t* __restrict__ bits, float* __restrict__ dl) {
  extern __shared__ __attribute__((aligned(16))) float dc[];  // [32][20][W2]
  __shared__ float w[288];
  const int i = blockIdx.x;
  if (i >= M) return;
  const int tid = threadIdx.x;
  const int W2 = k.H - 2;
  const int per_c = 38 * W2;
  for (int j = tid; j < 288; j += 256) w[j] = cw[j];
  for (int j = tid; j < 32 * 20 * W2; j += 256) {
    const int c = j / (20 * W2), rem = j - c * 20 * W2;
    const int o = c * per_c + rem;  // rows 0..19 of channel c
    const float f = flat[(size_t)i * k.hid + o];
    const float g = dflat[(size_t)i * k.hid + o];
    dc[j] = (f > 0.f) ? (k.has_fm ? g * k.scale_fm : g) * bna[1 + c] : 0.f;
  }
  __syncthreads();
  const float a1 = bna[0];
  for (int j = tid; j < 20 * k.H; j += 256) {
    const int yy = j / k.H, xx = j - yy * k.H;
    float acc = 0.f;
    for (int c = 0; c < 32; ++c) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int y = yy - ky;
        if (y < 0 || y >= 20) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int x = xx - kx;
          if (x < 0 || x >= W2) continue;
          acc += dc[(c * 20 + y) * W2 + x] * w[c * 9 + ky * 3 + kx];
        }
      }
    }
    if (k.has_in) acc *= noise_at(bits, mb[i].in, j, k.scale_in);
    dl[(size_t)i * k.dp + j] = acc * a1;
  }
}

// kp_cv_conv_fwd with the width specialised for d = 200 (H = 10)
#define KP_CONV_FWD(grid, block, shm, stream, M, src, E, X, R, kk, ...)                                      \
  do {                                                                                                      \
    if ((kk).H == 10)                                                                                       \
      hipLaunchKernelGGL(kp_cv_conv_fwd<8>, grid, block, shm, stream, M, src, E, X, R, kk, __VA_ARGS__);    \
    else                                                                                                    \
      hipLaunchKernelGGL(kp_cv_conv_fwd<0>, grid, block, shm, stream, M, src, E, X, R, kk, __VA_ARGS__);    \
  } while (0)

struct CvOpt {
  float lr, b1, b2, eps, one_minus_b1, one_minus_b2, step_size, bc2_sqrt;
};

// the frozen-head pairs' part of a slot's gradient (o, r_inv, kelpie): the kelpie
// column's BCE gradient G * x_fc, in chunks of up to FCH pairs of one slot, one workgroup per
// chunk (a hub slot's hundreds of pairs no longer run as one workgroup's serial loop);
// ch = (slot's act index in the step, first pair, pair count); fpart[chunk][d]
constexpr int FCH = 16;
__global__ __launch_bounds__(256) void kp_cv_fgrad(CvConst k, const int4* __restrict__ chunks,
                                                   const CvAct* __restrict__ act, const CvFInst* __restrict__ fi,
                                                   const float* __restrict__ fcf, const int32_t* __restrict__ bits,
                                                   const float* __restrict__ bna, const float* __restrict__ bnb,
                                                   const float* __restrict__ X, float* __restrict__ fpart) {
  __shared__ float xs[640];
  __shared__ float gw_s[4][640];  // per-wave partial sums
  const int4 ch = chunks[blockIdx.x];
  const CvAct A = act[ch.x];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const float* x = X + (size_t)A.slot * k.dp;
  for (int d = tid; d < k.dp; d += 256) xs[d] = x[d];
  __syncthreads();
  const float* a3 = bna + 33;
  const float* b3 = bnb + 33;
  float gw[10];
#pragma unroll
  for (int u = 0; u < 10; ++u) gw[u] = 0.f;
  auto load_pair = [&](const CvFInst& F, float (&v)[10]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int d = lane + 64 * u;
      v[u] = 0.f;
      if (d < k.dim) {
        if (k.fr_step) {  // encoded this step with its own masks (kp_cv_post_fc)
          v[u] = fcf[(size_t)F.fp * k.dp + d];
        } else {
          const float fc = fcf[(size_t)F.fp * k.dim + d];
          const float nz = k.has_mask ? noise_at(bits, F.mb.hid, d, k.scale) : 1.0f;
          const float dr = k.has_mask ? fc * nz : fc;
          v[u] = fmaxf(dr * a3[d] + b3[d], 0.f);
        }
      }
    }
  };
  auto add_pair = [&](const CvFInst& F, const float (&v)[10]) __attribute__((always_inline)) {
    float part = 0.f;
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int d = lane + 64 * u;
      if (d < k.dim) part += v[u] * xs[d];
    }
    const float s = wave_sum(part);
    const float gs = 1.0f / (float)((long long)F.b * (long long)(k.n_ent + 1));
    const float G = bce_g(s, k.yhi, gs);
#pragma unroll
    for (int u = 0; u < 10; ++u) gw[u] += G * v[u];
  };
  // a wave's pairs (wave, wave + 4, ...) two at a time: both rows loaded before either
  // reduction
  const int f0 = A.f_begin + ch.y;
  int j = wave;
  for (; j + 4 < ch.z; j += 8) {
    const CvFInst F0 = fi[f0 + j], F1 = fi[f0 + j + 4];
    float v0[10], v1[10];
    load_pair(F0, v0);
    load_pair(F1, v1);
    add_pair(F0, v0);
    add_pair(F1, v1);
  }
  if (j < ch.z) {
    const CvFInst F0 = fi[f0 + j];
    float v0[10];
    load_pair(F0, v0);
    add_pair(F0, v0);
  }
#pragma unroll
  for (int u = 0; u < 10; ++u) {
    const int d = lane + 64 * u;
    if (d < k.dim) gw_s[wave][d] = gw[u];
  }
  __syncthreads();
  for (int d = tid; d < k.dim; d += 256)
    fpart[(size_t)blockIdx.x * k.dim + d] = (gw_s[0][d] + gw_s[1][d]) + (gw_s[2][d] + gw_s[3][d]);
}

// gradient assembly + Adam, one workgroup per active slot; its frozen-head pairs' part is
// the sum of its kp_cv_fgrad chunks (A.pad0: first chunk of the step, A.pad1: count)
__global__ __launch_bounds__(256) void kp_cv_update(CvConst k, const CvAct* __restrict__ act,
                                                    const float* __restrict__ Q, const float* __restrict__ gk,
                                                    const float* __restrict__ dl, const float* __restrict__ fpart,
                                                    float* __restrict__ X, float* __restrict__ S1,
                                                    float* __restrict__ S2, CvOpt opt) {
  __shared__ float xs[640];
  const CvAct A = act[blockIdx.x];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  float* x = X + (size_t)A.slot * k.dp;
  for (int d = tid; d < k.dp; d += 256) xs[d] = x[d];
  __syncthreads();
  float g[3] = {0.f, 0.f, 0.f};
  // kelpie-head pair rows: a slot with more than 4 sums them in four wave-strided
  // partials with two chains each (one chain per dimension was bound by load latency);
  // the choice is block-uniform
  __shared__ float gk_s[4][640];
  const bool wide = A.k_count > 4;
  if (wide) {
    for (int d = lane; d < k.dim; d += 64) {
      float a0 = 0.f, a1 = 0.f;
      int j = wave;
      for (; j + 4 < A.k_count; j += 8) {
        const int i0 = A.k_begin + j, i1 = i0 + 4;
        a0 += gk[i0] * Q[(size_t)i0 * k.dp + d] + dl[(size_t)i0 * k.dp + d];
        a1 += gk[i1] * Q[(size_t)i1 * k.dp + d] + dl[(size_t)i1 * k.dp + d];
      }
      if (j < A.k_count) {
        const int i0 = A.k_begin + j;
        a0 += gk[i0] * Q[(size_t)i0 * k.dp + d] + dl[(size_t)i0 * k.dp + d];
      }
      gk_s[wave][d] = a0 + a1;
    }
  } else {
    for (int j = 0; j < A.k_count; ++j) {
      const int ii = A.k_begin + j;
      const float G = gk[ii];
      for (int u = 0; u < 3; ++u) {
        const int d = tid + 256 * u;
        if (d < k.dim) g[u] += G * Q[(size_t)ii * k.dp + d] + dl[(size_t)ii * k.dp + d];
      }
    }
  }
  __syncthreads();
  for (int u = 0; u < 3; ++u) {
    const int d = tid + 256 * u;
    if (d >= k.dim) continue;
    if (wide) g[u] = (gk_s[0][d] + gk_s[1][d]) + (gk_s[2][d] + gk_s[3][d]);
    float fw = 0.f;
    for (int c = 0; c < A.pad1; ++c) fw += fpart[(size_t)(A.pad0 + c) * k.dim + d];
    g[u] += fw;
  }
  for (int u = 0; u < 3; ++u) {
    const int d = tid + 256 * u;
    if (d >= k.dim) continue;
    const size_t o = (size_t)A.slot * k.dp + d;
    float m1 = S1[o], v2 = S2[o];
    const float gd = g[u];
    m1 = m1 + opt.one_minus_b1 * (gd - m1);
    v2 = v2 * opt.b2;
    v2 = v2 + (opt.one_minus_b2 * gd) * gd;
    const float den = sqrtf(v2) / opt.bc2_sqrt + opt.eps;
    x[d] = xs[d] + (-opt.step_size * m1) / den;
    S1[o] = m1;
    S2[o] = v2;
  }
}

// fp64 ranking queries (launch_rank_f64, act 1): the encoder output of the post-trained
// row (fp32, eval mode) widened to fp64; its logit against the target and against the
// kelpie row as one sequential fp64 FMA chain over d (exact products of fp32 operands),
// the order kp_rank_f64_count scores every entity in.  At the reference init the sigmoid
// scores of ~10^5 entities lie within ~0.005 of 0.5, a few per fp32 ulp there, so fp32
// scores tie and their rounding moves the rank; the logits order them as a fp64 run does.
__global__ void kp_cv_rankq64(const float* __restrict__ Qr, const float* __restrict__ X,
                              const float* __restrict__ E, int n_ent, int dp, const int32_t* __restrict__ po,
                              int n_slots, double* __restrict__ Q, double* __restrict__ t64,
                              double* __restrict__ kcol64) {
  const int s = blockIdx.x;
  if (s >= n_slots) return;
  double* q = Q + (size_t)s * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) q[d] = (double)Qr[(size_t)s * dp + d];
  __syncthreads();
  if (threadIdx.x == 0) {
    const float* x = X + (size_t)s * dp;
    const int o = po[s];
    double z = 0.0, t = 0.0;
    for (int d = 0; d < dp; ++d) z = __fma_rn(q[d], (double)x[d], z);
    if (o < n_ent) {
      const float* eo = E + (size_t)o * dp;
      for (int d = 0; d < dp; ++d) t = __fma_rn(q[d], (double)eo[d], t);
    } else {
      t = z;  // the kelpie entity is its own object
    }
    kcol64[s] = z;
    t64[s] = t;
  }
}

// kelpie column of the rank scores: sigmoid(q_s . x_s)
__global__ void kp_cv_kcol(int n, CvConst k, const float* __restrict__ Q, const float* __restrict__ X,
                           float* __restrict__ scores, int ld) {
  const int s = blockIdx.x;
  if (s >= n) return;
  float z = 0.f;
  for (int d = threadIdx.x; d < k.dim; d += 64) z += Q[(size_t)s * k.dp + d] * X[(size_t)s * k.dp + d];
  z = wave_sum(z);
  if (threadIdx.x == 0) scores[(size_t)s * ld + k.n_ent] = 1.0f / (1.0f + expf(-z));
}

CvConst make_const(kp_ctx* c, const kp_hp* hp) {
  CvConst k{};
  k.n_ent = c->n_ent;
  k.dim = c->dim;
  k.dp = c->dp;
  k.H = c->dim / 20;
  k.hid = c->hidden;
  // ATen's noise value: 1 / (1 - p) in float32 (the dropout's div_ of the bernoulli mask);
  // p == 1 ships zero keep bits, so its infinite scale is never selected
  auto scale_of = [](double p) { return (p > 0.0 && p < 1.0) ? (1.0f / (float)(1.0 - p)) : 1.0f; };
  const double p = hp ? hp->hidden_dropout : 0.0;
  k.has_mask = (p > 0.0) ? 1 : 0;
  k.scale = scale_of(p);
  const double pin = hp ? hp->input_dropout : 0.0, pfm = hp ? hp->fmap_dropout : 0.0;
  k.has_in = (pin > 0.0) ? 1 : 0;
  k.has_fm = (pfm > 0.0) ? 1 : 0;
  k.scale_in = scale_of(pin);
  k.scale_fm = scale_of(pfm);
  k.fr_step = (k.has_in || k.has_fm) ? 1 : 0;
  const double ls = hp ? hp->label_smoothing : 0.0;
  if (ls != 0.0) {
    const float inv_n = (float)(1.0 / (double)(c->n_ent + 1));
    k.ylo = inv_n;
    k.yhi = (float)(1.0 - ls) * 1.0f + inv_n;
  } else {
    k.ylo = 0.f;
    k.yhi = 1.f;
  }
  return k;
}

// encoder (eval mode) for n (lhs, rel) sources -> Q [n][dp]
void encode_eval(kp_ctx* c, int n, const int2* dsrc, const float* dX, float* dQ) {
  if (n <= 0) return;
  CvConst k = make_const(c, nullptr);
  float* dflat = reinterpret_cast<float*>(c->ws[12].ensure(sizeof(float) * (size_t)n * c->hidden));
  float* dfc = reinterpret_cast<float*>(c->ws[13].ensure(sizeof(float) * (size_t)n * c->dim));
  KP_CONV_FWD(dim3(n), dim3(256), 0, c->stream, n, dsrc, c->dE, dX, c->dR, k, c->d_conv_w,
                     c->d_conv_b, c->d_bn_a, c->d_bn_b, nullptr, nullptr, dflat);
  KP_HIP(hipGetLastError());
  launch_gemm_abt(c, dflat, c->hidden, n, c->d_fc_w, c->hidden, c->dim, c->hidden, dfc, c->dim, c->d_fc_b, 0, 1);
  hipLaunchKernelGGL(kp_cv_post_fc, dim3(n), dim3(256), 0, c->stream, n, dfc, 1, k, nullptr, nullptr, c->d_bn_a,
                     c->d_bn_b, dQ);
  KP_HIP(hipGetLastError());
}

}  // namespace

float* conve_fc_wt(kp_ctx* c);

// kp_cv_fused.hpp's weight images (built once per context; the FC layer is frozen)
static void conve_fused_images(kp_ctx* c, const __bf16** fw, const __bf16** bw) {
  if (!c->cvf_ready) {
    const long long n1 = (long long)kpcvf::NR * kpcvf::HID, n2 = (long long)kpcvf::NBL * kpcvf::KB;
    __bf16* a = reinterpret_cast<__bf16*>(c->cvf_fw3.ensure(3 * sizeof(__bf16) * (size_t)n1));
    __bf16* b = reinterpret_cast<__bf16*>(c->cvf_bw3.ensure(3 * sizeof(__bf16) * (size_t)n2));
    hipLaunchKernelGGL(kpcvf::kp_cv_fwd_image, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_fc_w, c->dim, a);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL(kpcvf::kp_cv_bwd_image, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_fc_w, c->dim, b);
    KP_HIP(hipGetLastError());
    c->cvf_ready = true;
  }
  *fw = c->cvf_fw3.as<__bf16>();
  *bw = c->cvf_bw3.as<__bf16>();
}

void conve_encode_dev(kp_ctx* c, int n, const int2* d_src, float* d_out) { encode_eval(c, n, d_src, nullptr, d_out); }

// KP_HOST_TIMES=1 (diagnostic): per call, on stderr, the host time of the planning, the
// uploads, enqueueing the step loop, and the rank with the final wait
static const bool g_cv_host_times = std::getenv("KP_HOST_TIMES") != nullptr;
static double cv_host_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void conve_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* bt) {
  const double t_in = g_cv_host_times ? cv_host_ms() : 0.0;
  const int ns = bt->n_slots;
  const int K = c->n_ent;
  const int DP = c->dp;
  const int DBV = DP / 16;
  KP_REQUIRE(hp->batch_size >= 1 && hp->epochs >= 0, "ConvE: bad hyper-parameters");
  CvConst kc = make_const(c, hp);
  const int E_ = hp->epochs;

  // ---------------- host planning: er_vocab per slot (bce_optimizer.py:92-96)
  struct Pair {
    int h, r;
    std::vector<int> tails;
    int tail_begin = -1, tail_count = 0;  // kelpie pair: its distinct tails in `tails`; frozen: its FC row
  };
  std::vector<int2> fpairs;                // frozen (h, r) -> fc precompute
  std::unordered_map<long long, int> fp_id;
  std::vector<int32_t> tails;
  std::vector<CvInst> kinst;
  std::vector<CvFInst> finst;
  std::vector<CvAct> acts;
  // per slot: batches (pair ranges) and mask word offsets per step
  struct SlotPlan {
    std::vector<Pair> pairs;
    int nb = 0;
  };
  std::vector<SlotPlan> plan(ns);
  int T = 0;
  for (int s = 0; s < ns; ++s) {
    const int r0 = bt->row_off[s], r1 = bt->row_off[s + 1];
    KP_REQUIRE(r1 >= r0, "ConvE: bad row_off");
    std::unordered_map<long long, int> idx;
    auto& P = plan[s].pairs;
    for (int j = r0; j < r1; ++j) {
      const int h = bt->rows[3 * j], r = bt->rows[3 * j + 1], t = bt->rows[3 * j + 2];
      KP_REQUIRE(h >= 0 && h <= K && t >= 0 && t <= K && r >= 0 && r < c->n_rel2, "ConvE: row id out of range");
      const long long key = (long long)h * c->n_rel2 + r;
      auto it = idx.find(key);
      if (it == idx.end()) {
        idx.emplace(key, (int)P.size());
        P.push_back(Pair{h, r, {t}});
      } else {
        P[it->second].tails.push_back(t);
      }
    }
    plan[s].nb = P.empty() ? 0 : (int)((P.size() + hp->batch_size - 1) / hp->batch_size);
    T = std::max(T, E_ * plan[s].nb);
    for (auto& pr : P)
      if (pr.h != K) {
        for (int tt : pr.tails) KP_REQUIRE(tt == K, "ConvE: a training row does not involve the kelpie entity");
        const long long key = (long long)pr.h * c->n_rel2 + pr.r;
        if (!fp_id.count(key)) {
          fp_id.emplace(key, (int)fpairs.size());
          fpairs.push_back(make_int2(pr.h, pr.r));
        }
      }
  }
  // keep-bit offsets: per slot, steps in order; per step one word-aligned run per drawn
  // dropout, in the forward's order (input b x 2d, feature map b x 32, hidden b x d)
  struct StepBits {
    long long in, fm, hid;  // word offsets (-1: not drawn)
  };
  std::vector<std::vector<StepBits>> moff(ns);
  for (int s = 0; s < ns; ++s) {
    const int nb = plan[s].nb;
    const int P = (int)plan[s].pairs.size();
    long long off = bt->rng_off[s];
    for (int t = 0; t < E_ * nb; ++t) {
      const int j = t % nb;
      const long long b = std::min(hp->batch_size, P - j * hp->batch_size);
      StepBits sb{-1, -1, -1};
      if (kc.has_in) { sb.in = off; off += (b * 2 * c->dim + 31) / 32; }
      if (kc.has_fm) { sb.fm = off; off += (b * 32 + 31) / 32; }
      if (kc.has_mask) { sb.hid = off; off += (b * c->dim + 31) / 32; }
      moff[s].push_back(sb);
    }
    KP_REQUIRE(off <= bt->rng_off[s + 1], "ConvE: missing dropout keep bits");
  }
  auto pair_bits = [&](const StepBits& sb, int pos) {
    return CvBits{sb.in < 0 ? -1 : 32 * sb.in + (long long)pos * 2 * c->dim,
                  sb.fm < 0 ? -1 : 32 * sb.fm + (long long)pos * 32,
                  sb.hid < 0 ? -1 : 32 * sb.hid + (long long)pos * c->dim};
  };
  // per-step instance lists; the step's encoder rows (kelpie pairs, then with fr_step the
  // frozen-head pairs) with their keep-bit offsets
  std::vector<int> kin_off(T + 1, 0), fin_off(T + 1, 0), act_o(T + 1, 0), enc_off(T + 1, 0);
  std::vector<int2> enc_src;
  std::vector<CvBits> enc_bits;
  // the shared-encoder path's kelpie rows per step (one per slot with a kelpie pair in the
  // step: its source and its pairs' range in the step's list), and per kelpie pair (its
  // kelpie row, first pair of that row)
  std::vector<int> sr_off(T + 1, 0);
  // the frozen-head pairs' chunks per step (kp_cv_fgrad)
  std::vector<int> fch_off(T + 1, 0);
  std::vector<int4> fchunks;
  int max_fch = 0;
  std::vector<int2> sr_src, sr_rng, psr;
  int max_k = 0, max_enc = 0, max_sr = 0;
  for (int t = 0; t < T; ++t) {
    kin_off[t] = (int)kinst.size();
    fin_off[t] = (int)finst.size();
    act_o[t] = (int)acts.size();
    enc_off[t] = (int)enc_src.size();
    std::vector<int2> fr_hr;  // the step's frozen-head (h, r), with fr_step
    int local_k = 0;
    sr_off[t] = (int)sr_src.size();
    fch_off[t] = (int)fchunks.size();
    for (int s = 0; s < ns; ++s) {
      const int nb = plan[s].nb;
      if (nb == 0 || t >= E_ * nb) continue;
      const int j = t % nb;
      auto& P = plan[s].pairs;
      const int p0 = j * hp->batch_size, p1 = std::min((int)P.size(), p0 + hp->batch_size);
      const int b = p1 - p0;
      CvAct A{};
      A.slot = s;
      A.k_begin = local_k;
      A.f_begin = (int)finst.size() - fin_off[t];
      int my_sr = -1;
      for (int q = p0; q < p1; ++q) {
        auto& pr = P[q];
        if (pr.h == K) {
          const bool first = my_sr < 0;
          if (first) {
            my_sr = (int)sr_src.size() - sr_off[t];
            sr_src.push_back(make_int2(-s - 1, 0));
          }
          psr.push_back(make_int2(my_sr, first ? 1 : 0));
          CvInst I{};
          I.slot = s;
          I.rel = pr.r;
          I.b = b;
          I.pos = q - p0;
          I.mb = pair_bits(moff[s][t], I.pos);
          if (pr.tail_begin < 0) {  // the pair's distinct tails, stored once for every step
            pr.tail_begin = (int)tails.size();
            for (int tt : pr.tails)
              if (std::find(tails.begin() + pr.tail_begin, tails.end(), tt) == tails.end()) tails.push_back(tt);
            pr.tail_count = (int)tails.size() - pr.tail_begin;
          }
          I.tail_begin = pr.tail_begin;
          I.tail_count = pr.tail_count;
          kinst.push_back(I);
          ++local_k;
        } else {
          CvFInst F{};
          F.slot = s;
          if (!kc.fr_step && pr.tail_begin < 0) pr.tail_begin = fp_id.at((long long)pr.h * c->n_rel2 + pr.r);
          F.fp = kc.fr_step ? (int)finst.size() - fin_off[t] : pr.tail_begin;  // (frozen pair: its FC row)
          F.b = b;
          F.pos = q - p0;
          F.mb = pair_bits(moff[s][t], F.pos);
          finst.push_back(F);
          if (kc.fr_step) fr_hr.push_back(make_int2(pr.h, pr.r));
        }
      }
      A.k_count = local_k - A.k_begin;
      A.f_count = (int)finst.size() - fin_off[t] - A.f_begin;
      A.pad0 = (int)fchunks.size() - fch_off[t];
      A.pad1 = (A.f_count + FCH - 1) / FCH;
      for (int f = 0; f < A.f_count; f += FCH)
        fchunks.push_back(make_int4((int)acts.size() - act_o[t], f, std::min(FCH, A.f_count - f), 0));
      acts.push_back(A);
      if (my_sr >= 0) sr_rng.push_back(make_int2(A.k_begin, A.k_begin + A.k_count));
    }
    max_sr = std::max(max_sr, (int)sr_src.size() - sr_off[t]);
    max_fch = std::max(max_fch, (int)fchunks.size() - fch_off[t]);
    for (int i = kin_off[t]; i < (int)kinst.size(); ++i) {
      enc_src.push_back(make_int2(-kinst[i].slot - 1, kinst[i].rel));
      enc_bits.push_back(kinst[i].mb);
    }
    if (kc.fr_step)
      for (int i = fin_off[t]; i < (int)finst.size(); ++i) {
        finst[i].fp += local_k;  // its row in the step's encoder output, after the kelpie pairs
        enc_src.push_back(fr_hr[i - fin_off[t]]);
        enc_bits.push_back(finst[i].mb);
      }
    max_k = std::max(max_k, local_k);
    max_enc = std::max(max_enc, (int)enc_src.size() - enc_off[t]);
  }
  enc_off[T] = (int)enc_src.size();
  sr_off[T] = (int)sr_src.size();
  fch_off[T] = (int)fchunks.size();
  kin_off[T] = (int)kinst.size();
  fin_off[T] = (int)finst.size();
  act_o[T] = (int)acts.size();

  const double t_plan = g_cv_host_times ? cv_host_ms() : 0.0;
  // ---------------- uploads
  std::vector<float> xp((size_t)ns * DP, 0.f);
  for (int s = 0; s < ns; ++s) std::memcpy(&xp[(size_t)s * DP], bt->x0 + (size_t)s * c->dim, sizeof(float) * c->dim);
  float* dX = upload(c, c->ws[0], xp.data(), xp.size());
  float* dS1 = reinterpret_cast<float*>(c->ws[1].ensure(sizeof(float) * xp.size()));
  float* dS2 = reinterpret_cast<float*>(c->ws[2].ensure(sizeof(float) * xp.size()));
  KP_HIP(hipMemsetAsync(dS1, 0, sizeof(float) * xp.size(), c->stream));
  KP_HIP(hipMemsetAsync(dS2, 0, sizeof(float) * xp.size(), c->stream));
  CvInst* dKI = upload(c, c->ws[3], kinst.data(), std::max<size_t>(1, kinst.size()));
  CvFInst* dFI = upload(c, c->ws[4], finst.data(), std::max<size_t>(1, finst.size()));
  CvAct* dAct = upload(c, c->ws[5], acts.data(), std::max<size_t>(1, acts.size()));
  int32_t* dTails = upload(c, c->ws[6], tails.data(), std::max<size_t>(1, tails.size()));
  const int64_t nbits = bt->rng_off[ns];
  // the keep bits, plus one zero guard word (kp_cv_fwd_fused reads a row's input bits as
  // a 64-bit window)
  int32_t* dBits = reinterpret_cast<int32_t*>(c->ws[7].ensure(sizeof(int32_t) * (size_t)(nbits + 2)));
  if (nbits > 0)
    KP_HIP(hipMemcpyAsync(dBits, bt->rng, sizeof(int32_t) * (size_t)nbits, hipMemcpyHostToDevice, c->stream));
  KP_HIP(hipMemsetAsync(dBits + nbits, 0, 2 * sizeof(int32_t), c->stream));
  const int nfp = kc.fr_step ? 0 : (int)fpairs.size();

  const double t_up = g_cv_host_times ? cv_host_ms() : 0.0;
  KP_HIP(hipEventRecord(c->ev0, c->stream));
  // frozen-head pairs without an input / feature-map dropout: FC output (pre-dropout)
  // once per batch
  float* dFcf = reinterpret_cast<float*>(c->ws[8].ensure(sizeof(float) * (size_t)std::max(1, nfp) * c->dim));
  if (nfp > 0) {
    int2* dFp = upload(c, c->ws[9], fpairs.data(), fpairs.size());
    float* dflat = reinterpret_cast<float*>(c->ws[12].ensure(sizeof(float) * (size_t)nfp * c->hidden));
    KP_CONV_FWD(dim3(nfp), dim3(256), 0, c->stream, nfp, dFp, c->dE, dX, c->dR, kc,
                       c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, nullptr, nullptr, dflat);
    KP_HIP(hipGetLastError());
    launch_gemm_abt(c, dflat, c->hidden, nfp, c->d_fc_w, c->hidden, c->dim, c->hidden, dFcf, c->dim, c->d_fc_b, 0, 1);
  }
  // step workspaces
  // fused encoder kernels (kp_cv_fused.hpp) for d = 200: the feature map stays on chip
  const bool fused = c->cv_fused && c->dim == 200 && c->hidden == kpcvf::HID;
  const int KS = fused ? kpcvf::NSPLIT : 8;  // split-K of the FC forward
  const int mk = std::max(1, max_k);
  const int me = std::max(1, max_enc);  // encoder rows per step (kelpie pairs + per-step frozen pairs)
  float* dflat = reinterpret_cast<float*>(c->ws[12].ensure(sizeof(float) * (size_t)std::max(fused ? 1 : me, nfp) * c->hidden));
  float* dslab = reinterpret_cast<float*>(c->ws[13].ensure(sizeof(float) * (size_t)KS * me * c->dim));
  const __bf16* cvf_fw = nullptr;
  const __bf16* cvf_bw = nullptr;
  uint8_t* dRelu = nullptr;
  __bf16* dG3 = nullptr;
  if (fused) {
    conve_fused_images(c, &cvf_fw, &cvf_bw);
    dRelu = reinterpret_cast<uint8_t*>(c->ws[24].ensure((size_t)me * kpcvf::MASK_B));
    dG3 = reinterpret_cast<__bf16*>(c->ws[25].ensure(3 * sizeof(__bf16) * (size_t)mk * kpcvf::KB));
  }
  // the shared-encoder split (kp_cv_fused.hpp): kelpie rows' map rows 0-17 in NB_L bands,
  // the pairs' rows 18-19 in NB_M, the relations' rows 20-37 (once per context) in NB_L
  const bool shared = fused && c->cv_shared && !kc.has_in && !kc.has_fm;
  constexpr int NB_L = 24;
  const int msr = std::max(1, max_sr);
  int2* dSrSrc = nullptr;
  int2* dSrRng = nullptr;
  int2* dPsr = nullptr;
  uint8_t* dReluS = nullptr;
  float* dSlabL = nullptr;  // kelpie rows' FC split-K slabs [KSL][rows][dim]
  float* dMid = nullptr;    // pairs' map-row-18-19 FC terms [pairs][dim]
  float* dMapL = nullptr;   // kelpie rows' map rows 0-17, then (backward) g W_lhs
  float* dMapM = nullptr;   // pairs' map rows 18-19, then (backward) dfc W_mid [pairs][512]
  float* dGs = nullptr;     // kelpie rows' summed pair dfc
  float* dDls = nullptr;    // kelpie rows' lhs image gradient [rows][DP]
  if (shared) {
    if (!c->cv_shared_ready) {
      float* wtm = reinterpret_cast<float*>(c->cv_wtm.ensure(sizeof(float) * (size_t)c->dim * kpcvf::NMID));
      hipLaunchKernelGGL(kpcvf::kp_cv_mid_wt, dim3((c->dim * kpcvf::NMID + 255) / 256), dim3(256), 0, c->stream,
                         c->d_fc_w, c->dim, wtm);
      KP_HIP(hipGetLastError());
      float* wtl = reinterpret_cast<float*>(c->cv_wtl.ensure(sizeof(float) * (size_t)c->dim * kpcvf::NLHS));
      float* wlc = reinterpret_cast<float*>(c->cv_wlc.ensure(sizeof(float) * (size_t)c->dim * kpcvf::NLHS));
      float* wfm = reinterpret_cast<float*>(c->cv_wfm.ensure(sizeof(float) * (size_t)c->dim * kpcvf::NMID));
      const int nw = (kpcvf::NLHS + kpcvf::NMID) * c->dim;
      hipLaunchKernelGGL(kpcvf::kp_cv_lhs_wt, dim3((nw + 255) / 256), dim3(256), 0, c->stream, c->d_fc_w, c->dim, wlc,
                         wtl, wfm);
      KP_HIP(hipGetLastError());
      // the relations' FC terms: map rows 20-37 (the relation half only), no bias
      const int nr = c->n_rel2;
      std::vector<int2> rs(nr);
      for (int r = 0; r < nr; ++r) rs[r] = make_int2(0, r);
      DevBuf bs, bo;
      int2* dRs = upload(c, bs, rs.data(), rs.size());
      float* sl = reinterpret_cast<float*>(bo.ensure(sizeof(float) * (size_t)NB_L * nr * c->dim));
      const int g = NB_L * ((nr + kpcvf::MT - 1) / kpcvf::MT);
      hipLaunchKernelGGL(kpcvf::kp_cv_fwd_fused<false>, dim3(g), dim3(512), kpcvf::FWD_LDS, c->stream, nr, dRs, c->dE,
                         dX, c->dR, DP, c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, cvf_fw, nullptr, c->dim,
                         nullptr, dBits, 1.0f, 1.0f, sl, nullptr, 8 * (kpcvf::MID_Y + 2),
                         8 * (kpcvf::FR - kpcvf::MID_Y - 2), NB_L, 2);
      KP_HIP(hipGetLastError());
      float* tr = reinterpret_cast<float*>(c->cv_trel.ensure(sizeof(float) * (size_t)nr * c->dim));
      hipLaunchKernelGGL(kpcvf::kp_cv_slab_sum, dim3((nr * c->dim + 255) / 256), dim3(256), 0, c->stream, nr, NB_L,
                         c->dim, sl, tr);
      KP_HIP(hipGetLastError());
      KP_HIP(hipStreamSynchronize(c->stream));
      bs.release();
      bo.release();
      c->cv_shared_ready = true;
    }
    dSrSrc = upload(c, c->cvs[0], sr_src.data(), std::max<size_t>(1, sr_src.size()));
    dSrRng = upload(c, c->cvs[1], sr_rng.data(), std::max<size_t>(1, sr_rng.size()));
    dPsr = upload(c, c->cvs[2], psr.data(), std::max<size_t>(1, psr.size()));
    dReluS = reinterpret_cast<uint8_t*>(c->cvs[3].ensure((size_t)msr * kpcvf::MASK_B));
    KP_HIP(hipMemsetAsync(dReluS, 0, (size_t)msr * kpcvf::MASK_B, c->stream));  // rows 18-19 stay 0
    dSlabL = reinterpret_cast<float*>(c->cvs[4].ensure(sizeof(float) * (size_t)kpcvf::KSL * msr * c->dim));
    dMapM = reinterpret_cast<float*>(c->cvs[9].ensure(sizeof(float) * (size_t)mk * kpcvf::NMID));
    dMid = reinterpret_cast<float*>(c->cvs[5].ensure(sizeof(float) * (size_t)mk * c->dim));
    dMapL = reinterpret_cast<float*>(c->cvs[6].ensure(sizeof(float) * (size_t)msr * kpcvf::NLHS));
    dGs = reinterpret_cast<float*>(c->cvs[7].ensure(sizeof(float) * (size_t)msr * c->dim));
    dDls = reinterpret_cast<float*>(c->cvs[8].ensure(sizeof(float) * (size_t)msr * DP));
  }
  const int n_dl = fused ? kpcvf::NSPLIT : 1;  // lhs image-gradient slabs per pair (kp_cv_bwd_fused, reduced in slab 0)
  float* dQ = reinterpret_cast<float*>(c->ws[14].ensure(sizeof(float) * (size_t)me * DP));
  int2* dSrc = upload(c, c->ws[15], enc_src.data(), std::max<size_t>(1, enc_src.size()));
  int4* dFch = upload(c, c->cvs[10], fchunks.data(), std::max<size_t>(1, fchunks.size()));
  float* dFpart = reinterpret_cast<float*>(c->ws[31].ensure(sizeof(float) * (size_t)std::max(1, max_fch) * c->dim));
  CvBits* dEncBits = upload(c, c->ws[26], enc_bits.data(), std::max<size_t>(1, enc_bits.size()));
  float* dgs = reinterpret_cast<float*>(c->ws[16].ensure(sizeof(float) * (size_t)std::max<size_t>(1, kinst.size())));
  {
    std::vector<float> gsv(kinst.size());
    for (size_t i = 0; i < kinst.size(); ++i) gsv[i] = 1.0f / (float)((long long)kinst[i].b * (long long)(K + 1));
    if (!gsv.empty())
      KP_HIP(hipMemcpyAsync(dgs, gsv.data(), sizeof(float) * gsv.size(), hipMemcpyHostToDevice, c->stream));
  }
  int attn_slots = c->n_cu * (DBV <= 13 ? 2 : 1);  // co-resident attention workgroups
  if (c->attn_mode == 1) {
    switch (DBV) {
      case 4: attn_slots = c->n_cu * attn3_wpc<4, ATT_BCE_O>(c); break;
      case 8: attn_slots = c->n_cu * attn3_wpc<8, ATT_BCE_O>(c); break;
      case 13: attn_slots = c->n_cu * attn3_wpc<13, ATT_BCE_O>(c); break;
      case 16: attn_slots = c->n_cu * attn3_wpc<16, ATT_BCE_O>(c); break;
      case 25: attn_slots = c->n_cu * attn3_wpc<25, ATT_BCE_O>(c); break;
      default: throw KpError{KP_ENOTSUP, "ConvE: unsupported padded dimension"};
    }
  }
  std::vector<AttnPlan> step_plan(T);
  size_t o_rows = 1;
  for (int t = 0; t < T; ++t) {
    const int nk = kin_off[t + 1] - kin_off[t];
    step_plan[t] = attn_plan_ctx(c, std::max(nk, 1), K, attn_slots);
    o_rows = std::max(o_rows, (size_t)nk * step_plan[t].wk.n_parts);
  }
  float* dO = reinterpret_cast<float*>(c->ws[17].ensure(sizeof(float) * o_rows * DP));
  float* ddfc = reinterpret_cast<float*>(c->ws[18].ensure(sizeof(float) * (size_t)mk * c->dim));
  float* dgk = reinterpret_cast<float*>(c->ws[19].ensure(sizeof(float) * (size_t)mk));
  float* ddflat = reinterpret_cast<float*>(c->ws[20].ensure(sizeof(float) * (size_t)(fused ? 1 : mk) * c->hidden));
  float* ddl = reinterpret_cast<float*>(c->ws[21].ensure(sizeof(float) * (size_t)n_dl * mk * DP));
  float* dWt = conve_fc_wt(c);
  // the masks' multipliers as the fused kernels take them (1: not drawn)
  const float s_in = kc.has_in ? kc.scale_in : 1.0f, s_fm = kc.has_fm ? kc.scale_fm : 1.0f;

  CvOpt opt{};
  opt.lr = hp->lr;
  opt.b1 = hp->beta1;
  opt.b2 = hp->beta2;
  opt.eps = hp->eps;
  opt.one_minus_b1 = (float)(1.0 - (double)hp->beta1);
  opt.one_minus_b2 = (float)(1.0 - (double)hp->beta2);
  double hot = 0.0, work = 0.0;
  int64_t launches = 0;
  c->hot_pairs.clear();
  c->hot_iv.clear();
  const size_t shm_attn = attn_lds_bytes(DP / 16);
  const size_t shm_cbwd = sizeof(float) * 32 * 20 * (c->dim / 20 - 2);
  for (int t = 0; t < T; ++t) {
    const int nk = kin_off[t + 1] - kin_off[t];
    const int ne = enc_off[t + 1] - enc_off[t];  // nk kelpie rows first
    const int na = act_o[t + 1] - act_o[t];
    const CvInst* KI = dKI + kin_off[t];
    const int2* ES = dSrc + enc_off[t];
    const CvBits* EB = dEncBits + enc_off[t];
    const int nsr = sr_off[t + 1] - sr_off[t];
    if (ne > 0 && shared) {  // encoder forward, shared split (kp_cv_fused.hpp); ne == nk here
      hipLaunchKernelGGL(kpcvf::kp_cv_lhs_map, dim3(nsr), dim3(256), 0, c->stream, nsr, dSrSrc + sr_off[t], dX, DP,
                         c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, dMapL, dReluS);
      KP_HIP(hipGetLastError());
      launch_gemm_abt(c, dMapL, kpcvf::NLHS, nsr, c->cv_wlc.as<float>(), kpcvf::NLHS, c->dim, kpcvf::NLHS, dSlabL,
                      c->dim, c->d_fc_b, 0, kpcvf::KSL);
      hipLaunchKernelGGL(kpcvf::kp_cv_mid_map, dim3((ne * kpcvf::CH * 2 + 255) / 256), dim3(256), 0, c->stream, ne, ES,
                         c->dE, dX, c->dR, DP, c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, dMapM, dRelu);
      KP_HIP(hipGetLastError());
      launch_gemm_abt(c, dMapM, kpcvf::NMID, ne, c->cv_wtm.as<float>(), kpcvf::NMID, c->dim, kpcvf::NMID, dMid, c->dim,
                      nullptr, 0, 1);
      hipLaunchKernelGGL(kp_cv_post_fc3, dim3(ne), dim3(256), 0, c->stream, ne, dSlabL, kpcvf::KSL, nsr, dMid, 1,
                         c->cv_trel.as<float>(), ES, dPsr + kin_off[t], kc, EB, dBits, c->d_bn_a, c->d_bn_b, dQ);
      KP_HIP(hipGetLastError());
    } else if (ne > 0) {  // encoder forward (conve.py:133-153, train-mode dropouts)
      if (fused) {
        const int fgrid = kpcvf::NSPLIT * ((ne + kpcvf::MT - 1) / kpcvf::MT);
        if (kc.fr_step)
          hipLaunchKernelGGL(kpcvf::kp_cv_fwd_fused<true>, dim3(fgrid), dim3(512), kpcvf::FWD_LDS, c->stream, ne, ES,
                             c->dE, dX, c->dR, DP, c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, cvf_fw, c->d_fc_b,
                             c->dim, EB, dBits, s_in, s_fm, dslab, dRelu, 0, kpcvf::FR * 8,
                             kpcvf::NSPLIT, 8);
        else
          hipLaunchKernelGGL(kpcvf::kp_cv_fwd_fused<false>, dim3(fgrid), dim3(512), kpcvf::FWD_LDS, c->stream, ne, ES,
                             c->dE, dX, c->dR, DP, c->d_conv_w, c->d_conv_b, c->d_bn_a, c->d_bn_b, cvf_fw, c->d_fc_b,
                             c->dim, EB, dBits, s_in, s_fm, dslab, dRelu, 0, kpcvf::FR * 8,
                             kpcvf::NSPLIT, 8);
        KP_HIP(hipGetLastError());
      } else {
        KP_CONV_FWD(dim3(ne), dim3(256), 0, c->stream, ne, ES, c->dE, dX, c->dR, kc, c->d_conv_w, c->d_conv_b,
                    c->d_bn_a, c->d_bn_b, EB, dBits, dflat);
        KP_HIP(hipGetLastError());
        launch_gemm_abt(c, dflat, c->hidden, ne, c->d_fc_w, c->hidden, c->dim, c->hidden, dslab, c->dim, c->d_fc_b, 0,
                        KS);
      }
      hipLaunchKernelGGL(kp_cv_post_fc, dim3(ne), dim3(256), 0, c->stream, ne, dslab, KS, kc, EB, dBits, c->d_bn_a,
                         c->d_bn_b, dQ);
      KP_HIP(hipGetLastError());
    }
    if (nk > 0) {
      const int n_split = step_plan[t].wk.n_parts;
      hipEvent_t ea = nullptr, eb = nullptr;
      if (c->time_hot) {
        ea = c->event(2 * launches);
        eb = c->event(2 * launches + 1);
        KP_HIP(hipEventRecord(ea, c->stream));
      }
      dim3 grid(step_plan[t].n_wg);
#define CV_ATT(DBX)                                                                                                  \
  if (c->attn_mode == 1)                                                                                             \
    launch_attn3<DBX, ATT_BCE_O>(c, K, dQ, nk, step_plan[t], nullptr, nullptr, dO, dgs + kin_off[t], kc.ylo);       \
  else                                                                                                               \
    hipLaunchKernelGGL((kp_attn<DBX, ATT_BCE_O>), grid, dim3(256), shm_attn, c->stream, c->dE, K, dQ, nk,          \
                       step_plan[t].wk,                                                                               \
                       nullptr, nullptr, dO, dgs + kin_off[t], kc.ylo)
      switch (DBV) {
        case 4: CV_ATT(4); break;
        case 8: CV_ATT(8); break;
        case 13: CV_ATT(13); break;
        case 16: CV_ATT(16); break;
        case 25: CV_ATT(25); break;
        default: throw KpError{KP_ENOTSUP, "ConvE: unsupported padded dimension"};
      }
#undef CV_ATT
      KP_HIP(hipGetLastError());
      if (c->time_hot) {
        KP_HIP(hipEventRecord(eb, c->stream));
        c->hot_pairs.push_back({(double)nk, 0.0});
      }
      ++launches;
      {
        __bf16* g3p = shared ? nullptr : dG3;
        const int nj = (c->dp + 63) / 64;
#define CV_DX1(J)                                                                                                  \
  hipLaunchKernelGGL(kp_cv_dx1<J>, dim3(nk), dim3(64), 0, c->stream, nk, kc, KI, dQ, dO, n_split, dTails, c->dE, dX, \
                     dBits, c->d_bn_a, ddfc, dgk, g3p)
        if (!c->cv_dx_block && nj <= 2)
          CV_DX1(2);
        else if (!c->cv_dx_block && nj <= 4)
          CV_DX1(4);
        else if (!c->cv_dx_block && nj <= 6)
          CV_DX1(6);
        else if (!c->cv_dx_block && nj <= 8)
          CV_DX1(8);
        else
          hipLaunchKernelGGL(kp_cv_dx, dim3(nk), dim3(256), 0, c->stream, nk, kc, KI, dQ, dO, n_split, dTails, c->dE,
                             dX, dBits, c->d_bn_a, ddfc, dgk, g3p);
#undef CV_DX1
      }
      KP_HIP(hipGetLastError());
      if (shared) {
        // map rows 0-17 once per kelpie row (the sum of its pairs' dfc; rows 18-19 of its
        // ReLU bytes are 0), then rows 18-19 per pair, assembled into the pairs' dl rows
        hipLaunchKernelGGL(kpcvf::kp_cv_slot_g, dim3(nsr), dim3(256), 0, c->stream, nsr, dSrRng + sr_off[t], ddfc,
                           c->dim, dGs);
        KP_HIP(hipGetLastError());
        launch_gemm_abt(c, dGs, c->dim, nsr, c->cv_wtl.as<float>(), c->dim, kpcvf::NLHS, c->dim, dMapL, kpcvf::NLHS,
                        nullptr, 0, 1);
        hipLaunchKernelGGL(kpcvf::kp_cv_lhs_convt, dim3(nsr), dim3(256), 0, c->stream, nsr, dMapL, dReluS, c->d_conv_w,
                           c->d_bn_a, DP, dDls);
        KP_HIP(hipGetLastError());
        launch_gemm_abt(c, ddfc, c->dim, nk, c->cv_wfm.as<float>(), c->dim, kpcvf::NMID, c->dim, dMapM, kpcvf::NMID,
                        nullptr, 0, 1);
        hipLaunchKernelGGL(kpcvf::kp_cv_mid_convt, dim3((nk + kpcvf::MPW - 1) / kpcvf::MPW), dim3(256), 0, c->stream, nk,
                           dMapM, dRelu, c->d_conv_w, c->d_bn_a, dPsr + kin_off[t], dDls, DP, ddl);
        KP_HIP(hipGetLastError());
      } else if (fused) {
        const int bgrid = kpcvf::NSPLIT * ((nk + kpcvf::MT - 1) / kpcvf::MT);
        hipLaunchKernelGGL(kpcvf::kp_cv_bwd_fused, dim3(bgrid), dim3(512), kpcvf::BWD_LDS, c->stream, nk, dG3,
                           cvf_bw, dRelu, c->d_conv_w, c->d_bn_a, s_fm, DP, ddl);
        KP_HIP(hipGetLastError());
        const long long nr = (long long)nk * kpcvf::LR * kpcvf::IW;
        hipLaunchKernelGGL(kpcvf::kp_cv_dl_reduce, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, c->stream, nk, DP,
                           kc.has_in ? EB : nullptr, dBits, s_in, ddl);
        KP_HIP(hipGetLastError());
      } else {
        launch_gemm_abt(c, ddfc, c->dim, nk, dWt, c->dim, c->hidden, c->dim, ddflat, c->hidden, nullptr, 0, 1);
      }
      if (!fused) {
        hipLaunchKernelGGL(kp_cv_conv_bwd, dim3(nk), dim3(256), shm_cbwd, c->stream, nk, kc, ddflat, dflat, c->d_conv_w,
                           c->d_bn_a, EB, dBits, ddl);
        KP_HIP(hipGetLastError());
      }
    }
    const double step = (double)(t + 1);
    opt.step_size = (float)((double)hp->lr / (1.0 - std::pow((double)hp->beta1, step)));
    opt.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)hp->beta2, step));
    if (na > 0) {
      // dAct entries index kinst/finst relative to this step's lists; the frozen-head pairs
      // read their encodings from dQ (fr_step) or the batch's FC rows
      const int nch = fch_off[t + 1] - fch_off[t];
      if (nch > 0) {
        hipLaunchKernelGGL(kp_cv_fgrad, dim3(nch), dim3(256), 0, c->stream, kc, dFch + fch_off[t], dAct + act_o[t],
                           dFI + fin_off[t], kc.fr_step ? dQ : dFcf, dBits, c->d_bn_a, c->d_bn_b, dX, dFpart);
        KP_HIP(hipGetLastError());
      }
      hipLaunchKernelGGL(kp_cv_update, dim3(na), dim3(256), 0, c->stream, kc, dAct + act_o[t], dQ, dgk, ddl, dFpart,
                         dX, dS1, dS2, opt);
      KP_HIP(hipGetLastError());
    }
  }

  const double t_loop = g_cv_host_times ? cv_host_ms() : 0.0;
  // ---------------- rank: sigmoid(enc(x, R_p) . E_e), kelpie column, maximizer
  std::vector<int2> rsrc(ns);
  std::vector<int32_t> po(ns);
  for (int s = 0; s < ns; ++s) {
    KP_REQUIRE(bt->pred[3 * s] == K, "ConvE: the ranked triple must start at the kelpie entity");
    KP_REQUIRE(bt->pred[3 * s + 1] >= 0 && bt->pred[3 * s + 1] < c->n_rel2, "ConvE: ranked relation out of range");
    KP_REQUIRE(bt->pred[3 * s + 2] >= 0 && bt->pred[3 * s + 2] <= K, "ConvE: ranked object out of range");
    rsrc[s] = make_int2(-s - 1, bt->pred[3 * s + 1]);
    po[s] = bt->pred[3 * s + 2];
  }
  int2* dRsrc = upload(c, c->ws[11], rsrc.data(), rsrc.size());
  float* dQr = reinterpret_cast<float*>(c->ws[14].ensure(sizeof(float) * (size_t)std::max(ns, mk) * DP));
  encode_eval(c, ns, dRsrc, dX, dQr);
  int32_t* dPo = upload(c, c->ws[22], po.data(), po.size());
  int32_t* dFo = upload(c, c->ws[23], bt->filt_off, (size_t)ns + 1);
  // context buffers (a per-call buffer's hipFree waits for the whole device, every context)
  int32_t* dF = upload(c, c->cvs[11], bt->filt, (size_t)std::max(1, bt->filt_off[ns]));
  float* dTarget = reinterpret_cast<float*>(c->cvs[12].ensure(sizeof(float) * ns));
  int64_t* dRank = reinterpret_cast<int64_t*>(c->cvs[13].ensure(sizeof(int64_t) * ns));
  if (c->cv_rank64) {
    double* dQ64 = reinterpret_cast<double*>(c->ws[29].ensure(sizeof(double) * (size_t)ns * DP));
    double* dT64 = reinterpret_cast<double*>(c->ws[30].ensure(sizeof(double) * 2 * (size_t)ns));
    hipLaunchKernelGGL(kp_cv_rankq64, dim3(ns), dim3(64), 0, c->stream, dQr, dX, c->dE, K, DP, dPo, ns, dQ64, dT64,
                       dT64 + ns);
    KP_HIP(hipGetLastError());
    launch_rank_f64(c, ns, dQ64, dT64, dT64 + ns, dPo, dFo, dF, dTarget, dRank, RANK64_SIGMOID);
  } else {
    const int ld = round_up(K + 1, 4);
    float* dScores = reinterpret_cast<float*>(c->ws[10].ensure(sizeof(float) * (size_t)ns * ld));
    launch_score_gemm(c, dQr, ns, dScores, ld, 1);
    hipLaunchKernelGGL(kp_cv_kcol, dim3(ns), dim3(64), 0, c->stream, ns, kc, dQr, dX, dScores, ld);
    KP_HIP(hipGetLastError());
    launch_rank_count(c, ns, dScores, ld, K + 1, dPo, dFo, dF, 0, dTarget, dRank);
  }
  KP_HIP(hipEventRecord(c->ev1, c->stream));
  if (bt->out_x) KP_HIP(hipMemcpyAsync(xp.data(), dX, sizeof(float) * xp.size(), hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipMemcpyAsync(bt->out_score, dTarget, sizeof(float) * ns, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipMemcpyAsync(bt->out_rank, dRank, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  if (g_cv_host_times)
    std::fprintf(stderr, "[kp_cv] slots %d steps %d pairs %zu: plan %.2f ms, uploads %.2f ms, loop enqueue %.2f ms, "
                 "rank + wait %.2f ms\n", ns, T, kinst.size(), t_plan - t_in, t_up - t_plan, t_loop - t_up,
                 cv_host_ms() - t_loop);
  if (bt->out_x)
    for (int s = 0; s < ns; ++s) std::memcpy(bt->out_x + (size_t)s * c->dim, &xp[(size_t)s * DP], sizeof(float) * c->dim);
  float ms_all = 0.f;
  KP_HIP(hipEventElapsedTime(&ms_all, c->ev0, c->ev1));
  for (size_t i = 0; i < c->hot_pairs.size(); ++i) {
    float ms = 0.f;
    KP_HIP(hipEventElapsedTime(&ms, c->event(2 * i), c->event(2 * i + 1)));
    hot += ms * 1e-3;
    kp_push_interval(c, c->event(2 * i), c->event(2 * i + 1));
    work += c->hot_pairs[i].first * (double)K;
  }
  c->timing.device_s = ms_all * 1e-3;
  c->timing.loop_s = ms_all * 1e-3;
  c->timing.hot_s = hot;
  c->timing.hot_launches = launches;
  c->timing.hot_work = work;
}

float* conve_fc_wt(kp_ctx* c) {
  // FC weight transposed [hidden][dim] for the backward GEMM (built once, kept in the context)
  if (!c->dEt) {
    std::vector<float> w((size_t)c->dim * c->hidden), wt((size_t)c->dim * c->hidden);
    KP_HIP(hipMemcpy(w.data(), c->d_fc_w, sizeof(float) * w.size(), hipMemcpyDeviceToHost));
    for (int o = 0; o < c->dim; ++o)
      for (int j = 0; j < c->hidden; ++j) wt[(size_t)j * c->dim + o] = w[(size_t)o * c->hidden + j];
    KP_HIP(hipMalloc(&c->dEt, sizeof(float) * wt.size()));
    KP_HIP(hipMemcpy(c->dEt, wt.data(), sizeof(float) * wt.size(), hipMemcpyHostToDevice));
  }
  return c->dEt;
}

void conve_scores_dev(kp_ctx* c, int n, const int32_t* d_heads, const int32_t* d_rels, float* d_out, int ld) {
  if (n <= 0) return;
  std::vector<int32_t> h(n), r(n);
  KP_HIP(hipMemcpyAsync(h.data(), d_heads, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipMemcpyAsync(r.data(), d_rels, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  std::vector<int2> src(n);
  for (int i = 0; i < n; ++i) src[i] = make_int2(h[i], r[i]);
  DevBuf bs, bq;
  int2* dsrc = upload(c, bs, src.data(), src.size());
  float* dQ = reinterpret_cast<float*>(bq.ensure(sizeof(float) * (size_t)n * c->dp));
  encode_eval(c, n, dsrc, nullptr, dQ);
  launch_gemm_abt(c, dQ, c->dp, n, c->dE, c->dp, c->n_ent, c->dp, d_out, ld, nullptr, 1, 1);
  KP_HIP(hipStreamSynchronize(c->stream));
  bs.release();
  bq.release();
}

void conve_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out) {
  if (n <= 0) return;
  DevBuf bh, br, bs;
  int32_t* dh = upload(c, bh, heads, (size_t)n);
  int32_t* dr = upload(c, br, rels, (size_t)n);
  float* dS = reinterpret_cast<float*>(bs.ensure(sizeof(float) * (size_t)n * c->n_ent));
  conve_scores_dev(c, n, dh, dr, dS, c->n_ent);
  KP_HIP(hipMemcpyAsync(out, dS, sizeof(float) * (size_t)n * c->n_ent, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  for (DevBuf* b : {&bh, &br, &bs}) b->release();
}

#ifdef KP_ATTN_STAMPS
// the ConvE translation unit's copy of kpattn::g_attn_stamps (device globals are per code object)
extern "C" int kp_debug_attn_stamps_conve(unsigned long long* out, int reset) {
  KP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(kpattn::g_attn_stamps), sizeof(unsigned long long) * 8));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    KP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kpattn::g_attn_stamps), z, sizeof(z)));
  }
  return 0;
}
#endif
