// kp_cv_fused.hpp -- ConvE encoder forward and backward of the post-training step loop
// with the 9,728-wide feature map kept on chip (d = 200), for gfx950.
//
// Reference layers (src/link_prediction/models/conve.py:133-158): the image is the
// kelpie row and the relation row as two 20 x 10 halves -> BN1 -> conv 3x3 (32 channels,
// no padding: 38 x 8 maps) -> BN2 -> ReLU -> flatten (c, y, x) -> FC (200 x 9728).
// The unfused loop (kp_conve.hip) writes the flattened map of every kelpie pair to HBM
// (kp_cv_conv_fwd), reads it back in the FC GEMM and again in the backward
// (kp_cv_conv_bwd, for the ReLU mask), and writes / reads the 9,728-wide gradient of the
// map between the FC^T GEMM and the transposed convolution: 4 x 39 KB per pair per step.
// Here:
//
// kp_cv_fwd_fused: workgroup = 128 pairs (8 waves x 16) x one band of feature-map rows
// (split-K: the FC reduction runs over a band's 32 channels x rows x 8 columns).  A lane
// computes, per 32-deep k step, the 8 map columns of one channel at one row for its pair
// straight into its MFMA A operand (bf16x3 pieces, the operand layout of
// v_mfma_f32_16x16x32_bf16: lane (g, c) = row c, k = 8 g .. 8 g + 7 -> channel 4 cg + g,
// columns 0..7); the FC weights arrive as a split image permuted to that k order and are
// staged through LDS (two stages, one barrier per k step).  The map never leaves the
// registers; the ReLU signs of the rows the backward needs (rows < 20: the lhs half) are
// kept as one byte per (pair, channel, row).  Output: split-K slabs for kp_cv_post_fc.
//
// kp_cv_bwd_fused: workgroup = 128 pairs x two channels.  Per channel: the gradient of
// the 20 x 8 map rows the kelpie half feeds (5,120 of 9,728 columns: rows >= 20 only
// reach the frozen relation half) = dfc (bf16x3, 224-deep) . W_c^T on MFMA, masked by the
// stored ReLU signs and BN2 in registers, parked in LDS, and run through the transposed
// 3x3 convolution into per-thread accumulators of the 20 x 10 lhs image gradient.
// Output: one partial image gradient per channel group (16 slabs), summed by kp_cv_update.
//
// Train-mode dropouts (conve.py:142,147; the masks are host-drawn keep bits, a pair's
// CvBits row gives the bit offsets, -1 = not drawn): the input mask multiplies each
// image row as it enters the window (after BN1); the feature-map mask multiplies the
// ReLU output of a dropped-or-kept channel, and a dropped channel's ReLU bits are stored
// as 0, so the backward's mask covers both and it only applies the kept scale; the input
// mask of the lhs half is applied to the reduced image gradient (kp_cv_dl_reduce).
//
// XCD-aware: blockIdx b runs on XCD b % 8; both kernels give XCD x the bands / channel
// groups x and x + 8, so each XCD's 4 MB L2 holds only its slices of the weight images
// (forward ~1.5 MB of 12 MB, backward ~0.9 MB of 6.9 MB).
#pragma once

#include "kp_common.hpp"
#include "kp_attn3.hpp"

namespace kpcvf {

using kpattn::bf16x8;

// bit offsets of one pair's dropout keep bits in a batch's draws (-1: that dropout is
// not drawn): input image (2 d bits, row-major 40 x d/20), feature-map channels (32),
// hidden units (d)
struct CvBits {
  long long in, fm, hid;
};

constexpr int CH = 32;                // conv channels
constexpr int IW = 10;                // image width (d = 200: 20 x 10 per half)
constexpr int FW = 8;                 // feature-map width
constexpr int FR = 38;                // feature-map rows (40 - 2)
constexpr int HID = CH * FR * FW;     // 9728
constexpr int LR = 20;                // map rows that reach the lhs half
constexpr int NR = 208;               // FC outputs padded to 13 x 16
constexpr int NBF = NR / 16;          // 13 output blocks per wave (forward)
constexpr int KB = 224;               // backward reduction depth (200 padded to 7 x 32)
constexpr int NBL = CH * LR * FW;     // 5120 backward columns
constexpr int NBB = LR * FW / 16;     // 10 output blocks per channel (backward)
constexpr int NSPLIT = 16;            // forward bands = backward channel groups
constexpr int CGRP = CH / NSPLIT;     // 2 channels per backward workgroup
constexpr int MT = 128;               // pairs per workgroup (8 waves x 16)
constexpr int RS = 48;                // LDS row stride in bf16 (96 B: conflict-free ds_read_b128)
constexpr int MASK_B = CH * LR;       // ReLU sign bytes per pair (bit x = map column x)
constexpr int DCS = 164;              // LDS row stride (floats) of the parked map gradient
constexpr size_t FWD_LDS = 2u * 3u * NR * RS * sizeof(__bf16);     // 119,808 B
constexpr size_t BWD_LDS = 2u * 3u * LR * FW * RS * sizeof(__bf16);  // 92,160 B
static_assert(MT * DCS * sizeof(float) <= BWD_LDS, "the parked map gradient must fit the B stages");

// band z of the forward: feature-map rows [band_y0(z), band_y0(z + 1)) (2 or 3 rows)
__host__ __device__ constexpr int band_y0(int z) { return (FR * z) / NSPLIT; }

// the permuted k order of the forward weight image: k' = 256 y + 32 cg + 8 cl + x holds
// flat column (4 cg + cl) * 304 + 8 y + x
__host__ __device__ constexpr int fwd_flat(int kp) {
  return (4 * ((kp & 255) >> 5) + ((kp >> 3) & 3)) * (FR * FW) + (kp >> 8) * FW + (kp & 7);
}

// blockIdx -> (band / channel group, 128-pair tile); XCD b % 8 owns groups x and x + 8
__device__ __forceinline__ void xcd_map(int b, int& z, int& mt) {
  const int x = b & 7, j = b >> 3;
  z = x + 8 * (j & 1);
  mt = j >> 1;
}
// the same for nb bands (a multiple of 8): XCD x owns bands x, x + 8, x + 16, ...
__device__ __forceinline__ void xcd_map_n(int b, int nb, int& z, int& mt) {
  const int x = b & 7, j = b >> 3, per = nb >> 3;
  z = x + 8 * (j % per);
  mt = j / per;
}

// W [dim][HID] fp32 -> forward image [3][NR][HID] (k' order) and backward image
// [3][NBL][KB] (row = 160 c + 8 y + x, y < 20; column = FC output; zero padded)
__global__ void kp_cv_fwd_image(const float* __restrict__ W, int dim, __bf16* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)NR * HID) return;
  const int n = (int)(i / HID), kp = (int)(i % HID);
  const float v = n < dim ? W[(size_t)n * HID + fwd_flat(kp)] : 0.f;
  __bf16 h, m, l;
  kpattn::split3(v, h, m, l);
  const size_t ps = (size_t)NR * HID;
  out[i] = h;
  out[ps + i] = m;
  out[2 * ps + i] = l;
}

__global__ void kp_cv_bwd_image(const float* __restrict__ W, int dim, __bf16* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)NBL * KB) return;
  const int row = (int)(i / KB), k = (int)(i % KB);
  const int ch = row / (LR * FW), rr = row % (LR * FW);
  const int o = ch * (FR * FW) + rr;  // rows < 20 of channel ch: 8 y + x
  const float v = k < dim ? W[(size_t)k * HID + o] : 0.f;
  __bf16 h, m, l;
  kpattn::split3(v, h, m, l);
  const size_t ps = (size_t)NBL * KB;
  out[i] = h;
  out[ps + i] = m;
  out[2 * ps + i] = l;
}

// forward: out[z][i][n] = sum over band z of map_i[k] W[n][k] (+ fc bias in band 0 when
// fcb is given); relu[i][20 ch + y] = ReLU signs of row y < 20 of channel ch.
// The k steps (32 deep: one map row y and one group of four channels cg, q = 8 y + cg)
// [q_lo, q_lo + n_q) are cut into n_band bands (a multiple of 8) on multiples of gran
// steps (even): the whole map is (0, 304, 16, 8), 16 bands of whole rows; the shared-
// encoder path (kp_conve.hip) runs the kelpie rows' map rows 0-17, the pairs' rows 18-19
// and the relations' rows 20-37 apart.
// DROP: the input / feature-map dropout code is compiled in (the model has one of them)
template <bool DROP>
__global__ __launch_bounds__(512) void kp_cv_fwd_fused(int M, const int2* __restrict__ src,
                                                       const float* __restrict__ E, const float* __restrict__ X,
                                                       const float* __restrict__ R, int dp,
                                                       const float* __restrict__ cw, const float* __restrict__ cb,
                                                       const float* __restrict__ bna, const float* __restrict__ bnb,
                                                       const __bf16* __restrict__ W3, const float* __restrict__ fcb,
                                                       int dim, const CvBits* __restrict__ mb,
                                                       const int32_t* __restrict__ bits, float s_in, float s_fm,
                                                       float* __restrict__ out, uint8_t* __restrict__ relu,
                                                       int q_lo, int n_q, int n_band, int gran) {
  extern __shared__ __attribute__((aligned(16))) __bf16 bsh[];  // [stage][piece][NR][RS]
  __shared__ float sw[CH * 9], sc[CH], sa[CH], sbb[CH];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  int z, mt;
  xcd_map_n(blockIdx.x, n_band, z, mt);
  const int m0 = mt * MT;
  if (m0 >= M) return;  // whole-workgroup exit (uniform), before any barrier
  for (int j = tid; j < CH * 9; j += 512) sw[j] = cw[j];
  if (tid < CH) {
    sc[tid] = cb[tid];
    sa[tid] = bna[1 + tid];
    sbb[tid] = bnb[1 + tid];
  }
  // the lane's pair (rows past M compute a clamped pair and store nothing)
  const int i = m0 + 16 * w + c;
  const bool ok = i < M;
  const int2 s = src[ok ? i : M - 1];
  const float* lhs = s.x >= 0 ? E + (size_t)s.x * dp : X + (size_t)(-s.x - 1) * dp;
  const float* rel = R + (size_t)s.y * dp;
  const float a1 = bna[0], b1 = bnb[0];
  // the pair's dropout keep bits: the input image (bit 10 r + x of row r) and the 32
  // feature-map channels (one word: its run starts on a multiple of 32)
  const CvBits pb = DROP ? mb[ok ? i : M - 1] : CvBits{-1, -1, -1};
  const uint32_t fm_keep = DROP && pb.fm >= 0 ? (uint32_t)bits[pb.fm >> 5] : 0xffffffffu;
  const bool fm_on = DROP && pb.fm >= 0;
  // BN1 then the input dropout of image row r (conve.py:141-142), in place
  auto bn1_row = [&](int r, float (&o)[IW]) __attribute__((always_inline)) {
    uint32_t kb = 0x3ffu;
    if (DROP && pb.in >= 0) {
      const long long b0 = pb.in + (long long)r * IW;
      const uint64_t w = (uint64_t)(uint32_t)bits[b0 >> 5] | ((uint64_t)(uint32_t)bits[(b0 >> 5) + 1] << 32);
      kb = (uint32_t)(w >> (b0 & 31)) & 0x3ffu;
    }
#pragma unroll
    for (int xx = 0; xx < IW; ++xx) {
      o[xx] = o[xx] * a1 + b1;
      if (DROP && pb.in >= 0) o[xx] *= ((kb >> xx) & 1u) ? s_in : 0.f;
    }
  };
  const int ng = n_q / gran;
  const int q0 = q_lo + gran * ((ng * z) / n_band), q1 = q_lo + gran * ((ng * (z + 1)) / n_band);
  const int y0 = q0 >> 3;
  const int nst = q1 - q0;  // even

  // staging: thread -> weight rows tid >> 2 and (while < NR) tid >> 2 + 128, k 8 (tid & 3) .. + 7
  const int srow = tid >> 2, sk = 8 * (tid & 3);
  const bool two = srow + 128 < NR;  // wave-uniform (tid < 320)
  const size_t ps = (size_t)NR * HID;
  const __bf16* gp = W3 + (size_t)srow * HID + (size_t)q0 * 32 + sk;
  // the second row's loads are unconditional (a wave without one re-reads its first row and
  // does not store it): loads under a branch were waited for at once and parked in scratch
  const __bf16* gp2 = gp + (two ? (size_t)128 * HID : 0);
  // weight staging of one k step into / out of register set R (macros: as a struct passed
  // to lambdas the two register sets were placed in scratch memory)
#define KP_CVF_GLOAD(R, Q)                                                  \
  do {                                                                      \
    R##0 = *reinterpret_cast<const uint4*>(gp + (Q) * 32);                  \
    R##1 = *reinterpret_cast<const uint4*>(gp + ps + (Q) * 32);             \
    R##2 = *reinterpret_cast<const uint4*>(gp + 2 * ps + (Q) * 32);         \
    R##3 = *reinterpret_cast<const uint4*>(gp2 + (Q) * 32);                 \
    R##4 = *reinterpret_cast<const uint4*>(gp2 + ps + (Q) * 32);            \
    R##5 = *reinterpret_cast<const uint4*>(gp2 + 2 * ps + (Q) * 32);        \
  } while (0)
#define KP_CVF_LSTORE(R, ST)                                                \
  do {                                                                      \
    __bf16* d = bsh + (ST) * (3 * NR * RS) + srow * RS + sk;                \
    *reinterpret_cast<uint4*>(d) = R##0;                                    \
    *reinterpret_cast<uint4*>(d + NR * RS) = R##1;                          \
    *reinterpret_cast<uint4*>(d + 2 * NR * RS) = R##2;                      \
    if (two) {                                                              \
      *reinterpret_cast<uint4*>(d + 128 * RS) = R##3;                       \
      *reinterpret_cast<uint4*>(d + NR * RS + 128 * RS) = R##4;             \
      *reinterpret_cast<uint4*>(d + 2 * NR * RS + 128 * RS) = R##5;         \
    }                                                                       \
  } while (0)
  uint4 ra0, ra1, ra2, ra3, ra4, ra5, rb0, rb1, rb2, rb3, rb4, rb5;

  f32x4 acc[NBF];
#pragma unroll
  for (int n = 0; n < NBF; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // image rows: rows < 20 from the lhs half, the rest from the relation (BN1 applied when a
  // row enters the window); a window of three rows, the next one loaded a map row ahead
  auto img_row = [&](int r, float (&o)[IW]) __attribute__((always_inline)) {
    const float* p = r < 20 ? lhs + r * IW : rel + (r - 20) * IW;
#pragma unroll
    for (int h = 0; h < IW / 2; ++h) {
      const float2 v = *reinterpret_cast<const float2*>(p + 2 * h);
      o[2 * h] = v.x;
      o[2 * h + 1] = v.y;
    }
  };
  float im[3][IW], nx[IW];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    img_row(y0 + ky, im[ky]);
    bn1_row(y0 + ky, im[ky]);
  }
  img_row(min(y0 + 3, FR + 1), nx);

  // one k step: the conv outputs of channel 4 cg + g at map row y straight into the A
  // operand, then 13 x 6 MFMAs against the staged weights of stage ST (a macro: as a
  // lambda called twice the accumulators were not promoted to registers)
#define KP_CVF_KSTEP(Q, ST)                                                                    \
  do {                                                                                         \
    const int y = (q0 + (Q)) >> 3, cg = (q0 + (Q)) & 7;                                        \
    if (cg == 0 && (Q) > 0) {                                                                  \
      bn1_row(y + 2, nx);                                                                      \
      _Pragma("unroll") for (int xx = 0; xx < IW; ++xx) {                                      \
        im[0][xx] = im[1][xx];                                                                 \
        im[1][xx] = im[2][xx];                                                                 \
        im[2][xx] = nx[xx];                                                                    \
      }                                                                                        \
      img_row(min(y + 3, FR + 1), nx);                                                         \
    }                                                                                          \
    const int ch = 4 * cg + g;                                                                 \
    const bool kept = ((fm_keep >> ch) & 1u) != 0;                                             \
    float wv[9];                                                                               \
    _Pragma("unroll") for (int t = 0; t < 9; ++t) wv[t] = sw[ch * 9 + t];                      \
    const float cbias = sc[ch], ca = sa[ch], cbb = sbb[ch];                                    \
    bf16x8 a[3];                                                                               \
    unsigned rb = 0;                                                                           \
    _Pragma("unroll") for (int x = 0; x < FW; ++x) {                                           \
      float v = 0.f;                                                                           \
      _Pragma("unroll") for (int ky = 0; ky < 3; ++ky)                                         \
        _Pragma("unroll") for (int kx = 0; kx < 3; ++kx) v += wv[ky * 3 + kx] * im[ky][x + kx]; \
      v += cbias;                                                                              \
      v = v * ca + cbb;                                                                        \
      rb |= (v > 0.f && kept ? 1u : 0u) << x;                                                  \
      float f = fmaxf(v, 0.f);                                                                 \
      if (fm_on) f *= kept ? s_fm : 0.f;                                                       \
      __bf16 h, m, l;                                                                          \
      kpattn::split3(f, h, m, l);                                                              \
      a[0][x] = h;                                                                             \
      a[1][x] = m;                                                                             \
      a[2][x] = l;                                                                             \
    }                                                                                          \
    if (y < LR && ok) relu[(size_t)i * MASK_B + ch * LR + y] = (uint8_t)rb;                    \
    const __bf16* sb = bsh + (ST) * (3 * NR * RS);                                             \
    _Pragma("unroll") for (int n = 0; n < NBF; ++n) {                                          \
      bf16x8 b[3];                                                                             \
      _Pragma("unroll") for (int p = 0; p < 3; ++p)                                            \
        b[p] = *reinterpret_cast<const bf16x8*>(sb + p * NR * RS + (16 * n + c) * RS + 8 * g); \
      acc[n] = kpattn::mfma3(a, b, acc[n]);                                                    \
    }                                                                                          \
  } while (0)

  // two register stages of weight loads in flight (each load is consumed two k steps after
  // it is issued: one step of cover left the barrier waiting on L2 misses), two LDS
  // stages, one barrier per k step; nst is even
  KP_CVF_GLOAD(ra, 0);
  KP_CVF_GLOAD(rb, 1);
  KP_CVF_LSTORE(ra, 0);
  __syncthreads();
  for (int q = 0; q < nst; q += 2) {
    if (q + 2 < nst) KP_CVF_GLOAD(ra, q + 2);
    KP_CVF_KSTEP(q, 0);
    KP_CVF_LSTORE(rb, 1);
    __syncthreads();
    if (q + 3 < nst) KP_CVF_GLOAD(rb, q + 3);
    KP_CVF_KSTEP(q + 1, 1);
    if (q + 2 < nst) KP_CVF_LSTORE(ra, 0);
    __syncthreads();
  }
#undef KP_CVF_KSTEP
#undef KP_CVF_GLOAD
#undef KP_CVF_LSTORE
  // C block n: lane (g, c) holds pairs 16 w + 4 g + r, output 16 n + c
#pragma unroll
  for (int n = 0; n < NBF; ++n) {
    const int col = 16 * n + c;
    if (col >= dim) continue;
    const float bias = (z == 0 && fcb) ? fcb[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * w + 4 * g + r;
      if (row < M) out[((size_t)z * M + row) * dim + col] = acc[n][r] + bias;
    }
  }
}

// backward: dl[z][i][j] = a1 * sum over channels 2 z, 2 z + 1 of the transposed 3x3
// convolution of dmap_c = [relu > 0] a2_c (dfc_i . W_c^T), j = 10 y + x over the lhs half
__global__ __launch_bounds__(512) void kp_cv_bwd_fused(int M, const __bf16* __restrict__ G3,
                                                       const __bf16* __restrict__ WT3,
                                                       const uint8_t* __restrict__ relu,
                                                       const float* __restrict__ cw, const float* __restrict__ bna,
                                                       float s_fm, int dp, float* __restrict__ dl) {
  extern __shared__ __attribute__((aligned(16))) __bf16 bsh[];  // [stage][piece][160][RS]; then dmap [MT][DCS] fp32
  __shared__ uint8_t rls[CGRP][MT * LR];                        // the tile's ReLU sign bytes
  constexpr int BR = LR * FW;                                   // 160 weight rows per channel
  constexpr int NQ = KB / 32;                                   // 7 k steps
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  int z, mt;
  xcd_map(blockIdx.x, z, mt);
  const int m0 = mt * MT;
  if (m0 >= M) return;
  const int i = m0 + 16 * w + c;
  const int ic = i < M ? i : M - 1;
  const size_t gps = (size_t)M * KB;
  const __bf16* ga = G3 + (size_t)ic * KB + 8 * g;
  // ReLU sign bytes of both channels: loaded now, parked in LDS before the first epilogue
  constexpr int RPT = CGRP * MT * LR / 512;  // 10 per thread
  uint32_t rb[RPT];
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const int j = tid + 512 * u, cc = j / (MT * LR), rem = j % (MT * LR);
    const int row = min(m0 + rem / LR, M - 1);
    rb[u] = relu[(size_t)row * MASK_B + (z * CGRP + cc) * LR + rem % LR];
  }
  const int srow = tid >> 2, sk = 8 * (tid & 3);
  const bool two = srow + 128 < BR;  // wave-uniform (tid < 128)
  const size_t wps = (size_t)NBL * KB;
  uint4 ga0, ga1, ga2, gb0, gb1, gb2;  // unconditional loads, as in the forward
  // transposed convolution: thread -> pair tid >> 2, lhs image rows (tid & 3) + 4 u; its
  // partial sums live in registers for one channel and go through the thread's own part
  // of the output slab between channels (keeps the GEMM's and these registers disjoint)
  const int tp = tid >> 2, ty = tid & 3;
  const int prow = m0 + tp;
  const float a1 = bna[0];
  float* dlo = dl + ((size_t)z * M + (prow < M ? prow : 0)) * dp;
  float* dms = reinterpret_cast<float*>(bsh);

  for (int cc = 0; cc < CGRP; ++cc) {
    const int ch = z * CGRP + cc;
    const __bf16* gp = WT3 + (size_t)(ch * BR + srow) * KB + sk;
    const __bf16* gp2 = gp + (two ? (size_t)128 * KB : 0);
    auto gload = [&](int q) {
      ga0 = *reinterpret_cast<const uint4*>(gp + q * 32);
      ga1 = *reinterpret_cast<const uint4*>(gp + wps + q * 32);
      ga2 = *reinterpret_cast<const uint4*>(gp + 2 * wps + q * 32);
      gb0 = *reinterpret_cast<const uint4*>(gp2 + q * 32);
      gb1 = *reinterpret_cast<const uint4*>(gp2 + wps + q * 32);
      gb2 = *reinterpret_cast<const uint4*>(gp2 + 2 * wps + q * 32);
    };
    auto lstore = [&](int st) {
      __bf16* d = bsh + st * (3 * BR * RS) + srow * RS + sk;
      *reinterpret_cast<uint4*>(d) = ga0;
      *reinterpret_cast<uint4*>(d + BR * RS) = ga1;
      *reinterpret_cast<uint4*>(d + 2 * BR * RS) = ga2;
      if (two) {
        *reinterpret_cast<uint4*>(d + 128 * RS) = gb0;
        *reinterpret_cast<uint4*>(d + BR * RS + 128 * RS) = gb1;
        *reinterpret_cast<uint4*>(d + 2 * BR * RS + 128 * RS) = gb2;
      }
    };
    f32x4 acc[NBB];
#pragma unroll
    for (int n = 0; n < NBB; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // A operand (the lane's dfc row) one k step ahead, like the weights
    bf16x8 an[3];
    auto aload = [&](int q) {
#pragma unroll
      for (int p = 0; p < 3; ++p) an[p] = *reinterpret_cast<const bf16x8*>(ga + p * gps + q * 32);
    };
    aload(0);
    gload(0);
    lstore(0);
    __syncthreads();
    int st = 0;
#pragma unroll 1
    for (int q = 0; q < NQ; ++q) {
      bf16x8 a[3] = {an[0], an[1], an[2]};
      if (q + 1 < NQ) {
        gload(q + 1);
        aload(q + 1);
      }
      const __bf16* sb = bsh + st * (3 * BR * RS);
#pragma unroll
      for (int n = 0; n < NBB; ++n) {
        bf16x8 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b[p] = *reinterpret_cast<const bf16x8*>(sb + p * BR * RS + (16 * n + c) * RS + 8 * g);
        acc[n] = kpattn::mfma3(a, b, acc[n]);
      }
      if (q + 1 < NQ) lstore(st ^ 1);
      __syncthreads();
      st ^= 1;
    }
    if (cc == 0) {
#pragma unroll
      for (int u = 0; u < RPT; ++u) (&rls[0][0])[tid + 512 * u] = (uint8_t)rb[u];
      __syncthreads();
    }
    // dmap = [ReLU > 0] a2 acc, parked over the (now idle) weight stages (rows past M
    // hold the clamped pair's values and are never stored)
    const float a2 = bna[1 + ch];
#pragma unroll
    for (int n = 0; n < NBB; ++n) {
      const int col = 16 * n + c;  // 8 y + x
      const int y = col >> 3, x = col & 7;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = 16 * w + 4 * g + r;
        // (feature-map dropout: the stored bits are 0 for a dropped channel; a kept one
        // carries 1/(1-p), s_fm = 1 without that dropout)
        dms[pl * DCS + col] = ((rls[cc][pl * LR + y] >> x) & 1u) ? (acc[n][r] * s_fm) * a2 : 0.f;
      }
    }
    __syncthreads();
    float wv[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wv[t] = cw[ch * 9 + t];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int yy = ty + 4 * u;
      float dacc[IW];
#pragma unroll
      for (int xx = 0; xx < IW; ++xx) dacc[xx] = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int y = yy - ky;
        if (y < 0) continue;  // y <= yy < 20 always
        float dm[FW];
        const float4 v0 = *reinterpret_cast<const float4*>(dms + tp * DCS + y * FW);
        const float4 v1 = *reinterpret_cast<const float4*>(dms + tp * DCS + y * FW + 4);
        dm[0] = v0.x; dm[1] = v0.y; dm[2] = v0.z; dm[3] = v0.w;
        dm[4] = v1.x; dm[5] = v1.y; dm[6] = v1.z; dm[7] = v1.w;
#pragma unroll
        for (int xx = 0; xx < IW; ++xx)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int x = xx - kx;
            if (x >= 0 && x < FW) dacc[xx] += dm[x] * wv[ky * 3 + kx];
          }
      }
      if (prow < M)
#pragma unroll
        for (int xx = 0; xx < IW; ++xx) {
          const float v = dacc[xx] * a1;
          dlo[yy * IW + xx] = cc == 0 ? v : dlo[yy * IW + xx] + v;
        }
    }
    __syncthreads();  // the next channel's weight stages overwrite dmap
  }
}

// dl[0][i][j] = sum over the channel-group slabs (in slab order), in place in slab 0,
// times the pair's input-dropout multiplier of lhs image element j (mb: with that dropout)
__global__ void kp_cv_dl_reduce(int M, int dp, const CvBits* __restrict__ mb, const int32_t* __restrict__ bits,
                                float s_in, float* __restrict__ dl) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int jn = LR * IW;
  if (t >= (long long)M * jn) return;
  const int i = (int)(t / jn), j = (int)(t % jn);
  const size_t o = (size_t)i * dp + j, zs = (size_t)M * dp;
  float v = dl[o];
#pragma unroll
  for (int zz = 1; zz < NSPLIT; ++zz) v += dl[zz * zs + o];
  if (mb) {
    const long long b = mb[i].in + j;
    v *= (((uint32_t)bits[b >> 5] >> (b & 31)) & 1u) ? s_in : 0.f;
  }
  dl[o] = v;
}

// ---------------------------------------------------------------------------------
// Shared-encoder path (no input or feature-map dropout; kp_conve.hip, KP_CV_SHARED).
// Map rows 0-17 read only the kelpie half of the image (rows 0-19), rows 20-37 only the
// relation half, rows 18-19 both.  So per step the FC input splits as
//   fc_i = W_lhs map_lhs(x_slot) + W_mid map_mid(x_slot, r_i) + W_rel map_rel(r_i) + b:
// the first term once per kelpie row (slot) instead of once per pair, the last once per
// relation and context (relations and layers are frozen), and only the 512 columns of
// rows 18-19 per pair.  The backward splits the same way: the ReLU signs of rows 0-17
// are the kelpie row's, so the pairs' gradients of those rows are one product with the
// sum of the pairs' dfc; rows 18-19 go per pair.  On the bench's ConvE step (3,456 pairs of
// 160 kelpie rows) that is under 10 % of the fused path's multiply-adds.
constexpr int MID_Y = 18;          // first map row that reads the relation half
constexpr int NMID = CH * 2 * FW;  // its 512 columns (rows 18-19 of every channel)
constexpr int MPW = 16;            // pairs per workgroup of kp_cv_mid_bwd

// W [dim][HID] -> the transposed mid columns [dim][512], col = 16 ch + 8 (y - 18) + x
__global__ void kp_cv_mid_wt(const float* __restrict__ W, int dim, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dim * NMID) return;
  const int d = i / NMID, col = i % NMID;
  const int ch = col >> 4, y = MID_Y + ((col >> 3) & 1), x = col & 7;
  out[i] = W[(size_t)d * HID + ch * (FR * FW) + y * FW + x];
}

// The maps and transposed convolutions are small fp32 kernels; the four products (the
// kelpie rows' map rows 0-17 and the pairs' rows 18-19 through the FC, and the two
// transposed products of the backward) go to the fp32 MFMA GEMM (kp_gemm_abt, 64 x 64
// tiles).  A step has ~160 kelpie rows, too few for the 128-row bf16x3 tiles above (their
// per-workgroup latency, not the arithmetic, set the time), and the plain fp32 loops over
// an LDS operand that were tried first ran 3 TFLOP/s.
constexpr int LHS_Y = 18;              // map rows 0-17 read the kelpie half only
constexpr int NLHS = CH * LHS_Y * FW;  // their 4608 columns, l = 144 c + 8 y + x
constexpr int KSL = 16;                // split-K slabs of the kelpie rows' FC product

__host__ __device__ constexpr int lhs_col(int l) { return (l / 144) * (FR * FW) + l % 144; }

// W [dim][HID] -> the kelpie rows' columns [dim][4608] and transposed [4608][dim], and the
// mid columns transposed [512][dim] (col = 16 ch + 8 (y - 18) + x)
__global__ void kp_cv_lhs_wt(const float* __restrict__ W, int dim, float* __restrict__ wlc, float* __restrict__ wl,
                             float* __restrict__ wm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NLHS * dim) {
    const int l = i / dim, o = i % dim;
    wl[i] = W[(size_t)o * HID + lhs_col(l)];
    const int o2 = i / NLHS, l2 = i % NLHS;
    wlc[i] = W[(size_t)o2 * HID + lhs_col(l2)];
  } else if (i < (NLHS + NMID) * dim) {
    const int e = i - NLHS * dim, col = e / dim, o = e % dim;
    const int ch = col >> 4, y = MID_Y + ((col >> 3) & 1), x = col & 7;
    wm[e] = W[(size_t)o * HID + ch * (FR * FW) + y * FW + x];
  }
}

// per pair i: map rows 18-19 (image rows 18-21: the kelpie half's rows 18-19 and the
// relation half's rows 0-1; BN1, conv, bias, BN2, ReLU) -> mm[i][512] and their ReLU
// sign bytes relu[i][20 ch + y]; one thread per (pair, channel, row)
__global__ void kp_cv_mid_map(int M, const int2* __restrict__ src, const float* __restrict__ E,
                              const float* __restrict__ X, const float* __restrict__ R, int dp,
                              const float* __restrict__ cw, const float* __restrict__ cb,
                              const float* __restrict__ bna, const float* __restrict__ bnb, float* __restrict__ mm,
                              uint8_t* __restrict__ relu) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= M * CH * 2) return;
  const int i = e / (CH * 2), c = (e / 2) % CH, yy = e % 2;
  const int2 s = src[i];
  const float* lhs = s.x >= 0 ? E + (size_t)s.x * dp : X + (size_t)(-s.x - 1) * dp;
  const float* rel = R + (size_t)s.y * dp;
  const float a1 = bna[0], b1 = bnb[0];
  float im[3][IW];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yr = MID_Y + yy + ky;
    const float* row = yr < LR ? lhs + yr * IW : rel + (yr - LR) * IW;
#pragma unroll
    for (int xx = 0; xx < IW; ++xx) im[ky][xx] = row[xx] * a1 + b1;
  }
  float w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = cw[c * 9 + t];
  const float bias = cb[c], a2 = bna[1 + c], b2 = bnb[1 + c];
  unsigned rb = 0;
#pragma unroll
  for (int xx = 0; xx < FW; ++xx) {
    float v = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) v += w[ky * 3 + kx] * im[ky][xx + kx];
    v += bias;
    v = v * a2 + b2;
    rb |= (v > 0.f ? 1u : 0u) << xx;
    mm[(size_t)i * NMID + c * 16 + yy * 8 + xx] = fmaxf(v, 0.f);
  }
  relu[(size_t)i * MASK_B + c * LR + MID_Y + yy] = (uint8_t)rb;
}

// per pair i (MPW per workgroup): dmap = [ReLU > 0] a2_c dmr[i] (dmr = dfc_i W_mid, from the
// GEMM) through the transposed 3x3 convolution into lhs image rows 18-19 (times a1); the
// pair's dl row [dp] gets that, plus, for the first pair of its kelpie row (psr[i] =
// (kelpie row, first)), the row's shared part dls (map rows 0-17), zero elsewhere
__global__ __launch_bounds__(256) void kp_cv_mid_convt(int M, const float* __restrict__ dmr,
                                                       const uint8_t* __restrict__ relu, const float* __restrict__ cw,
                                                       const float* __restrict__ bna, const int2* __restrict__ psr,
                                                       const float* __restrict__ dls, int dp, float* __restrict__ dl) {
  __shared__ float dm[MPW][NMID + 4];
  __shared__ float img[MPW][2 * IW];
  __shared__ uint8_t rbs[MPW][CH * 2];  // the pairs' ReLU bytes of rows 18-19
  __shared__ float a2s[CH];
  const int tid = threadIdx.x;
  const int i0 = blockIdx.x * MPW;
  if (i0 >= M) return;
  for (int e = tid; e < MPW * CH * 2; e += 256) {
    const int p = e / (CH * 2), c = (e >> 1) % CH, yy = e & 1, i = i0 + p;
    rbs[p][e % (CH * 2)] = i < M ? relu[(size_t)i * MASK_B + c * LR + MID_Y + yy] : 0;
  }
  if (tid < CH) a2s[tid] = bna[1 + tid];
  __syncthreads();
  for (int e = tid; e < MPW * NMID; e += 256) {
    const int p = e / NMID, col = e % NMID, i = i0 + p;
    const int ch = col >> 4, yy = (col >> 3) & 1, x = col & 7;
    const bool on = (rbs[p][2 * ch + yy] >> x) & 1u;
    dm[p][col] = on ? dmr[(size_t)min(i, M - 1) * NMID + col] * a2s[ch] : 0.f;
  }
  __syncthreads();
  const float a1 = bna[0];
  for (int e = tid; e < MPW * 2 * IW; e += 256) {
    const int p = e / (2 * IW), r = e % (2 * IW), yi = MID_Y + r / IW, xx = r % IW;
    float acc = 0.f;
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int y = yi - ky;
        if (y < MID_Y || y > MID_Y + 1) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int x = xx - kx;
          if (x >= 0 && x < FW) acc += dm[p][ch * 16 + (y - MID_Y) * 8 + x] * cw[ch * 9 + ky * 3 + kx];
        }
      }
    img[p][r] = acc * a1;
  }
  __syncthreads();
  for (int e = tid; e < MPW * dp; e += 256) {
    const int p = e / dp, j = e % dp, i = i0 + p;
    if (i >= M) continue;
    float v = 0.f;
    if (j >= MID_Y * IW && j < LR * IW) v = img[p][j - MID_Y * IW];
    const int2 s = psr[i];
    if (s.y && j < LR * IW) v += dls[(size_t)s.x * dp + j];
    dl[(size_t)i * dp + j] = v;
  }
}

// kelpie row k (src[k].x = -slot - 1): map rows 0-17 (BN1, conv, bias, BN2, ReLU; the
// forward's tap order) -> map[k][l]; their ReLU sign bytes -> relu[k][20 ch + y]
__global__ __launch_bounds__(256) void kp_cv_lhs_map(int n, const int2* __restrict__ src, const float* __restrict__ X,
                                                     int dp, const float* __restrict__ cw, const float* __restrict__ cb,
                                                     const float* __restrict__ bna, const float* __restrict__ bnb,
                                                     float* __restrict__ map, uint8_t* __restrict__ relu) {
  __shared__ float img[LR][IW];
  const int k = blockIdx.x;
  if (k >= n) return;
  const float* x = X + (size_t)(-src[k].x - 1) * dp;
  const float a1 = bna[0], b1 = bnb[0];
  for (int e = threadIdx.x; e < LR * IW; e += blockDim.x) img[e / IW][e % IW] = x[e] * a1 + b1;
  __syncthreads();
  for (int e = threadIdx.x; e < CH * LHS_Y; e += blockDim.x) {
    const int c = e / LHS_Y, y = e % LHS_Y;
    float w[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) w[t] = cw[c * 9 + t];
    const float bias = cb[c], a2 = bna[1 + c], b2 = bnb[1 + c];
    unsigned rb = 0;
#pragma unroll
    for (int xx = 0; xx < FW; ++xx) {
      float v = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) v += w[ky * 3 + kx] * img[y + ky][xx + kx];
      v += bias;
      v = v * a2 + b2;
      rb |= (v > 0.f ? 1u : 0u) << xx;
      map[(size_t)k * NLHS + c * 144 + y * FW + xx] = fmaxf(v, 0.f);
    }
    relu[(size_t)k * MASK_B + c * LR + y] = (uint8_t)rb;
  }
}

// per kelpie row k: g[k] = the sum of its pairs' dfc (pairs [rng.x, rng.y) in order)
__global__ void kp_cv_slot_g(int n, const int2* __restrict__ rng, const float* __restrict__ dfc, int dim,
                             float* __restrict__ g) {
  const int k = blockIdx.x;
  if (k >= n) return;
  const int2 r = rng[k];
  for (int d = threadIdx.x; d < dim; d += blockDim.x) {
    float v = 0.f;
    for (int i = r.x; i < r.y; ++i) v += dfc[(size_t)i * dim + d];
    g[(size_t)k * dim + d] = v;
  }
}

// dls[k][j] (j = 10 y + x, lhs image rows 0-19) = a1 times the transposed 3x3 convolution
// over map rows 0-17 (channels in order) of dmap = [ReLU > 0] a2_c dmr[k] (dmr = g_k W_lhs,
// from the GEMM)
__global__ __launch_bounds__(256) void kp_cv_lhs_convt(int n, const float* __restrict__ dmr,
                                                       const uint8_t* __restrict__ relu, const float* __restrict__ cw,
                                                       const float* __restrict__ bna, int dp, float* __restrict__ dls) {
  __shared__ float dm[NLHS];
  __shared__ uint8_t rbs[CH * LR];
  __shared__ float a2s[CH];
  const int k = blockIdx.x;
  if (k >= n) return;
  for (int e = threadIdx.x; e < CH * LR; e += blockDim.x) rbs[e] = relu[(size_t)k * MASK_B + e];
  if (threadIdx.x < CH) a2s[threadIdx.x] = bna[1 + threadIdx.x];
  __syncthreads();
  for (int e = threadIdx.x; e < NLHS; e += blockDim.x) {
    const int c = e / 144, rem = e % 144, y = rem >> 3, x = rem & 7;
    const bool on = (rbs[c * LR + y] >> x) & 1u;
    dm[e] = on ? dmr[(size_t)k * NLHS + e] * a2s[c] : 0.f;
  }
  __syncthreads();
  const int j = threadIdx.x;
  if (j >= LR * IW) return;
  const int yi = j / IW, xi = j % IW;
  float acc = 0.f;
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int y = yi - ky;
      if (y < 0 || y >= LHS_Y) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int x = xi - kx;
        if (x >= 0 && x < FW) acc += dm[c * 144 + y * FW + x] * cw[c * 9 + ky * 3 + kx];
      }
    }
  dls[(size_t)k * dp + j] = acc * bna[0];
}

// out[i] = sum over nz slabs [nz][n][dim] (slab order)
__global__ void kp_cv_slab_sum(int n, int nz, int dim, const float* __restrict__ slab, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * dim) return;
  float v = 0.f;
  for (int z = 0; z < nz; ++z) v += slab[(size_t)z * n * dim + i];
  out[i] = v;
}

}  // namespace kpcvf
