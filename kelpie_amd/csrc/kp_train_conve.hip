// kp_train_conve.hip -- full-model ConvE training on the device, for the retraining step
// of explanation verification (src/verify_explanations.py:141-143, :230-232: a fresh
// ConvE with init_random=True trained by BCEOptimizer on the edited training set).
//
// Reference (src/link_prediction/models/conve.py:133-158 all_scores in train mode,
// src/link_prediction/optimization/bce_optimizer.py:45-150): per batch of B (h, r) pairs
//   image  = [E_h ; R_r] as 40 x h                 (two 20 x h halves)
//   x1     = BN1(image) * in_noise                 (BatchNorm2d(1), Dropout)
//   c      = conv3x3(x1) + b                       (32 channels, 38 x (h - 2))
//   f      = ReLU(BN2(c)) * fm_noise[b][channel]   (BatchNorm2d(32), Dropout2d)
//   z      = ReLU(BN3((f W^T + b_fc) * hid_noise)) (Linear, Dropout, BatchNorm1d(d))
//   p      = sigmoid(z E^T)                        (every entity)
//   loss   = BCELoss(p, (1 - ls) onehot(tails) + 1 / N)   (mean over B x N)
// then the backward through every layer and Adam (torch defaults) on every parameter:
// the entity / relation tables (dense entity gradient: every entity is scored), conv,
// FC, and the three batch norms' affine parameters; batch statistics in train mode, the
// running statistics updated with momentum 0.1 (unbiased variance).  A batch of one
// pair runs the batch norms in eval mode (bce_optimizer.py:136-149).  The dropout
// noise (0 or 1 / (1 - p) per element / channel) is drawn by the host from the torch
// generator in the forward's order and passed in (RNG as input).
// Not the hot path: verification retrains once per explained set; plain fp32 kernels,
// the GEMMs on kp_gemm_abt, per-key row sums in batch order (deterministic).
#include <algorithm>
#include <cmath>
#include <vector>

#include "kp_common.hpp"

namespace {

constexpr float kBnEps = 1e-5f;
constexpr float kMomentum = 0.1f;

// image[b][j], j < 40 h: rows 0..19 the head entity's row, 20..39 the relation's
__global__ void cvt_image(int B, const int32_t* __restrict__ pairs, const float* __restrict__ E,
                          const float* __restrict__ R, int dp, int half, float* __restrict__ img) {
  const int b = blockIdx.x;
  if (b >= B) return;
  const float* e = E + (size_t)pairs[2 * b] * dp;
  const float* r = R + (size_t)pairs[2 * b + 1] * dp;
  for (int j = threadIdx.x; j < 2 * half; j += blockDim.x) img[(size_t)b * 2 * half + j] = j < half ? e[j] : r[j - half];
}

// per channel c of x (element (b, c, s) at b sb + c sc + s, s < S): batch mean and biased
// variance (two passes in double), one workgroup per channel
__global__ __launch_bounds__(256) void cvt_bn_stats(const float* __restrict__ x, int B, int S, long long sb,
                                                    long long sc, float* __restrict__ mean, float* __restrict__ var) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  const long long n = (long long)B * S;
  auto at = [&](long long i) { return x[(i / S) * sb + (long long)c * sc + (i % S)]; };
  double a = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) a += at(i);
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  const double m = (red[0] + red[1] + red[2] + red[3]) / (double)n;
  __syncthreads();
  double v = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const double d = (double)at(i) - m;
    v += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    mean[c] = (float)m;
    var[c] = (float)((red[0] + red[1] + red[2] + red[3]) / (double)n);
  }
}

// running statistics (train mode): rm = (1 - m) rm + m mean, rv = (1 - m) rv + m var n / (n - 1)
__global__ void cvt_bn_running(int C, long long n, const float* __restrict__ mean, const float* __restrict__ var,
                               float* __restrict__ rm, float* __restrict__ rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float unb = n > 1 ? var[c] * (float)((double)n / (double)(n - 1)) : var[c];
  rm[c] = (1.0f - kMomentum) * rm[c] + kMomentum * mean[c];
  rv[c] = (1.0f - kMomentum) * rv[c] + kMomentum * unb;
}

// y = (x - mean) rstd w + b per element; xhat saved; mode 0: y * noise[element] (or 1);
// mode 1: ReLU then * noise[b][c]; mode 2: ReLU (no noise).  pre = the BN output before
// ReLU (for the ReLU mask).  (b, c, s) layout as cvt_bn_stats, output in x's layout.
__global__ void cvt_bn_fwd(const float* __restrict__ x, int B, int C, int S, long long sb, long long sc,
                           const float* __restrict__ mean, const float* __restrict__ var, const float* __restrict__ w,
                           const float* __restrict__ bb, int mode, const float* __restrict__ noise,
                           float* __restrict__ xhat, float* __restrict__ pre, float* __restrict__ y) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)B * C * S;
  if (t >= n) return;
  const int b = (int)(t / ((long long)C * S));
  const int c = (int)((t / S) % C);
  const int s = (int)(t % S);
  const long long o = b * sb + (long long)c * sc + s;
  const float rstd = 1.0f / sqrtf(var[c] + kBnEps);
  const float xh = (x[o] - mean[c]) * rstd;
  const float v = xh * w[c] + bb[c];
  xhat[o] = xh;
  if (pre) pre[o] = v;
  float out;
  if (mode == 0)
    out = noise ? v * noise[o] : v;
  else if (mode == 1)
    out = noise ? fmaxf(v, 0.f) * noise[(size_t)b * C + c] : fmaxf(v, 0.f);
  else
    out = fmaxf(v, 0.f);
  y[o] = out;
}

// BN backward per channel (one workgroup per channel): dy (layout of x), returns
// dx = rstd / n (n w dy - sum(w dy) - xhat sum(w dy xhat)) in train mode, or
// dx = w rstd dy in eval mode; dw[c] = sum dy xhat, db[c] = sum dy
__global__ __launch_bounds__(256) void cvt_bn_bwd(const float* __restrict__ dy, const float* __restrict__ xhat, int B,
                                                  int S, long long sb, long long sc, const float* __restrict__ var,
                                                  const float* __restrict__ w, int train, float* __restrict__ dx,
                                                  float* __restrict__ dw, float* __restrict__ db) {
  __shared__ double red[2][4];
  const int c = blockIdx.x;
  const long long n = (long long)B * S;
  auto off = [&](long long i) { return (i / S) * sb + (long long)c * sc + (i % S); };
  double s1 = 0.0, s2 = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const long long o = off(i);
    s1 += dy[o];
    s2 += (double)dy[o] * xhat[o];
  }
  for (int k = 32; k > 0; k >>= 1) {
    s1 += __shfl_xor(s1, k, 64);
    s2 += __shfl_xor(s2, k, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  const double sdy = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const double sdyx = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  if (threadIdx.x == 0) {
    db[c] = (float)sdy;
    dw[c] = (float)sdyx;
  }
  const float rstd = 1.0f / sqrtf(var[c] + kBnEps);
  const float wc = w[c];
  for (long long i = threadIdx.x; i < n; i += 256) {
    const long long o = off(i);
    if (train)
      dx[o] = (float)((double)(wc * rstd) / (double)n * ((double)n * dy[o] - sdy - (double)xhat[o] * sdyx));
    else
      dx[o] = wc * rstd * dy[o];
  }
}

// conv 3x3 (32 channels, no padding) + bias: x1 [B][40][H] -> c [B][32][38][W2]
__global__ void cvt_conv_fwd(int B, int H, const float* __restrict__ x1, const float* __restrict__ cw,
                             const float* __restrict__ cb, float* __restrict__ out) {
  const int W2 = H - 2, per_c = 38 * W2;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)B * 32 * per_c) return;
  const int b = (int)(t / (32 * per_c)), rem = (int)(t % (32 * per_c));
  const int ch = rem / per_c, yx = rem % per_c, y = yx / W2, xx = yx % W2;
  const float* img = x1 + (size_t)b * 40 * H;
  float acc = 0.f;
  for (int ky = 0; ky < 3; ++ky)
    for (int kx = 0; kx < 3; ++kx) acc += cw[ch * 9 + ky * 3 + kx] * img[(y + ky) * H + xx + kx];
  out[t] = acc + cb[ch];
}

// conv backward: dx1 [B][40][H] (transposed conv of dc), one thread per image element
__global__ void cvt_conv_bwd_x(int B, int H, const float* __restrict__ dc, const float* __restrict__ cw,
                               float* __restrict__ dx1) {
  const int W2 = H - 2, per_c = 38 * W2;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)B * 40 * H) return;
  const int b = (int)(t / (40 * H)), rem = (int)(t % (40 * H));
  const int yy = rem / H, xx = rem % H;
  const float* d = dc + (size_t)b * 32 * per_c;
  float acc = 0.f;
  for (int ch = 0; ch < 32; ++ch)
    for (int ky = 0; ky < 3; ++ky) {
      const int y = yy - ky;
      if (y < 0 || y >= 38) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int x = xx - kx;
        if (x < 0 || x >= W2) continue;
        acc += d[ch * per_c + y * W2 + x] * cw[ch * 9 + ky * 3 + kx];
      }
    }
  dx1[t] = acc;
}

// conv weight / bias gradients: one workgroup per (channel, tap) (tap 9 = the bias)
__global__ __launch_bounds__(256) void cvt_conv_bwd_w(int B, int H, const float* __restrict__ dc,
                                                      const float* __restrict__ x1, float* __restrict__ dcw,
                                                      float* __restrict__ dcb) {
  __shared__ double red[4];
  const int ch = blockIdx.x / 10, tap = blockIdx.x % 10;
  const int W2 = H - 2, per_c = 38 * W2;
  const long long n = (long long)B * per_c;
  double a = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const int b = (int)(i / per_c), yx = (int)(i % per_c), y = yx / W2, x = yx % W2;
    const float g = dc[((size_t)b * 32 + ch) * per_c + yx];
    a += tap == 9 ? (double)g : (double)g * x1[(size_t)b * 40 * H + (y + tap / 3) * H + x + tap % 3];
  }
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)(red[0] + red[1] + red[2] + red[3]);
    if (tap == 9)
      dcb[ch] = v;
    else
      dcw[ch * 9 + tap] = v;
  }
}

// G[b][e] = d BCELoss / d logit from p = sigmoid(logit) (torch's BCELoss backward, then
// sigmoid's): targets (1 - ls) onehot(tails of pair b) + 1 / N; rows >= B zeroed
__global__ void cvt_bce_grad(float* __restrict__ P, int ld, int B, int N, const int32_t* __restrict__ toff,
                             const int32_t* __restrict__ tails, float ylo, float yhi, float gs) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ld) return;
  float* row = P + (size_t)b * ld;
  if (b >= B || e >= N) {
    row[e] = 0.f;
    return;
  }
  bool hit = false;
  for (int k = toff[b]; k < toff[b + 1]; ++k) hit |= tails[k] == e;
  const float p = row[e], y = hit ? yhi : ylo;
  const float w = (1.0f - p) * p;
  row[e] = ((p - y) / fmaxf(w, 1e-12f) * gs) * w;
}

// out[c][r] = in[r][c] for r < rows, c < cols; the rest of out's rows [0, cols) x [rows, ld_out) zero
__global__ void cvt_transpose(const float* __restrict__ in, int rows, int cols, int ld_in, float* __restrict__ out,
                              int ld_out) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? in[(size_t)r * ld_in + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < ld_out) out[(size_t)c * ld_out + r] = tile[tx][i];
  }
}

// elementwise y = x * m (m null: copy)
__global__ void cvt_mul(long long n, const float* __restrict__ x, const float* __restrict__ m, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = m ? x[i] * m[i] : x[i];
}

// dz = dz * [pre > 0] (ReLU backward)
__global__ void cvt_relu_bwd(long long n, const float* __restrict__ pre, float* __restrict__ d) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !(pre[i] > 0.f)) d[i] = 0.f;
}

// feature-map dropout then ReLU backward: d[b][c][s] *= noise[b][c] [pre > 0]
__global__ void cvt_fm_bwd(int B, int C, int S, const float* __restrict__ pre, const float* __restrict__ noise,
                           float* __restrict__ d) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * C * S) return;
  const long long bc = i / S;
  float v = d[i];
  if (noise) v *= noise[bc];
  d[i] = pre[i] > 0.f ? v : 0.f;
}

// column sums over the batch rows: out[k] = sum_b x[b][k] (k < K), one thread per column
__global__ void cvt_colsum(const float* __restrict__ x, int B, int K, int ld, float* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double a = 0.0;
  for (int b = 0; b < B; ++b) a += x[(size_t)b * ld + k];
  out[k] = (float)a;
}

// table gradient rows += the image-gradient halves of the pairs keyed to them, in batch
// order (keys / off / items: host CSR; item = pair index); part 0 = lhs rows, 1 = rel rows
__global__ void cvt_scatter(float* __restrict__ G, int dp, int half, const int32_t* __restrict__ keys,
                            const int32_t* __restrict__ off, const int32_t* __restrict__ items,
                            const float* __restrict__ dimg, int part) {
  const int k = blockIdx.x;
  float* g = G + (size_t)keys[k] * dp;
  for (int d = threadIdx.x; d < half; d += blockDim.x) {
    float acc = 0.f;
    for (int i = off[k]; i < off[k + 1]; ++i) acc += dimg[(size_t)items[i] * 2 * half + part * half + d];
    g[d] += acc;
  }
}

struct AdamArgs {
  float b1m, b2, b2m, eps, step_size, bc2_sqrt;
};

// torch.optim.Adam (defaults: betas (0.9, 0.999), eps 1e-8, no weight decay), torch op order
__global__ void cvt_adam(float* __restrict__ X, float* __restrict__ M, float* __restrict__ V,
                         const float* __restrict__ G, long long n, AdamArgs a) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = G[i];
  float m = M[i], v = V[i];
  m = m + a.b1m * (g - m);
  v = v * a.b2;
  v = v + (a.b2m * g) * g;
  X[i] = X[i] + (-a.step_size * m) / (sqrtf(v) / a.bc2_sqrt + a.eps);
  M[i] = m;
  V[i] = v;
}

inline unsigned nblk(long long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

}  // namespace

// Parameters beyond the context's (batch-norm affine and running statistics), the
// optimizer state of every parameter, and the scratch of a run.
struct kp_cv_train {
  int C3 = 0;  // 1 + 32 + dim: the three batch norms' channels, concatenated
  DevBuf bnw, bnb, rm, rv;
  DevBuf mE, vE, mR, vR, mcw, vcw, mcb, vcb, mfw, vfw, mfb, vfb, mbw, vbw, mbb, vbb;
  DevBuf gE, gR, gcw, gcb, gfw, gfb, gbw, gbb;
  DevBuf pairs, toff, tails, nin, nfm, nhid, keys, off, items;
  DevBuf img, xh1, x1, cv, xh2, pre2, f, h, hd, xh3, pre3, z, P, ET, PT, zT, dz, dh, dhT, fT, WT, df, dc, dx1, dimg;
  DevBuf mean, var;
  int64_t step = 0;
};

void cv_train_free(kp_ctx* c) {
  delete c->cvtrain;
  c->cvtrain = nullptr;
}

void conve_train_begin(kp_ctx* c, const float* bn_w, const float* bn_b, const float* bn_m, const float* bn_v) {
  KP_REQUIRE(c->model == KP_MODEL_CONVE, "kp_conve_train_begin: ConvE contexts only");
  delete c->cvtrain;
  c->cvtrain = new kp_cv_train();
  kp_cv_train& t = *c->cvtrain;
  t.C3 = 1 + 32 + c->dim;
  upload(c, t.bnw, bn_w, t.C3);
  upload(c, t.bnb, bn_b, t.C3);
  upload(c, t.rm, bn_m, t.C3);
  upload(c, t.rv, bn_v, t.C3);
  const size_t sizes[8] = {(size_t)c->n_ent * c->dp, (size_t)c->n_rel2 * c->dp, 288, 32,
                           (size_t)c->dim * c->hidden, (size_t)c->dim, (size_t)t.C3, (size_t)t.C3};
  DevBuf* ms[8] = {&t.mE, &t.mR, &t.mcw, &t.mcb, &t.mfw, &t.mfb, &t.mbw, &t.mbb};
  DevBuf* vs[8] = {&t.vE, &t.vR, &t.vcw, &t.vcb, &t.vfw, &t.vfb, &t.vbw, &t.vbb};
  for (int i = 0; i < 8; ++i)
    for (DevBuf* b : {ms[i], vs[i]}) {
      b->ensure(4 * sizes[i]);
      KP_HIP(hipMemsetAsync(b->p, 0, 4 * sizes[i], c->stream));
    }
  KP_HIP(hipStreamSynchronize(c->stream));
}

void conve_train_step(kp_ctx* c, int B, const int32_t* pairs, const int32_t* tail_off, const int32_t* tails,
                      const float* in_noise, const float* fm_noise, const float* hid_noise, float lr,
                      float label_smoothing, int bn_train) {
  KP_REQUIRE(c->model == KP_MODEL_CONVE && c->cvtrain, "kp_conve_train_step: call kp_conve_train_begin first");
  KP_REQUIRE(B >= 1, "kp_conve_train_step: empty batch");
  kp_cv_train& t = *c->cvtrain;
  const int N = c->n_ent, NR = c->n_rel2, dp = c->dp, d = c->dim, H = d / 20, half = 20 * H, hid = c->hidden;
  const int W2 = H - 2, per_c = 38 * W2;
  KP_REQUIRE(hid == 32 * per_c && d % 4 == 0 && hid % 4 == 0, "kp_conve_train_step: dim must be 20 h, h >= 3, 4 | dim");
  for (int b = 0; b < B; ++b) {
    KP_REQUIRE(pairs[2 * b] >= 0 && pairs[2 * b] < N && pairs[2 * b + 1] >= 0 && pairs[2 * b + 1] < NR,
               "kp_conve_train_step: pair id out of range");
    KP_REQUIRE(tail_off[b + 1] >= tail_off[b], "kp_conve_train_step: bad tail offsets");
  }
  for (int k = 0; k < tail_off[B]; ++k) KP_REQUIRE(tails[k] >= 0 && tails[k] < N, "kp_conve_train_step: tail out of range");
  const int Bp = (B + 3) / 4 * 4;
  const int ldN = (N + 3) / 4 * 4;
  const size_t nE = (size_t)N * dp, nR = (size_t)NR * dp;
  auto fbuf = [&](DevBuf& b, size_t n) { return reinterpret_cast<float*>(b.ensure(4 * std::max<size_t>(n, 1))); };
  float* img = fbuf(t.img, (size_t)Bp * 2 * half);
  float* xh1 = fbuf(t.xh1, (size_t)Bp * 2 * half);
  float* x1 = fbuf(t.x1, (size_t)Bp * 2 * half);
  float* cv = fbuf(t.cv, (size_t)Bp * hid);
  float* xh2 = fbuf(t.xh2, (size_t)Bp * hid);
  float* pre2 = fbuf(t.pre2, (size_t)Bp * hid);
  float* f = fbuf(t.f, (size_t)Bp * hid);
  float* h = fbuf(t.h, (size_t)Bp * dp);
  float* hd = fbuf(t.hd, (size_t)Bp * dp);
  float* xh3 = fbuf(t.xh3, (size_t)Bp * dp);
  float* pre3 = fbuf(t.pre3, (size_t)Bp * dp);
  float* z = fbuf(t.z, (size_t)Bp * dp);
  float* P = fbuf(t.P, (size_t)Bp * ldN);
  float* ET = fbuf(t.ET, (size_t)dp * ldN);
  float* PT = fbuf(t.PT, (size_t)N * Bp);
  float* zT = fbuf(t.zT, (size_t)dp * Bp);
  float* dz = fbuf(t.dz, (size_t)Bp * dp);
  float* dh = fbuf(t.dh, (size_t)Bp * dp);
  float* dhT = fbuf(t.dhT, (size_t)dp * Bp);
  float* fT = fbuf(t.fT, (size_t)hid * Bp);
  float* WT = fbuf(t.WT, (size_t)hid * d);
  float* df = fbuf(t.df, (size_t)Bp * hid);
  float* dc = fbuf(t.dc, (size_t)Bp * hid);
  float* dx1 = fbuf(t.dx1, (size_t)Bp * 2 * half);
  float* dimg = fbuf(t.dimg, (size_t)Bp * 2 * half);
  float* mean = fbuf(t.mean, t.C3);
  float* var = fbuf(t.var, t.C3);
  float* gE = fbuf(t.gE, nE);
  float* gR = fbuf(t.gR, nR);
  float* gcw = fbuf(t.gcw, 288);
  float* gcb = fbuf(t.gcb, 32);
  float* gfw = fbuf(t.gfw, (size_t)d * hid);
  float* gfb = fbuf(t.gfb, d);
  float* gbw = fbuf(t.gbw, t.C3);
  float* gbb = fbuf(t.gbb, t.C3);
  float* bnw = t.bnw.as<float>();
  float* bnb = t.bnb.as<float>();
  float* rm = t.rm.as<float>();
  float* rv = t.rv.as<float>();
  const hipStream_t s = c->stream;

  // ---- uploads: pairs, targets, noise; the per-key CSR of the image-gradient halves
  int32_t* dpairs = upload(c, t.pairs, pairs, 2 * (size_t)B);
  int32_t* dtoff = upload(c, t.toff, tail_off, (size_t)B + 1);
  int32_t* dtails = upload(c, t.tails, tails, (size_t)std::max(1, tail_off[B]));
  float* nin = in_noise ? upload(c, t.nin, in_noise, (size_t)B * 2 * half) : nullptr;
  float* nfm = fm_noise ? upload(c, t.nfm, fm_noise, (size_t)B * 32) : nullptr;
  float* nhid = nullptr;
  if (hid_noise) {  // [B][d] -> the [Bp][dp] layout of h (padding rows / columns 0)
    std::vector<float> hn((size_t)Bp * dp, 0.f);
    for (int b = 0; b < B; ++b) std::memcpy(&hn[(size_t)b * dp], hid_noise + (size_t)b * d, 4 * (size_t)d);
    nhid = upload(c, t.nhid, hn.data(), hn.size());
  }
  std::vector<int32_t> keys, off, items;
  std::vector<std::pair<int32_t, int32_t>> ek;
  int nk[2];
  for (int part = 0; part < 2; ++part) {
    ek.clear();
    for (int b = 0; b < B; ++b) ek.emplace_back(pairs[2 * b + part], b);
    std::stable_sort(ek.begin(), ek.end(), [](auto& x, auto& y) { return x.first < y.first; });
    const int k0 = (int)keys.size();
    for (size_t i = 0; i < ek.size(); ++i) {
      if (i == 0 || ek[i].first != ek[i - 1].first) {
        keys.push_back(ek[i].first);
        off.push_back((int32_t)items.size());
      }
      items.push_back(ek[i].second);
    }
    off.push_back((int32_t)items.size());
    nk[part] = (int)keys.size() - k0;
  }
  int32_t* dkeys = upload(c, t.keys, keys.data(), keys.size());
  int32_t* doff = upload(c, t.off, off.data(), off.size());
  int32_t* ditems = upload(c, t.items, items.data(), items.size());
  const bool train = bn_train != 0;
  float* w1 = bnw;
  float* w2 = bnw + 1;
  float* w3 = bnw + 33;
  float* m1 = mean;
  float* m2 = mean + 1;
  float* m3 = mean + 33;
  float* v1 = var;
  float* v2 = var + 1;
  float* v3 = var + 33;
  if (!train) {  // eval-mode batch norm: the running statistics
    KP_HIP(hipMemcpyAsync(mean, rm, 4 * (size_t)t.C3, hipMemcpyDeviceToDevice, s));
    KP_HIP(hipMemcpyAsync(var, rv, 4 * (size_t)t.C3, hipMemcpyDeviceToDevice, s));
  }

  // ---- forward
  hipLaunchKernelGGL(cvt_image, dim3(B), dim3(128), 0, s, B, dpairs, c->dE, c->dR, dp, half, img);
  if (train) hipLaunchKernelGGL(cvt_bn_stats, dim3(1), dim3(256), 0, s, img, B, 2 * half, (long long)2 * half, 0LL, m1, v1);
  hipLaunchKernelGGL(cvt_bn_fwd, dim3(nblk((long long)B * 2 * half)), dim3(256), 0, s, img, B, 1, 2 * half,
                     (long long)2 * half, 0LL, m1, v1, w1, bnb, 0, nin, xh1, nullptr, x1);
  hipLaunchKernelGGL(cvt_conv_fwd, dim3(nblk((long long)B * hid)), dim3(256), 0, s, B, H, x1, c->d_conv_w, c->d_conv_b,
                     cv);
  if (train)
    hipLaunchKernelGGL(cvt_bn_stats, dim3(32), dim3(256), 0, s, cv, B, per_c, (long long)hid, (long long)per_c, m2, v2);
  hipLaunchKernelGGL(cvt_bn_fwd, dim3(nblk((long long)B * hid)), dim3(256), 0, s, cv, B, 32, per_c, (long long)hid,
                     (long long)per_c, m2, v2, w2, bnb + 1, 1, nfm, xh2, pre2, f);
  KP_HIP(hipGetLastError());
  if (Bp > B) KP_HIP(hipMemsetAsync(f + (size_t)B * hid, 0, 4 * (size_t)(Bp - B) * hid, s));
  launch_gemm_abt(c, f, hid, Bp, c->d_fc_w, hid, d, hid, h, dp, c->d_fc_b, 0, 1);
  hipLaunchKernelGGL(cvt_mul, dim3(nblk((long long)Bp * dp)), dim3(256), 0, s, (long long)Bp * dp, h, nhid, hd);
  if (train) hipLaunchKernelGGL(cvt_bn_stats, dim3(d), dim3(256), 0, s, hd, B, 1, (long long)dp, 1LL, m3, v3);
  KP_HIP(hipMemsetAsync(z, 0, 4 * (size_t)Bp * dp, s));
  hipLaunchKernelGGL(cvt_bn_fwd, dim3(nblk((long long)B * d)), dim3(256), 0, s, hd, B, d, 1, (long long)dp, 1LL, m3,
                     v3, w3, bnb + 33, 2, nullptr, xh3, pre3, z);
  KP_HIP(hipGetLastError());
  launch_gemm_abt(c, z, dp, Bp, c->dE, dp, N, dp, P, ldN, nullptr, 1, 1);
  const float inv_n = (float)(1.0 / (double)N);
  const float ylo = label_smoothing != 0.f ? inv_n : 0.f;
  const float yhi = label_smoothing != 0.f ? (float)(1.0 - (double)label_smoothing) * 1.0f + inv_n : 1.0f;
  const float gs = (float)(1.0 / ((double)B * (double)N));
  hipLaunchKernelGGL(cvt_bce_grad, dim3(nblk(ldN), Bp), dim3(256), 0, s, P, ldN, B, N, dtoff, dtails, ylo, yhi, gs);
  KP_HIP(hipGetLastError());

  // ---- backward: scores
  hipLaunchKernelGGL(cvt_transpose, dim3((dp + 31) / 32, (ldN + 31) / 32), dim3(256), 0, s, c->dE, N, dp, dp, ET, ldN);
  launch_gemm_abt(c, P, ldN, Bp, ET, ldN, dp, ldN, dz, dp, nullptr, 0, 1);
  hipLaunchKernelGGL(cvt_transpose, dim3((N + 31) / 32, (Bp + 31) / 32), dim3(256), 0, s, P, Bp, N, ldN, PT, Bp);
  hipLaunchKernelGGL(cvt_transpose, dim3((dp + 31) / 32, (Bp + 31) / 32), dim3(256), 0, s, z, Bp, dp, dp, zT, Bp);
  KP_HIP(hipGetLastError());
  launch_gemm_abt(c, PT, Bp, N, zT, Bp, dp, Bp, gE, dp, nullptr, 0, 1);
  // ReLU, BN3, hidden dropout
  hipLaunchKernelGGL(cvt_relu_bwd, dim3(nblk((long long)Bp * dp)), dim3(256), 0, s, (long long)Bp * dp, pre3, dz);
  KP_HIP(hipMemsetAsync(dh, 0, 4 * (size_t)Bp * dp, s));
  hipLaunchKernelGGL(cvt_bn_bwd, dim3(d), dim3(256), 0, s, dz, xh3, B, 1, (long long)dp, 1LL, v3, w3, (int)train, dh,
                     gbw + 33, gbb + 33);
  hipLaunchKernelGGL(cvt_mul, dim3(nblk((long long)Bp * dp)), dim3(256), 0, s, (long long)Bp * dp, dh, nhid, dh);
  KP_HIP(hipGetLastError());
  // FC: bias, weight (dh^T f), input (dh W)
  hipLaunchKernelGGL(cvt_colsum, dim3(nblk(d)), dim3(256), 0, s, dh, B, d, dp, gfb);
  hipLaunchKernelGGL(cvt_transpose, dim3((dp + 31) / 32, (Bp + 31) / 32), dim3(256), 0, s, dh, Bp, dp, dp, dhT, Bp);
  hipLaunchKernelGGL(cvt_transpose, dim3((hid + 31) / 32, (Bp + 31) / 32), dim3(256), 0, s, f, Bp, hid, hid, fT, Bp);
  KP_HIP(hipGetLastError());
  launch_gemm_abt(c, dhT, Bp, d, fT, Bp, hid, Bp, gfw, hid, nullptr, 0, 1);
  hipLaunchKernelGGL(cvt_transpose, dim3((hid + 31) / 32, (d + 31) / 32), dim3(256), 0, s, c->d_fc_w, d, hid, hid, WT, d);
  KP_HIP(hipGetLastError());
  launch_gemm_abt(c, dh, dp, Bp, WT, d, hid, d, df, hid, nullptr, 0, 1);
  // feature-map dropout, ReLU, BN2
  hipLaunchKernelGGL(cvt_fm_bwd, dim3(nblk((long long)B * hid)), dim3(256), 0, s, B, 32, per_c, pre2, nfm, df);
  hipLaunchKernelGGL(cvt_bn_bwd, dim3(32), dim3(256), 0, s, df, xh2, B, per_c, (long long)hid, (long long)per_c, v2, w2,
                     (int)train, dc, gbw + 1, gbb + 1);
  // conv
  hipLaunchKernelGGL(cvt_conv_bwd_w, dim3(32 * 10), dim3(256), 0, s, B, H, dc, x1, gcw, gcb);
  hipLaunchKernelGGL(cvt_conv_bwd_x, dim3(nblk((long long)B * 2 * half)), dim3(256), 0, s, B, H, dc, c->d_conv_w, dx1);
  // input dropout, BN1
  hipLaunchKernelGGL(cvt_mul, dim3(nblk((long long)B * 2 * half)), dim3(256), 0, s, (long long)B * 2 * half, dx1, nin,
                     dx1);
  hipLaunchKernelGGL(cvt_bn_bwd, dim3(1), dim3(256), 0, s, dx1, xh1, B, 2 * half, (long long)2 * half, 0LL, v1, w1,
                     (int)train, dimg, gbw, gbb);
  KP_HIP(hipGetLastError());
  // the image gradient into the tables' gradients: lhs halves onto gE (already the
  // score GEMM's dense part), rel halves onto a cleared gR
  KP_HIP(hipMemsetAsync(gR, 0, 4 * nR, s));
  hipLaunchKernelGGL(cvt_scatter, dim3(nk[0]), dim3(64), 0, s, gE, dp, half, dkeys, doff, ditems, dimg, 0);
  hipLaunchKernelGGL(cvt_scatter, dim3(nk[1]), dim3(64), 0, s, gR, dp, half, dkeys + nk[0], doff + nk[0] + 1, ditems,
                     dimg, 1);
  KP_HIP(hipGetLastError());
  if (train) {
    const long long n1 = (long long)B * 2 * half, n2 = (long long)B * per_c, n3 = B;
    hipLaunchKernelGGL(cvt_bn_running, dim3(1), dim3(64), 0, s, 1, n1, m1, v1, rm, rv);
    hipLaunchKernelGGL(cvt_bn_running, dim3(1), dim3(64), 0, s, 32, n2, m2, v2, rm + 1, rv + 1);
    hipLaunchKernelGGL(cvt_bn_running, dim3(nblk(d)), dim3(256), 0, s, d, n3, m3, v3, rm + 33, rv + 33);
    KP_HIP(hipGetLastError());
  }  // eval mode (a batch of one pair): the running statistics stay

  // ---- Adam on every parameter
  ++t.step;
  AdamArgs a{};
  a.b1m = (float)(1.0 - 0.9);
  a.b2 = 0.999f;
  a.b2m = (float)(1.0 - 0.999);
  a.eps = 1e-8f;
  a.step_size = (float)((double)lr / (1.0 - std::pow(0.9, (double)t.step)));
  a.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(0.999, (double)t.step));
  auto adam = [&](float* X, DevBuf& M, DevBuf& V, const float* G, size_t n) {
    hipLaunchKernelGGL(cvt_adam, dim3(nblk((long long)n)), dim3(256), 0, s, X, M.as<float>(), V.as<float>(), G,
                       (long long)n, a);
  };
  adam(c->dE, t.mE, t.vE, gE, nE);
  adam(c->dR, t.mR, t.vR, gR, nR);
  adam(c->d_conv_w, t.mcw, t.vcw, gcw, 288);
  adam(c->d_conv_b, t.mcb, t.vcb, gcb, 32);
  adam(c->d_fc_w, t.mfw, t.vfw, gfw, (size_t)d * hid);
  adam(c->d_fc_b, t.mfb, t.vfb, gfb, d);
  adam(bnw, t.mbw, t.vbw, gbw, t.C3);
  adam(bnb, t.mbb, t.vbb, gbb, t.C3);
  KP_HIP(hipGetLastError());
  KP_HIP(hipStreamSynchronize(s));
  // the tables and layers changed: every derived image is stale
  c->e3_ready = c->e3pre_ready = c->eT_ready = c->cvf_ready = false;
  if (c->dEt) {
    (void)hipFree(c->dEt);
    c->dEt = nullptr;
  }
}

void conve_train_read(kp_ctx* c, float* conv_w, float* conv_b, float* fc_w, float* fc_b, float* bn_w, float* bn_b,
                      float* bn_m, float* bn_v) {
  KP_REQUIRE(c->model == KP_MODEL_CONVE && c->cvtrain, "kp_conve_train_read: no ConvE training state");
  kp_cv_train& t = *c->cvtrain;
  KP_HIP(hipStreamSynchronize(c->stream));
  KP_HIP(hipMemcpy(conv_w, c->d_conv_w, 4 * 288, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(conv_b, c->d_conv_b, 4 * 32, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(fc_w, c->d_fc_w, 4 * (size_t)c->dim * c->hidden, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(fc_b, c->d_fc_b, 4 * (size_t)c->dim, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(bn_w, t.bnw.p, 4 * (size_t)t.C3, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(bn_b, t.bnb.p, 4 * (size_t)t.C3, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(bn_m, t.rm.p, 4 * (size_t)t.C3, hipMemcpyDeviceToHost));
  KP_HIP(hipMemcpy(bn_v, t.rv.p, 4 * (size_t)t.C3, hipMemcpyDeviceToHost));
}
