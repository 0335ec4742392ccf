// kp_train.hip -- full-model training on the device, for the retraining step of
// explanation verification (src/verify_explanations.py:141-143 and :230-232: a fresh
// model with init_random=True trained by its optimizer on the edited training set).
//
// ComplEx + MultiClassNLLOptimizer (src/link_prediction/optimization/
// multiclass_nll_optimizer.py:101-135, models/complex.py:58-86, regularizers.py N3):
// per batch of B triples (h, r, t) of the epoch's permutation
//   Q     = lhs o rel                        (complex product, [Re | Im])
//   S     = Q . E^T                          (scores against every entity)
//   dS    = (softmax(S) - onehot(t)) / B     (CrossEntropyLoss(mean) backward)
//   dQ    = dS . E,   dE = dS^T . Q          (the full-table use of E)
//   d lhs, d rel through the complex product; N3 on |lhs|, |rel|, |rhs|:
//           d x = 3 (w / B) |f| x            (|f| = sqrt(re^2 + im^2))
//   optimizer (Adagrad / Adam / SGD, torch op order) over the WHOLE tables: the
//   entity gradient is dense, and Adam moves rows with a zero gradient too.
// The three GEMMs run on kp_gemm_abt (fp32 MFMA, C = A B^T) over transposed copies;
// the per-row gradients of lhs / rel / rhs are summed into the tables per key in
// batch order (a host-built CSR), so a run is deterministic.  Not the hot path: the
// verification retrains once per explained set.
#include <algorithm>
#include <cmath>
#include <vector>

#include "kp_attn.hpp"  // cx_q
#include "kp_common.hpp"

namespace {

struct TrOpt {
  int kind;
  float lr, b2, eps, one_minus_b1, one_minus_b2, step_size, bc2_sqrt;
};

// Q[b] = E[h] o R[r] for the batch rows b < B (rows B .. Bp zero)
__global__ void kp_tr_q(const float* __restrict__ E, const float* __restrict__ R, int dp, int half,
                        const int32_t* __restrict__ bt, int B, int Bp, float* __restrict__ Q) {
  const int b = blockIdx.x;
  if (b >= Bp) return;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) {
    float v = 0.f;
    if (b < B) v = kpattn::cx_q(E + (size_t)bt[3 * b] * dp, R + (size_t)bt[3 * b + 1] * dp, d, half);
    Q[(size_t)b * dp + d] = v;
  }
}

// row b of S [Bp][ld]: (softmax - onehot(t)) * inv_b in place; rows >= B zeroed
__global__ __launch_bounds__(256) void kp_tr_softmax(float* __restrict__ S, int ld, int n_ent,
                                                     const int32_t* __restrict__ bt, int B, float inv_b) {
  const int b = blockIdx.x;
  float* row = S + (size_t)b * ld;
  if (b >= B) {
    for (int e = threadIdx.x; e < ld; e += blockDim.x) row[e] = 0.f;
    return;
  }
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float m = -3.0e38f;
  for (int e = threadIdx.x; e < n_ent; e += blockDim.x) m = fmaxf(m, row[e]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float l = 0.f;
  for (int e = threadIdx.x; e < n_ent; e += blockDim.x) l += expf(row[e] - m);
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
  if (lane == 0) red[w] = l;
  __syncthreads();
  l = (red[0] + red[1]) + (red[2] + red[3]);
  const float inv_l = 1.0f / l;
  const int t = bt[3 * b + 2];
  for (int e = threadIdx.x; e < ld; e += blockDim.x) {
    float g = 0.f;
    if (e < n_ent) g = (expf(row[e] - m) * inv_l - (e == t ? 1.0f : 0.0f)) * inv_b;
    row[e] = g;
  }
}

// out[c][r] = in[r][c] for r < rows, c < cols (32 x 32 tiles through LDS)
__global__ void kp_tr_transpose(const float* __restrict__ in, int rows, int cols, int ld_in, float* __restrict__ out,
                                int ld_out) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? in[(size_t)r * ld_in + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) out[(size_t)c * ld_out + r] = tile[tx][i];
  }
}

// per batch row: the gradients of lhs (complex product + N3), rel (complex product +
// N3) and rhs (N3 only); reg3 = 3 w / B
__global__ void kp_tr_rowgrads(const float* __restrict__ E, const float* __restrict__ R, int dp, int half,
                               const int32_t* __restrict__ bt, int B, const float* __restrict__ dQ, float reg3,
                               float* __restrict__ gl, float* __restrict__ gr, float* __restrict__ gt) {
  const int b = blockIdx.x;
  if (b >= B) return;
  const float* lhs = E + (size_t)bt[3 * b] * dp;
  const float* rel = R + (size_t)bt[3 * b + 1] * dp;
  const float* rhs = E + (size_t)bt[3 * b + 2] * dp;
  const float* dq = dQ + (size_t)b * dp;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float a = lhs[i], bb = lhs[i + half], c = rel[i], e = rel[i + half];
    const float dr = dq[i], di = dq[i + half];
    // real = a c - b e, imag = a e + b c
    float la = dr * c + di * e, lb = di * c - dr * e;
    float rc = dr * a + di * bb, re = di * a - dr * bb;
    float ta = 0.f, tb = 0.f;
    if (reg3 != 0.f) {
      const float ml = sqrtf(a * a + bb * bb), mr = sqrtf(c * c + e * e);
      const float x = rhs[i], y = rhs[i + half], mt = sqrtf(x * x + y * y);
      la += (reg3 * ml) * a;
      lb += (reg3 * ml) * bb;
      rc += (reg3 * mr) * c;
      re += (reg3 * mr) * e;
      ta = (reg3 * mt) * x;
      tb = (reg3 * mt) * y;
    }
    gl[(size_t)b * dp + i] = la;
    gl[(size_t)b * dp + i + half] = lb;
    gr[(size_t)b * dp + i] = rc;
    gr[(size_t)b * dp + i + half] = re;
    gt[(size_t)b * dp + i] = ta;
    gt[(size_t)b * dp + i + half] = tb;
  }
  // the row padding [2 half, dp): kp_tr_scatter sums all dp columns into the table
  // gradient, and the buffers are not cleared between calls
  for (int i = 2 * half + threadIdx.x; i < dp; i += blockDim.x) {
    gl[(size_t)b * dp + i] = 0.f;
    gr[(size_t)b * dp + i] = 0.f;
    gt[(size_t)b * dp + i] = 0.f;
  }
}

// G[key] += the key's row gradients in batch order (items: 4 row + role; role 0 = lhs,
// 1 = rhs, 2 = rel)
__global__ void kp_tr_scatter(float* __restrict__ G, int dp, const int32_t* __restrict__ keys,
                              const int32_t* __restrict__ off, const int32_t* __restrict__ items,
                              const float* __restrict__ gl, const float* __restrict__ gt,
                              const float* __restrict__ gr) {
  const int k = blockIdx.x;
  const int i0 = off[k], i1 = off[k + 1];
  float* g = G + (size_t)keys[k] * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) {
    float acc = 0.f;
    for (int i = i0; i < i1; ++i) {
      const int it = items[i], row = it >> 2, role = it & 3;
      const float* src = role == 0 ? gl : (role == 1 ? gt : gr);
      acc += src[(size_t)row * dp + d];
    }
    g[d] += acc;
  }
}

// one optimizer step over a whole table (torch op order: optim/adagrad.py, adam.py, sgd.py)
__global__ void kp_tr_opt(float* __restrict__ X, float* __restrict__ S1, float* __restrict__ S2,
                          const float* __restrict__ G, size_t n, TrOpt o) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = G[i];
  float x = X[i];
  if (o.kind == KP_OPT_ADAGRAD) {
    const float s = S1[i] + g * g;
    x = x + (-o.lr * g) / (sqrtf(s) + o.eps);
    S1[i] = s;
  } else if (o.kind == KP_OPT_ADAM) {
    float m = S1[i], v = S2[i];
    m = m + o.one_minus_b1 * (g - m);
    v = v * o.b2;
    v = v + (o.one_minus_b2 * g) * g;
    x = x + (-o.step_size * m) / (sqrtf(v) / o.bc2_sqrt + o.eps);
    S1[i] = m;
    S2[i] = v;
  } else {
    x = x + (-o.lr) * g;
  }
  X[i] = x;
}

// TransE: per row i of the batch (positive row pos[i], corrupted row neg[i]) the
// gradients of MarginRankingLoss(margin, mean) on the L2 distances and of the L2
// regulariser (mean of each factor squared, times w / 3, averaged over the positive and
// negative factors): roles 0..2 = positive lhs, rel, rhs; 3..5 = negative ones.
//   score = ||lhs + rel - rhs||,  hinge_i = score_pos - score_neg + margin > 0
//   d lhs = (+-1 / B) (lhs + rel - rhs) / score [hinge] + (w / (3 B d)) lhs, etc.
// l1 (norm p = 1): score = sum |lhs + rel - rhs|, d lhs = (+-1 / B) sgn(lhs + rel - rhs) [hinge] + ...
__global__ void kp_tr_te_rowgrads(const float* __restrict__ E, const float* __restrict__ R, int dp, int dim,
                                  const int32_t* __restrict__ pos, const int32_t* __restrict__ neg, int B,
                                  float margin, float inv_b, float wl, int l1, float* __restrict__ grads) {
  const int i = blockIdx.x;
  if (i >= B) return;
  const int lane = threadIdx.x;  // one wave per row
  const float *ph = E + (size_t)pos[3 * i] * dp, *pr = R + (size_t)pos[3 * i + 1] * dp,
              *pt = E + (size_t)pos[3 * i + 2] * dp;
  const float *nh = E + (size_t)neg[3 * i] * dp, *nr = R + (size_t)neg[3 * i + 1] * dp,
              *nt = E + (size_t)neg[3 * i + 2] * dp;
  float sp = 0.f, sn = 0.f;
  for (int d = lane; d < dim; d += 64) {
    const float a = (ph[d] + pr[d]) - pt[d], b = (nh[d] + nr[d]) - nt[d];
    sp += l1 ? fabsf(a) : a * a;
    sn += l1 ? fabsf(b) : b * b;
  }
  sp = wave_sum(sp);
  sn = wave_sum(sn);
  const float np_ = l1 ? sp : sqrtf(sp), nn = l1 ? sn : sqrtf(sn);
  const bool hinge = (np_ - nn) + margin > 0.f;
  const float cp = hinge ? (l1 ? inv_b : inv_b / np_) : 0.f, cn = hinge ? (l1 ? -inv_b : -inv_b / nn) : 0.f;
  float* g = grads + (size_t)i * 6 * dp;
  for (int d = lane; d < dp; d += 64) {
    float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (d < dim) {
      float a = (ph[d] + pr[d]) - pt[d], b = (nh[d] + nr[d]) - nt[d];
      if (l1) {
        a = a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f);
        b = b > 0.f ? 1.f : (b < 0.f ? -1.f : 0.f);
      }
      v[0] = cp * a + wl * ph[d];
      v[1] = cp * a + wl * pr[d];
      v[2] = -cp * a + wl * pt[d];
      v[3] = cn * b + wl * nh[d];
      v[4] = cn * b + wl * nr[d];
      v[5] = -cn * b + wl * nt[d];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) g[(size_t)k * dp + d] = v[k];
  }
}

// G[key] += the key's row gradients in batch order (items: 8 row + role, rows of
// kp_tr_te_rowgrads' [B][6][dp] output)
__global__ void kp_tr_scatter6(float* __restrict__ G, int dp, const int32_t* __restrict__ keys,
                               const int32_t* __restrict__ off, const int32_t* __restrict__ items,
                               const float* __restrict__ grads) {
  const int k = blockIdx.x;
  const int i0 = off[k], i1 = off[k + 1];
  float* g = G + (size_t)keys[k] * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) {
    float acc = 0.f;
    for (int i = i0; i < i1; ++i) {
      const int it = items[i];
      acc += grads[((size_t)(it >> 3) * 6 + (it & 7)) * dp + d];
    }
    g[d] += acc;
  }
}

}  // namespace

// Optimizer state and scratch of a training run, owned by the context.
struct kp_train_state {
  DevBuf s1E, s2E, s1R, s2R, gE, gR, bt, Q, QT, S, ST, ET, dQ, gl, gr, gt, keys, off, items;
  int64_t step = 0;
};

void train_state_free(kp_ctx* c) {
  delete c->train;
  c->train = nullptr;
}

// One epoch of MultiClassNLLOptimizer.epoch on the context's own tables.
void complex_train_epoch(kp_ctx* c, const kp_hp* hp, int n, const int32_t* triples, const int32_t* perm, int epoch) {
  KP_REQUIRE(c->model == KP_MODEL_COMPLEX, "kp_train_epoch: ComplEx contexts only");
  KP_REQUIRE(n > 0 && hp->batch_size > 0, "kp_train_epoch: empty training set or batch");
  for (int i = 0; i < n; ++i) {
    KP_REQUIRE(perm[i] >= 0 && perm[i] < n, "kp_train_epoch: permutation value out of range");
    const int32_t* t = triples + 3 * (size_t)i;
    KP_REQUIRE(t[0] >= 0 && t[0] < c->n_ent && t[2] >= 0 && t[2] < c->n_ent && t[1] >= 0 && t[1] < c->n_rel2,
               "kp_train_epoch: triple id out of range");
  }
  if (epoch == 0 || !c->train) {
    delete c->train;
    c->train = new kp_train_state();
  }
  kp_train_state& st = *c->train;
  const int dp = c->dp, half = c->dim / 2, N = c->n_ent, NR = c->n_rel2;
  const size_t nE = (size_t)N * dp, nR = (size_t)NR * dp;
  if (st.step == 0) {
    for (DevBuf* b : {&st.s1E, &st.s2E}) {
      b->ensure(4 * nE);
      KP_HIP(hipMemsetAsync(b->p, 0, 4 * nE, c->stream));
    }
    for (DevBuf* b : {&st.s1R, &st.s2R}) {
      b->ensure(4 * nR);
      KP_HIP(hipMemsetAsync(b->p, 0, 4 * nR, c->stream));
    }
  }
  const int bs = std::min(hp->batch_size, n);
  const int Bp_max = (bs + 3) / 4 * 4;
  const int ldS = (N + 3) / 4 * 4;
  float* gE = reinterpret_cast<float*>(st.gE.ensure(4 * nE));
  float* gR = reinterpret_cast<float*>(st.gR.ensure(4 * nR));
  int32_t* dbt = reinterpret_cast<int32_t*>(st.bt.ensure(4 * 3 * (size_t)bs));
  float* Q = reinterpret_cast<float*>(st.Q.ensure(4 * (size_t)Bp_max * dp));
  float* QT = reinterpret_cast<float*>(st.QT.ensure(4 * (size_t)dp * Bp_max));
  float* S = reinterpret_cast<float*>(st.S.ensure(4 * (size_t)Bp_max * ldS));
  float* ST = reinterpret_cast<float*>(st.ST.ensure(4 * (size_t)ldS * Bp_max));
  float* ET = reinterpret_cast<float*>(st.ET.ensure(4 * (size_t)dp * ldS));
  float* dQ = reinterpret_cast<float*>(st.dQ.ensure(4 * (size_t)Bp_max * dp));
  float* gl = reinterpret_cast<float*>(st.gl.ensure(4 * (size_t)bs * dp));
  float* gr = reinterpret_cast<float*>(st.gr.ensure(4 * (size_t)bs * dp));
  float* gt = reinterpret_cast<float*>(st.gt.ensure(4 * (size_t)bs * dp));
  int32_t* dkeys = reinterpret_cast<int32_t*>(st.keys.ensure(4 * 3 * (size_t)bs));
  int32_t* doff = reinterpret_cast<int32_t*>(st.off.ensure(4 * (3 * (size_t)bs + 2)));
  int32_t* ditems = reinterpret_cast<int32_t*>(st.items.ensure(4 * 3 * (size_t)bs));

  TrOpt o{};
  o.kind = hp->optimizer;
  o.lr = hp->lr;
  o.b2 = hp->beta2;
  o.eps = hp->eps;
  o.one_minus_b1 = (float)(1.0 - (double)hp->beta1);
  o.one_minus_b2 = (float)(1.0 - (double)hp->beta2);
  const float reg3_per_b = 3.0f * hp->reg_weight;

  std::vector<int32_t> hbt(3 * (size_t)bs), keys, off, items;
  std::vector<std::pair<int64_t, int32_t>> ek;  // (key, item) sorted stably by key
  // batch_start advances by hp->batch_size (multiclass_nll_optimizer.py:118)
  for (int start = 0; start < n; start += hp->batch_size) {
    // the host vectors below are refilled per batch: the previous batch's copies from
    // them must have left
    if (start) KP_HIP(hipStreamSynchronize(c->stream));
    const int B = std::min(bs, n - start);
    const int Bp = (B + 3) / 4 * 4;
    for (int b = 0; b < B; ++b) std::memcpy(&hbt[3 * (size_t)b], triples + 3 * (size_t)perm[start + b], 12);
    // per-key CSR of the row gradients, entity keys then relation keys, batch order
    ek.clear();
    for (int b = 0; b < B; ++b) {
      ek.emplace_back((int64_t)hbt[3 * b], 4 * b + 0);
      ek.emplace_back((int64_t)hbt[3 * b + 2], 4 * b + 1);
    }
    std::stable_sort(ek.begin(), ek.end(),
                     [](const std::pair<int64_t, int32_t>& x, const std::pair<int64_t, int32_t>& y) {
                       return x.first < y.first;
                     });
    keys.clear();
    off.clear();
    items.clear();
    for (size_t i = 0; i < ek.size(); ++i) {
      if (i == 0 || ek[i].first != ek[i - 1].first) {
        keys.push_back((int32_t)ek[i].first);
        off.push_back((int32_t)items.size());
      }
      items.push_back(ek[i].second);
    }
    off.push_back((int32_t)items.size());
    const int n_ek = (int)keys.size();
    ek.clear();
    for (int b = 0; b < B; ++b) ek.emplace_back((int64_t)hbt[3 * b + 1], 4 * b + 2);
    std::stable_sort(ek.begin(), ek.end(),
                     [](const std::pair<int64_t, int32_t>& x, const std::pair<int64_t, int32_t>& y) {
                       return x.first < y.first;
                     });
    const int rk0 = (int)keys.size();
    for (size_t i = 0; i < ek.size(); ++i) {
      if (i == 0 || ek[i].first != ek[i - 1].first) {
        keys.push_back((int32_t)ek[i].first);
        off.push_back((int32_t)items.size());
      }
      items.push_back(ek[i].second);
    }
    off.push_back((int32_t)items.size());
    const int n_rk = (int)keys.size() - rk0;
    KP_HIP(hipMemcpyAsync(dbt, hbt.data(), 12 * (size_t)B, hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(dkeys, keys.data(), 4 * keys.size(), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(doff, off.data(), 4 * off.size(), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(ditems, items.data(), 4 * items.size(), hipMemcpyHostToDevice, c->stream));

    const float inv_b = 1.0f / (float)B;
    hipLaunchKernelGGL(kp_tr_q, dim3(Bp), dim3(128), 0, c->stream, c->dE, c->dR, dp, half, dbt, B, Bp, Q);
    KP_HIP(hipGetLastError());
    // S = Q E^T, then dS in place
    launch_gemm_abt(c, Q, dp, Bp, c->dE, dp, N, dp, S, ldS, nullptr, 0, 1);
    hipLaunchKernelGGL(kp_tr_softmax, dim3(Bp), dim3(256), 0, c->stream, S, ldS, N, dbt, B, inv_b);
    KP_HIP(hipGetLastError());
    // dQ = dS E: A = dS [Bp][ldS], B = E^T [dp][ldS]
    hipLaunchKernelGGL(kp_tr_transpose, dim3((dp + 31) / 32, (ldS + 31) / 32), dim3(256), 0, c->stream, c->dE, N,
                       dp, dp, ET, ldS);
    KP_HIP(hipGetLastError());
    if (ldS > N) KP_HIP(hipMemset2DAsync(ET + N, 4 * (size_t)ldS, 0, 4 * (size_t)(ldS - N), dp, c->stream));
    launch_gemm_abt(c, S, ldS, Bp, ET, ldS, dp, ldS, dQ, dp, nullptr, 0, 1);
    // dE = dS^T Q: A = dS^T [N][Bp], B = Q^T [dp][Bp]
    hipLaunchKernelGGL(kp_tr_transpose, dim3((N + 31) / 32, (Bp + 31) / 32), dim3(256), 0, c->stream, S, Bp, N,
                       ldS, ST, Bp);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL(kp_tr_transpose, dim3((dp + 31) / 32, (Bp + 31) / 32), dim3(256), 0, c->stream, Q, Bp, dp,
                       dp, QT, Bp);
    KP_HIP(hipGetLastError());
    launch_gemm_abt(c, ST, Bp, N, QT, Bp, dp, Bp, gE, dp, nullptr, 0, 1);
    // row gradients, summed per key into gE / gR
    hipLaunchKernelGGL(kp_tr_rowgrads, dim3(B), dim3(128), 0, c->stream, c->dE, c->dR, dp, half, dbt, B, dQ,
                       reg3_per_b * inv_b, gl, gr, gt);
    KP_HIP(hipGetLastError());
    KP_HIP(hipMemsetAsync(gR, 0, 4 * nR, c->stream));
    hipLaunchKernelGGL(kp_tr_scatter, dim3(n_ek), dim3(128), 0, c->stream, gE, dp, dkeys, doff, ditems, gl, gt, gr);
    KP_HIP(hipGetLastError());
    if (n_rk > 0) {
      hipLaunchKernelGGL(kp_tr_scatter, dim3(n_rk), dim3(128), 0, c->stream, gR, dp, dkeys + rk0, doff + rk0 + 1,
                         ditems, gl, gt, gr);
      KP_HIP(hipGetLastError());
    }
    // optimizer step over both tables
    ++st.step;
    o.step_size = (float)((double)hp->lr / (1.0 - std::pow((double)hp->beta1, (double)st.step)));
    o.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)hp->beta2, (double)st.step));
    hipLaunchKernelGGL(kp_tr_opt, dim3((unsigned)((nE + 255) / 256)), dim3(256), 0, c->stream, c->dE,
                       st.s1E.as<float>(), st.s2E.as<float>(), gE, nE, o);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL(kp_tr_opt, dim3((unsigned)((nR + 255) / 256)), dim3(256), 0, c->stream, c->dR,
                       st.s1R.as<float>(), st.s2R.as<float>(), gR, nR, o);
    KP_HIP(hipGetLastError());
  }
  KP_HIP(hipStreamSynchronize(c->stream));
  // the tables changed: the attention image and its prefix sums are stale
  c->e3_ready = false;
  c->e3pre_ready = false;
  c->eT_ready = false;
}

// One PairwiseRankingOptimizer epoch (TransE) on the context's own tables: positive
// rows pos[n][3] and corrupted rows neg[n][3] in the epoch's order, batches of
// hp->batch_size, Adam over both whole tables.
void transe_train_epoch(kp_ctx* c, const kp_hp* hp, int n, const int32_t* pos, const int32_t* neg, int epoch) {
  KP_REQUIRE(c->model == KP_MODEL_TRANSE, "kp_train_epoch: TransE contexts only");
  KP_REQUIRE(n > 0 && hp->batch_size > 0, "kp_train_epoch: empty training set or batch");
  for (int i = 0; i < 3 * n; i += 3)
    for (const int32_t* t : {pos + i, neg + i})
      KP_REQUIRE(t[0] >= 0 && t[0] < c->n_ent && t[2] >= 0 && t[2] < c->n_ent && t[1] >= 0 && t[1] < c->n_rel2,
                 "kp_train_epoch: triple id out of range");
  if (epoch == 0 || !c->train) {
    delete c->train;
    c->train = new kp_train_state();
  }
  kp_train_state& st = *c->train;
  const int dp = c->dp, dim = c->dim, N = c->n_ent, NR = c->n_rel2;
  const size_t nE = (size_t)N * dp, nR = (size_t)NR * dp;
  if (st.step == 0) {
    for (DevBuf* b : {&st.s1E, &st.s2E}) {
      b->ensure(4 * nE);
      KP_HIP(hipMemsetAsync(b->p, 0, 4 * nE, c->stream));
    }
    for (DevBuf* b : {&st.s1R, &st.s2R}) {
      b->ensure(4 * nR);
      KP_HIP(hipMemsetAsync(b->p, 0, 4 * nR, c->stream));
    }
  }
  const int bs = hp->batch_size;
  const int Bmax = std::min(bs, n);
  float* gE = reinterpret_cast<float*>(st.gE.ensure(4 * nE));
  float* gR = reinterpret_cast<float*>(st.gR.ensure(4 * nR));
  int32_t* dpos = reinterpret_cast<int32_t*>(st.bt.ensure(4 * 3 * (size_t)n));
  int32_t* dneg = reinterpret_cast<int32_t*>(st.Q.ensure(4 * 3 * (size_t)n));
  float* grads = reinterpret_cast<float*>(st.gl.ensure(4 * 6 * (size_t)Bmax * dp));
  int32_t* dkeys = reinterpret_cast<int32_t*>(st.keys.ensure(4 * 6 * (size_t)Bmax));
  int32_t* doff = reinterpret_cast<int32_t*>(st.off.ensure(4 * (6 * (size_t)Bmax + 2)));
  int32_t* ditems = reinterpret_cast<int32_t*>(st.items.ensure(4 * 6 * (size_t)Bmax));
  KP_HIP(hipMemcpyAsync(dpos, pos, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  KP_HIP(hipMemcpyAsync(dneg, neg, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream));

  TrOpt o{};
  o.kind = KP_OPT_ADAM;
  o.lr = hp->lr;
  o.b2 = hp->beta2;
  o.eps = hp->eps;
  o.one_minus_b1 = (float)(1.0 - (double)hp->beta1);
  o.one_minus_b2 = (float)(1.0 - (double)hp->beta2);
  std::vector<int32_t> keys, off, items;
  std::vector<std::pair<int64_t, int32_t>> ek;
  for (int start = 0; start < n; start += bs) {
    if (start) KP_HIP(hipStreamSynchronize(c->stream));  // host CSR vectors are refilled
    const int B = std::min(bs, n - start);
    const int32_t* P = pos + 3 * (size_t)start;
    const int32_t* Ng = neg + 3 * (size_t)start;
    // per-key CSR, entity keys (roles 0, 2, 3, 5) then relation keys (roles 1, 4), batch order
    int n_ek = 0;
    keys.clear();
    off.clear();
    items.clear();
    for (int pass = 0; pass < 2; ++pass) {
      ek.clear();
      for (int b = 0; b < B; ++b) {
        if (pass == 0) {
          ek.emplace_back(P[3 * b], 8 * b + 0);
          ek.emplace_back(P[3 * b + 2], 8 * b + 2);
          ek.emplace_back(Ng[3 * b], 8 * b + 3);
          ek.emplace_back(Ng[3 * b + 2], 8 * b + 5);
        } else {
          ek.emplace_back(P[3 * b + 1], 8 * b + 1);
          ek.emplace_back(Ng[3 * b + 1], 8 * b + 4);
        }
      }
      std::stable_sort(ek.begin(), ek.end(),
                       [](const std::pair<int64_t, int32_t>& x, const std::pair<int64_t, int32_t>& y) {
                         return x.first < y.first;
                       });
      for (size_t i = 0; i < ek.size(); ++i) {
        if (i == 0 || ek[i].first != ek[i - 1].first) {
          keys.push_back((int32_t)ek[i].first);
          off.push_back((int32_t)items.size());
        }
        items.push_back(ek[i].second);
      }
      off.push_back((int32_t)items.size());
      if (pass == 0) n_ek = (int)keys.size();  // the relation part's keys and offsets follow
    }
    const int n_rk = (int)keys.size() - n_ek;
    KP_HIP(hipMemcpyAsync(dkeys, keys.data(), 4 * keys.size(), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(doff, off.data(), 4 * off.size(), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(ditems, items.data(), 4 * items.size(), hipMemcpyHostToDevice, c->stream));
    const float inv_b = 1.0f / (float)B;
    const float wl = hp->reg_weight / (3.0f * (float)B * (float)dim);
    hipLaunchKernelGGL(kp_tr_te_rowgrads, dim3(B), dim3(64), 0, c->stream, c->dE, c->dR, dp, dim,
                       dpos + 3 * (size_t)start, dneg + 3 * (size_t)start, B, hp->margin, inv_b, wl,
                       c->te_norm == 1 ? 1 : 0, grads);
    KP_HIP(hipGetLastError());
    KP_HIP(hipMemsetAsync(gE, 0, 4 * nE, c->stream));
    KP_HIP(hipMemsetAsync(gR, 0, 4 * nR, c->stream));
    hipLaunchKernelGGL(kp_tr_scatter6, dim3(n_ek), dim3(128), 0, c->stream, gE, dp, dkeys, doff, ditems, grads);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL(kp_tr_scatter6, dim3(n_rk), dim3(128), 0, c->stream, gR, dp, dkeys + n_ek, doff + n_ek + 1,
                       ditems, grads);
    KP_HIP(hipGetLastError());
    ++st.step;
    o.step_size = (float)((double)hp->lr / (1.0 - std::pow((double)hp->beta1, (double)st.step)));
    o.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)hp->beta2, (double)st.step));
    hipLaunchKernelGGL(kp_tr_opt, dim3((unsigned)((nE + 255) / 256)), dim3(256), 0, c->stream, c->dE,
                       st.s1E.as<float>(), st.s2E.as<float>(), gE, nE, o);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL(kp_tr_opt, dim3((unsigned)((nR + 255) / 256)), dim3(256), 0, c->stream, c->dR,
                       st.s1R.as<float>(), st.s2R.as<float>(), gR, nR, o);
    KP_HIP(hipGetLastError());
  }
  KP_HIP(hipStreamSynchronize(c->stream));
  c->e3_ready = false;
  c->e3pre_ready = false;
  c->eT_ready = false;
}
