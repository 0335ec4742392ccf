// kp_baselines.hip -- the two baseline relevance engines of the reference
// (SURVEY.md §8(f) f4), batched on the GPU:
//
//   data poisoning  src/relevance_engines/data_poisoning_engine.py:21-152
//     per candidate: the gradient of the prediction's ComplEx score w.r.t. the
//     perspective entity, that entity's embedding moved by epsilon along it, and
//     the candidate triple's score with and without the move.  One wave per
//     candidate (latency kernel: three rows in, one float out).
//
//   CRIAGE          src/relevance_engines/criage_engine.py:30-177
//     per perspective entity e: H_e = sum over its tail triples (h, r, e) of
//     sig'(e . x) x^T x with x = E_h * R_r (float32 terms, float64 sum in triple
//     order, criage_engine.py:74-104); per candidate: A = H_e + sig'(e . z_t)
//     z_t^T z_t, y = A^{-1} z_t^T by Gaussian elimination with partial pivoting in
//     float64 (the reference inverts A with LAPACK; A is symmetric, so z_t A^{-1}
//     = y^T), relevance = z_p . ((1 - sig) y).  z = criage_first_step: the ComplEx
//     query (complex.py:131) or the ConvE encoder output (conve.py:102-124).
//     One workgroup per candidate eliminates its own D x D system in a device
//     workspace (float64 VALU; D^3/3 multiply-adds, bound by the L2 traffic of
//     the trailing updates).
#include <cmath>

#include "kp_common.hpp"

namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------- data poisoning
// items[i] = (pred s, p, o, perspective entity, triple h, r, t)
__global__ __launch_bounds__(256) void kp_dp_complex(int n, const int32_t* __restrict__ items,
                                                     const float* __restrict__ E, const float* __restrict__ R,
                                                     int dp, int rd, float eps, float lambd, float step_sign,
                                                     float rel_sign, float* __restrict__ out) {
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (item >= n) return;
  const int32_t* it = items + 7 * (size_t)item;
  const int s = it[0], p = it[1], o = it[2], e = it[3], h = it[4], r = it[5], t = it[6];
  const float* Ls = E + (size_t)s * dp;
  const float* Rp = R + (size_t)p * dp;
  const float* Ho = E + (size_t)o * dp;
  const float* Ee = E + (size_t)e * dp;
  const float* Lh = E + (size_t)h * dp;
  const float* Rr = R + (size_t)r * dp;
  const float* Ht = E + (size_t)t * dp;
  float orig = 0.f, pert = 0.f;
  for (int j = lane; j < rd; j += 64) {
    const float l0 = Ls[j], l1 = Ls[rd + j], r0 = Rp[j], r1 = Rp[rd + j], h0 = Ho[j], h1 = Ho[rd + j];
    float g0, g1;
    if (e == s) {  // d score / d lhs (data_poisoning_engine.py:37-47; autograd's two products per element)
      g0 = h0 * r0 + h1 * r1;
      g1 = -(h0 * r1) + h1 * r0;
    } else {  // d score / d rhs
      g0 = l0 * r0 - l1 * r1;
      g1 = l0 * r1 + l1 * r0;
    }
    const float p0 = Ee[j] + step_sign * (eps * g0), p1 = Ee[rd + j] + step_sign * (eps * g1);
    const float a0 = Lh[j], a1 = Lh[rd + j], c0 = Rr[j], c1 = Rr[rd + j], b0 = Ht[j], b1 = Ht[rd + j];
    // complex.py:48-57: (l0 r0 - l1 r1) rh0 + (l0 r1 + l1 r0) rh1
    orig += (a0 * c0 - a1 * c1) * b0 + (a0 * c1 + a1 * c0) * b1;
    const bool on_lhs = (h == e);  // data_poisoning_engine.py:79-82: else the rhs is perturbed
    const float x0 = on_lhs ? p0 : a0, x1 = on_lhs ? p1 : a1;
    const float y0 = on_lhs ? b0 : p0, y1 = on_lhs ? b1 : p1;
    pert += (x0 * c0 - x1 * c1) * y0 + (x0 * c1 + x1 * c0) * y1;
  }
  orig = wsum(orig);
  pert = wsum(pert);
  if (lane == 0) out[item] = rel_sign * (orig - lambd * pert);
}

// ---------------------------------------------------------------------------- CRIAGE
// x_k = E_h * R_r and w_k = sig'(E_e . x_k), one wave per tail triple
__global__ __launch_bounds__(256) void kp_criage_terms(int nk, const int32_t* __restrict__ tails,
                                                       const int32_t* __restrict__ tail_ent,
                                                       const float* __restrict__ E, const float* __restrict__ R,
                                                       int dp, int D, float* __restrict__ X, float* __restrict__ W) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= nk) return;
  const float* lh = E + (size_t)tails[2 * k] * dp;
  const float* rl = R + (size_t)tails[2 * k + 1] * dp;
  const float* ee = E + (size_t)tail_ent[k] * dp;
  float dot = 0.f;
  for (int j = lane; j < D; j += 64) {
    const float x = lh[j] * rl[j];
    X[(size_t)k * D + j] = x;
    dot += ee[j] * x;
  }
  dot = wsum(dot);
  if (lane == 0) {
    const float sg = 1.0f / (1.0f + expf(-dot));
    W[k] = sg * (1.0f - sg);
  }
}

// H_e[i][j] = sum_k (double)(w_k * (x_ki * x_kj)), k in triple order; grid (tiles, entities)
__global__ __launch_bounds__(256) void kp_criage_hessian(int D, const int32_t* __restrict__ off,
                                                         const float* __restrict__ X, const float* __restrict__ W,
                                                         double* __restrict__ H) {
  const int ent = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= D * D) return;
  const int i = idx / D, j = idx - (idx / D) * D;
  double acc = 0.0;
  for (int k = off[ent]; k < off[ent + 1]; ++k) {
    const float* x = X + (size_t)k * D;
    acc += (double)(W[k] * (x[i] * x[j]));
  }
  H[(size_t)ent * D * D + idx] = acc;
}

// ComplEx criage_first_step: q = [a c - b d, a d + b c] (complex.py:113-132)
__global__ __launch_bounds__(256) void kp_criage_zq(int n, const int2* __restrict__ src, const float* __restrict__ E,
                                                    const float* __restrict__ R, int dp, int rd,
                                                    float* __restrict__ Z) {
  const int i = blockIdx.x;
  if (i >= n) return;
  const float* l = E + (size_t)src[i].x * dp;
  const float* r = R + (size_t)src[i].y * dp;
  for (int j = threadIdx.x; j < rd; j += 256) {
    const float a = l[j], b = l[rd + j], c = r[j], d = r[rd + j];
    Z[(size_t)i * dp + j] = a * c - b * d;
    Z[(size_t)i * dp + rd + j] = a * d + b * c;
  }
}

// One workgroup per candidate: A = H_e + fl32(c * fl32(z_i z_j)), c = fl32(sig (1 - sig)),
// Gaussian elimination with partial pivoting on [A | z_t], back substitution,
// out = z_p . ((1 - sig) y).  items[i] = (z_pred row, z_triple row, entity slot, entity id).
__global__ __launch_bounds__(256) void kp_criage_solve(int D, int dp, const int32_t* __restrict__ items,
                                                       const float* __restrict__ Z, const float* __restrict__ E,
                                                       const double* __restrict__ H, double* __restrict__ Aws,
                                                       double* __restrict__ out, int32_t* __restrict__ status) {
  __shared__ double lcol[512], prow[512], bsh[512];
  __shared__ double rv[256];
  __shared__ int ri[256];
  __shared__ float sig_s;
  __shared__ int bad;
  const int tid = threadIdx.x;
  const int32_t* it = items + 4 * (size_t)blockIdx.x;
  const float* zp = Z + (size_t)it[0] * dp;
  const float* zt = Z + (size_t)it[1] * dp;
  const double* He = H + (size_t)it[2] * D * D;
  const float* ee = E + (size_t)it[3] * dp;
  double* A = Aws + (size_t)blockIdx.x * D * D;
  // sig = sigmoid(e . z_t) in float32
  float part = 0.f;
  for (int j = tid; j < D; j += 256) part += ee[j] * zt[j];
  part = wsum(part);
  __shared__ float red[4];
  if ((tid & 63) == 0) red[tid >> 6] = part;
  if (tid == 0) bad = 0;
  __syncthreads();
  if (tid == 0) {
    const float dot = (red[0] + red[1]) + (red[2] + red[3]);
    sig_s = 1.0f / (1.0f + expf(-dot));
  }
  __syncthreads();
  const float sig = sig_s;
  const float c = sig * (1.0f - sig);
  for (int i = tid >> 5; i < D; i += 8) {
    const float zi = zt[i];
    for (int j = tid & 31; j < D; j += 32) A[(size_t)i * D + j] = He[(size_t)i * D + j] + (double)(c * (zi * zt[j]));
  }
  for (int i = tid; i < D; i += 256) bsh[i] = (double)zt[i];
  __syncthreads();
  for (int k = 0; k < D; ++k) {
    // pivot: first row of maximal |A[i][k]|, i >= k (idamax)
    double best = -1.0;
    int bi = D;
    for (int i = k + tid; i < D; i += 256) {
      const double v = fabs(A[(size_t)i * D + k]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    rv[tid] = best;
    ri[tid] = bi;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) {
        const double a = rv[tid], b = rv[tid + s];
        const int ia = ri[tid], ib = ri[tid + s];
        if (b > a || (b == a && ib < ia)) {
          rv[tid] = b;
          ri[tid] = ib;
        }
      }
      __syncthreads();
    }
    const int piv = ri[0];
    if (rv[0] == 0.0) {  // exactly singular: LAPACK's getrf reports it, numpy.linalg.inv raises
      if (tid == 0) bad = 1;
      break;
    }
    if (piv != k) {
      for (int j = k + tid; j < D; j += 256) {
        const double a = A[(size_t)k * D + j];
        A[(size_t)k * D + j] = A[(size_t)piv * D + j];
        A[(size_t)piv * D + j] = a;
      }
      if (tid == 0) {
        const double b = bsh[k];
        bsh[k] = bsh[piv];
        bsh[piv] = b;
      }
    }
    __syncthreads();
    const double pv = A[(size_t)k * D + k];
    for (int i = k + 1 + tid; i < D; i += 256) {
      lcol[i] = A[(size_t)i * D + k] / pv;
      prow[i] = A[(size_t)k * D + i];
    }
    __syncthreads();
    // trailing update: 8 row groups x 32 consecutive columns (coalesced rows, no index division)
    for (int i = k + 1 + (tid >> 5); i < D; i += 8) {
      const double li = lcol[i];
      double* Ai = A + (size_t)i * D;
      for (int j = k + 1 + (tid & 31); j < D; j += 32) Ai[j] -= li * prow[j];
    }
    for (int i = k + 1 + tid; i < D; i += 256) bsh[i] -= lcol[i] * bsh[k];
    __syncthreads();
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) {
      out[blockIdx.x] = NAN;
      status[blockIdx.x] = 1;
    }
    return;
  }
  // back substitution, column-oriented: y_i = b_i / U_ii, then b_j -= U_ji y_i for j < i
  for (int i = D - 1; i >= 0; --i) {
    if (tid == 0) bsh[i] = bsh[i] / A[(size_t)i * D + i];
    __syncthreads();
    const double yi = bsh[i];
    for (int j = tid; j < i; j += 256) bsh[j] -= A[(size_t)j * D + i] * yi;
    __syncthreads();
  }
  const double om = (double)(1.0f - sig);
  double acc = 0.0;
  for (int j = tid; j < D; j += 256) acc += (double)zp[j] * (om * bsh[j]);
  rv[tid] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) rv[tid] += rv[tid + s];
    __syncthreads();
  }
  if (tid == 0) {
    out[blockIdx.x] = rv[0];
    status[blockIdx.x] = 0;
  }
}

}  // namespace

void dp_relevance(kp_ctx* c, int n, const int32_t* items, float eps, float lambd, int step_sign, int rel_sign,
                  float* out) {
  KP_REQUIRE(c->model == KP_MODEL_COMPLEX,
             "data poisoning: the reference scores with score_embeddings, which only ComplEx has");
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 7; ++k) {
      const int v = items[7 * i + k];
      const bool rel = (k == 1 || k == 5);
      KP_REQUIRE(v >= 0 && v < (rel ? c->n_rel2 : c->n_ent), "data poisoning: id out of range");
    }
  DevBuf bi, bo;
  int32_t* dI = upload(c, bi, items, (size_t)7 * n);
  float* dO = reinterpret_cast<float*>(bo.ensure(sizeof(float) * (size_t)n));
  hipLaunchKernelGGL(kp_dp_complex, dim3((n + 3) / 4), dim3(256), 0, c->stream, n, dI, c->dE, c->dR, c->dp,
                     c->dim / 2, eps, lambd, (float)step_sign, (float)rel_sign, dO);
  KP_HIP(hipGetLastError());
  KP_HIP(hipMemcpyAsync(out, dO, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  bi.release();
  bo.release();
}

void criage_relevance(kp_ctx* c, int n, const int32_t* items, int n_ents, const int32_t* ent_ids,
                      const int32_t* tails_off, const int32_t* tails, double* out, int32_t* status) {
  KP_REQUIRE(c->model == KP_MODEL_COMPLEX || c->model == KP_MODEL_CONVE, "Criage does not support this model.");
  const int D = c->dim;
  KP_REQUIRE(D <= 512, "CRIAGE: dimension > 512 not supported");
  KP_REQUIRE(tails_off[0] == 0, "CRIAGE: tails_off[0] must be 0");
  for (int e = 0; e < n_ents; ++e) {
    KP_REQUIRE(ent_ids[e] >= 0 && ent_ids[e] < c->n_ent, "CRIAGE: entity out of range");
    KP_REQUIRE(tails_off[e + 1] >= tails_off[e], "CRIAGE: bad tail offsets");
  }
  const int nk = tails_off[n_ents];
  for (int k = 0; k < nk; ++k)
    KP_REQUIRE(tails[2 * k] >= 0 && tails[2 * k] < c->n_ent && tails[2 * k + 1] >= 0 &&
                   tails[2 * k + 1] < c->n_rel2,
               "CRIAGE: tail triple out of range");
  // distinct (s, p) pairs whose criage_first_step is needed
  std::vector<int2> src;
  std::vector<int32_t> it4((size_t)4 * n);
  {
    std::vector<std::pair<long long, int>> seen;
    auto zrow = [&](int s, int p) {
      KP_REQUIRE(s >= 0 && s < c->n_ent && p >= 0 && p < c->n_rel2, "CRIAGE: (s, p) out of range");
      const long long key = (long long)s * c->n_rel2 + p;
      for (auto& kv : seen)
        if (kv.first == key) return kv.second;
      src.push_back(make_int2(s, p));
      seen.push_back({key, (int)src.size() - 1});
      return (int)src.size() - 1;
    };
    for (int i = 0; i < n; ++i) {
      const int32_t* q = items + 5 * (size_t)i;
      KP_REQUIRE(q[4] >= 0 && q[4] < n_ents, "CRIAGE: entity slot out of range");
      it4[4 * i] = zrow(q[0], q[1]);
      it4[4 * i + 1] = zrow(q[2], q[3]);
      it4[4 * i + 2] = q[4];
      it4[4 * i + 3] = ent_ids[q[4]];
    }
  }
  const int nz = (int)src.size();
  std::vector<int32_t> tail_ent(std::max(nk, 1));
  for (int e = 0; e < n_ents; ++e)
    for (int k = tails_off[e]; k < tails_off[e + 1]; ++k) tail_ent[k] = ent_ids[e];
  DevBuf bsrc, bz, bt, bte, bx, bw, boff, bh, bit, ba, bo, bs;
  int2* dSrc = upload(c, bsrc, src.data(), src.size());
  float* dZ = reinterpret_cast<float*>(bz.ensure(sizeof(float) * (size_t)nz * c->dp));
  if (c->model == KP_MODEL_COMPLEX) {
    hipLaunchKernelGGL(kp_criage_zq, dim3(nz), dim3(256), 0, c->stream, nz, dSrc, c->dE, c->dR, c->dp, D / 2, dZ);
    KP_HIP(hipGetLastError());
  } else {
    conve_encode_dev(c, nz, dSrc, dZ);
  }
  int32_t* dT = upload(c, bt, tails, (size_t)2 * std::max(nk, 1));
  int32_t* dTe = upload(c, bte, tail_ent.data(), tail_ent.size());
  float* dX = reinterpret_cast<float*>(bx.ensure(sizeof(float) * (size_t)std::max(nk, 1) * D));
  float* dW = reinterpret_cast<float*>(bw.ensure(sizeof(float) * (size_t)std::max(nk, 1)));
  if (nk > 0) {
    hipLaunchKernelGGL(kp_criage_terms, dim3((nk + 3) / 4), dim3(256), 0, c->stream, nk, dT, dTe, c->dE, c->dR, c->dp,
                       D, dX, dW);
    KP_HIP(hipGetLastError());
  }
  int32_t* dOff = upload(c, boff, tails_off, (size_t)n_ents + 1);
  double* dH = reinterpret_cast<double*>(bh.ensure(sizeof(double) * (size_t)n_ents * D * D));
  hipLaunchKernelGGL(kp_criage_hessian, dim3((D * D + 255) / 256, n_ents), dim3(256), 0, c->stream, D, dOff, dX, dW,
                     dH);
  KP_HIP(hipGetLastError());
  // candidates in chunks: one float64 D x D system per workgroup
  const int chunk = std::max(1, std::min(n, (int)(((size_t)512 << 20) / ((size_t)D * D * sizeof(double)))));
  double* dA = reinterpret_cast<double*>(ba.ensure(sizeof(double) * (size_t)chunk * D * D));
  for (int i0 = 0; i0 < n; i0 += chunk) {
    const int m = std::min(chunk, n - i0);
    int32_t* dIt = upload(c, bit, it4.data() + 4 * (size_t)i0, (size_t)4 * m);
    double* dO = reinterpret_cast<double*>(bo.ensure(sizeof(double) * (size_t)m));
    int32_t* dS = reinterpret_cast<int32_t*>(bs.ensure(sizeof(int32_t) * (size_t)m));
    hipLaunchKernelGGL(kp_criage_solve, dim3(m), dim3(256), 0, c->stream, D, c->dp, dIt, dZ, c->dE, dH, dA, dO, dS);
    KP_HIP(hipGetLastError());
    KP_HIP(hipMemcpyAsync(out + i0, dO, sizeof(double) * m, hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipMemcpyAsync(status + i0, dS, sizeof(int32_t) * m, hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
  }
  for (DevBuf* b : {&bsrc, &bz, &bt, &bte, &bx, &bw, &boff, &bh, &bit, &ba, &bo, &bs}) b->release();
}
