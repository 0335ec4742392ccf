// kp_complex.hip -- ComplEx batched post-training (KelpieComplEx +
// KelpieMultiClassNLLOptimizer) and ranking, for gfx950.
//
// Reference semantics (src/link_prediction/models/complex.py:59-112,144-159,
// src/link_prediction/optimization/multiclass_nll_optimizer.py:57-164):
//   rows   = kelpie triples + inverses; per epoch torch.randperm; minibatches of
//            min(batch_size, R) rows stepping by batch_size;
//   loss   = CrossEntropy(q_i . E_all^T, t_i) (mean) + N3;  E_all = [E ; x]
//   step   = Adagrad / Adam / SGD on the single kelpie row x.
//
// Decomposition used here (ComplEx), per minibatch of b rows:
//   * rows whose head is the kelpie ("queries"): q = x o r changes every step.
//     Rows sharing a relation share q and the softmax, so they are merged
//     into one query with count c, kelpie-target count ck and frozen-target
//     sum Tsum.  Each query needs, over the FROZEN entities, the softmax
//     statistics (m, l) and O = sum_e exp(s_e - m) E_e -> kp_cx_attn, a
//     flash-attention-shaped pass with K = V = E on fp32 MFMA.
//   * rows whose head is frozen ("tails"; their target is always the kelpie):
//     q is fixed, so the frozen log-sum-exp is computed once per batch
//     (kp_cx_attn in pair mode) and each step only needs q . x.
//   * the kelpie column (entity |E|) is merged analytically in kp_cx_update,
//     which assembles the single-row gradient and applies the optimizer.
//   When R <= batch_size (one step per epoch) the permutation only reorders
//   the batch, so every epoch reuses one plan; otherwise each (epoch, step)
//   gets its own plan from the permutation.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <unordered_map>

#include "kp_attn.hpp"
#include "kp_attn3.hpp"

namespace {
using namespace kpattn;

struct CxPlan {
  int b, q_begin, q_count, t_begin, t_count, cnt_l, cnt_r, pad;
};
struct CxQuery {
  int rel, c, ck, tg_begin, tg_count, pad0, pad1, pad2;
};
struct CxTail {
  int pair, c;
};


// qpair[p] = E[h] o R[r] for the frozen-head rows
__global__ void kp_cx_qpair(const float* __restrict__ E, const float* __restrict__ R, int dp, int half,
                            const int2* __restrict__ pairs, int n_pairs, float* __restrict__ out) {
  int p = blockIdx.x;
  if (p >= n_pairs) return;
  int2 hr = pairs[p];
  const float* lhs = E + (size_t)hr.x * dp;
  const float* rel = R + (size_t)hr.y * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) out[(size_t)p * dp + d] = cx_q(lhs, rel, d, half);
}

// lsef[p] = the frozen-head pair's log-sum-exp over the frozen entities, merged from the
// attention's split statistics (one thread per pair; fp64 sum of the rescaled l's)
__global__ void kp_cx_lse_merge(int npairs, int n_split, const float* __restrict__ am, const float* __restrict__ al,
                                float* __restrict__ lsef) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  float mm = kNegInf;
  for (int s = 0; s < n_split; ++s) mm = fmaxf(mm, am[(size_t)s * npairs + p]);
  double ll = 0.0;
  for (int s = 0; s < n_split; ++s) {
    const float ms = am[(size_t)s * npairs + p];
    if (ms != kNegInf) ll += (double)al[(size_t)s * npairs + p] * exp((double)ms - (double)mm);
  }
  lsef[p] = (float)((double)mm + log(ll));
}

// Tsum[q] = sum of frozen target rows of a plan query
__global__ void kp_cx_tsum(const float* __restrict__ E, int dp, const CxQuery* __restrict__ pq, int nq,
                           const int32_t* __restrict__ targets, float* __restrict__ tsum) {
  int q = blockIdx.x;
  if (q >= nq) return;
  CxQuery Q = pq[q];
  for (int d = threadIdx.x; d < dp; d += blockDim.x) {
    float acc = 0.f;
    for (int i = 0; i < Q.tg_count; ++i) acc += E[(size_t)targets[Q.tg_begin + i] * dp + d];
    tsum[(size_t)q * dp + d] = acc;
  }
}

// ----------------------------------------------------------------------------
// kp_cx_update: one workgroup per active slot at this step.  Assembles the
// single-row gradient of the minibatch loss and applies the
// optimizer with torch's op order (optim/adagrad.py, optim/adam.py).
// ----------------------------------------------------------------------------
struct CxOpt {
  int kind;
  float lr, b1, b2, eps;
  float one_minus_b1, one_minus_b2;
  float step_size;  // Adam: lr / (1 - b1^t)
  float bc2_sqrt;   // Adam: sqrt(1 - b2^t)
  float reg_w;
  int reg_n2;  // KP_REG_N2: N2 on the whole row's L2 norm (regularizers.py:25-35) instead of N3
};

#define UPD_MAXSPLIT 16

// One wave per (query or frozen-head row) of this step: its contribution to the
// kelpie row's gradient (un-normalised by the batch size).
//   query (kelpie-head rows sharing relation r, count c, kelpie targets ck):
//     J_r^T (c <E> - Tsum - ck x) + (c p_k - ck) q,   <E> = softmax-weighted entity
//     (frozen part sum_sp w_sp O_sp merged with the kelpie column p_k x)
//   frozen-head row pair (count c, target = kelpie):  c (p_k - 1) q_pair
template <int DP>
__global__ __launch_bounds__(256) void kp_cx_contrib(int half, const int4* __restrict__ stepq, int nq,
                                                     const int4* __restrict__ stept, int nt,
                                                     const CxQuery* __restrict__ pq, const float* __restrict__ X,
                                                     const float* __restrict__ R, const float* __restrict__ Tsum,
                                                     const float* __restrict__ Qpair, const float* __restrict__ lsef,
                                                     const float* __restrict__ att_m, const float* __restrict__ att_l,
                                                     const float* __restrict__ att_O, int n_split,
                                                     float* __restrict__ contrib) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= nq + nt) return;
  float* out = contrib + (size_t)item * DP;
  if (item < nq) {
    const int4 sq = stepq[item];  // slot, rel, plan-query index
    const float* x = X + (size_t)sq.x * DP;
    const float* rel = R + (size_t)sq.y * DP;
    const CxQuery Q = pq[sq.z];
    float z = 0.f;
    for (int d = lane; d < 2 * half; d += 64) z += cx_q(x, rel, d, half) * x[d];
    z = wave_sum(z);
    // The softmax normalisation in fp64 with correctly rounded exp / log.  <E> below is
    // ~5e-4 per coordinate at the reference init and the row contributions cancel to a
    // gradient up to ~100x smaller on the coordinates Adagrad has not saturated, so a
    // one-sided ulp error of a fast exp / log here (every row, every step, the same
    // sign) became a one-sided drift of those coordinates of the kelpie row (measured
    // ~-4e-6 against the fp64 reference, tools/headline_probe.py).
    // The split statistics one split per lane (n_split <= 64): the max, the fp64 sum of
    // the rescaled l's (a butterfly, deterministic) and each split's weight, so a wave
    // makes two fp64 exp per lane instead of 2 n_split in sequence on every lane.
    const bool has = lane < n_split;
    const float ms_l = has ? att_m[(size_t)lane * nq + item] : kNegInf;
    const float ls_l = has ? att_l[(size_t)lane * nq + item] : 0.f;
    const float mm = wave_max(ms_l);
    double e_l = (ms_l == kNegInf) ? 0.0 : (double)ls_l * exp((double)ms_l - (double)mm);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) e_l += __shfl_xor(e_l, o, 64);
    const double lse_f = (double)mm + log(e_l);
    const double hi = fmax(lse_f, (double)z), lo = fmin(lse_f, (double)z);
    const double lse = hi + log1p(exp(lo - hi));
    const double pk = exp((double)z - lse);
    const double wv_l = (ms_l == kNegInf) ? 0.0 : exp((double)ms_l - lse);
    // merge the partials split by split (increasing split order), one split at a time:
    // 64 registers, so that a wave fits beside a resident kp_attn3 wave on its SIMD (that
    // one leaves 104 of the 512 registers per lane free; with two splits' loads in flight
    // this kernel took 94 and still fitted, the round-4 forms with 150 did not and ran
    // only on the CUs no attention workgroup held: 92 -> 192 us per launch under overlap)
    constexpr int NI = (DP / 2 + 63) / 64;
    double ore_k[NI], oim_k[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) ore_k[k] = oim_k[k] = 0.0;
    for (int sp = 0; sp < n_split; ++sp) {
      const double w0 = __shfl(wv_l, sp, 64);
      const float* O0 = att_O + ((size_t)sp * nq + item) * DP;
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        const int i = lane + 64 * k;
        const bool in = i < half;
        const float a0 = in ? O0[i] : 0.f, b0 = in ? O0[i + half] : 0.f;
        ore_k[k] += w0 * (double)a0;
        oim_k[k] += w0 * (double)b0;
      }
    }
    const double fc = (double)Q.c, fck = (double)Q.ck;
    const double cf = fc * pk - fck;
    const float* ts = Tsum + (size_t)sq.z * DP;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = lane + 64 * k;
      if (i >= half) continue;
      const double a = x[i], b = x[i + half];
      const double cc = rel[i], ee = rel[i + half];
      const double ere = ore_k[k] + pk * a, eim = oim_k[k] + pk * b;
      const double dre = fc * ere - (double)ts[i] - fck * a;
      const double dim_ = fc * eim - (double)ts[i + half] - fck * b;
      const double qre = a * cc - b * ee, qim = a * ee + b * cc;
      out[i] = (float)(dre * cc + dim_ * ee + cf * qre);
      out[i + half] = (float)(-dre * ee + dim_ * cc + cf * qim);
    }
  } else {
    const int4 st = stept[item - nq];  // slot, pair, count
    const float* x = X + (size_t)st.x * DP;
    const float* qp = Qpair + (size_t)st.y * DP;
    float z = 0.f;
    for (int d = lane; d < 2 * half; d += 64) z += qp[d] * x[d];
    z = wave_sum(z);
    const double lf = lsef[st.y];
    const double hi = fmax(lf, (double)z), lo = fmin(lf, (double)z);
    const double lse = hi + log1p(exp(lo - hi));
    const double coef = (double)st.z * (exp((double)z - lse) - 1.0);
    for (int d = lane; d < 2 * half; d += 64) out[d] = (float)(coef * (double)qp[d]);
  }
}

#ifndef KP_CX_UPD64
#define KP_CX_UPD64 0
#endif
// Sum a slot's contributions, add the N3 term, apply the optimizer (torch op order).
template <int DP>
__global__ __launch_bounds__(256) void kp_cx_update(int half, const int4* __restrict__ act,
                                                    const CxPlan* __restrict__ plans, int nq,
                                                    const float* __restrict__ contrib, float* __restrict__ X,
                                                    float* __restrict__ S1, float* __restrict__ S2, CxOpt opt) {
  const int tid = threadIdx.x;
  const int4 a4 = act[blockIdx.x];  // slot, plan, qoff, toff
  const int slot = a4.x;
  const CxPlan P = plans[a4.y];
  float* x = X + (size_t)slot * DP;
  const float inv_b = 1.0f / (float)P.b;
  // contribution rows: the slot's queries, then its frozen-head rows
  const int nc = P.q_count + P.t_count;
  auto crow = [&](int j) -> const float* {
    return j < P.q_count ? contrib + (size_t)(a4.z + j) * DP : contrib + (size_t)(nq + a4.w + j - P.q_count) * DP;
  };
  // The rows sum in four wave-strided partials with four chains each, so 16 rows'
  // loads are in flight at once (one sequential chain per dimension was bound by the
  // load latency: ~90 us per step at FB15k-237 sizes); a slot with at most UPD_WIDE
  // rows keeps the sequential chain (the choice is block-uniform).
  constexpr int UPD_WIDE = 4;
#if KP_CX_UPD64
  // the slot's gradient assembled in fp64 (row sums, 1/B, regulariser term) and rounded
  // once to fp32 before the optimizer; the four wave partials meet in two rounds through
  // 2 x DP doubles, the LDS of the fp32 form (6.4 KiB at D = 400: it still fits beside a
  // resident kp_attn3<25> workgroup)
  typedef double acc_t;
  __shared__ double red[2][DP];
  if (nc > UPD_WIDE) {
    const int w = tid >> 6, lane = tid & 63;
    double part[(DP + 63) / 64];
#pragma unroll
    for (int k = 0; k < (DP + 63) / 64; ++k) {
      const int d = lane + 64 * k;
      part[k] = 0.0;
      if (d >= 2 * half) continue;
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      int j = w;
      for (; j + 12 < nc; j += 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += crow(j + 4 * q)[d];
      }
      if (j < nc) acc[0] += crow(j)[d];  // at most three rows are left
      if (j + 4 < nc) acc[1] += crow(j + 4)[d];
      if (j + 8 < nc) acc[2] += crow(j + 8)[d];
      part[k] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      if (w >= 2) red[w - 2][d] = part[k];
    }
    __syncthreads();
    if (w < 2)
#pragma unroll
      for (int k = 0; k < (DP + 63) / 64; ++k) {
        const int d = lane + 64 * k;
        if (d < 2 * half) red[w][d] = part[k] + red[w][d];
      }
    __syncthreads();
  }
#else
  typedef float acc_t;
  __shared__ float red[4][DP];
  if (nc > UPD_WIDE) {
    const int w = tid >> 6, lane = tid & 63;
    for (int d = lane; d < 2 * half; d += 64) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      int j = w;
      for (; j + 12 < nc; j += 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += crow(j + 4 * k)[d];
      }
      if (j < nc) acc[0] += crow(j)[d];  // at most three rows are left
      if (j + 4 < nc) acc[1] += crow(j + 4)[d];
      if (j + 8 < nc) acc[2] += crow(j + 8)[d];
      red[w][d] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    __syncthreads();
  }
#endif
  // N2 (regularizers.py:25-35): the factor of each batch row holding the kelpie entity
  // is ||f||^3 with f_i = |x_i| (complex modulus, complex.py:80-84), so its gradient is
  // 3 w / B * ||f|| * x per such row; ||f|| over the whole row, before the update
  float n2 = 0.f;
  if (opt.reg_w != 0.f && opt.reg_n2) {
    __shared__ float n2red[4];
    float ps = 0.f;
    for (int i = tid; i < half; i += 256) {
      const float a = x[i], b = x[i + half];
      const float f = sqrtf(a * a + b * b);
      ps += f * f;
    }
    ps = wave_sum(ps);
    if ((tid & 63) == 0) n2red[tid >> 6] = ps;
    __syncthreads();
    n2 = sqrtf((n2red[0] + n2red[1]) + (n2red[2] + n2red[3]));
  }
#pragma unroll
  for (int u = 0; u < (DP / 2 + 255) / 256; ++u) {
    const int i = tid + 256 * u;
    if (i >= half) continue;
    acc_t gv[2] = {0.f, 0.f};
    if (nc > UPD_WIDE) {
#if KP_CX_UPD64
      gv[0] = red[0][i] + red[1][i];
      gv[1] = red[0][i + half] + red[1][i + half];
#else
      gv[0] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
      gv[1] = (red[0][i + half] + red[1][i + half]) + (red[2][i + half] + red[3][i + half]);
#endif
    } else {
      for (int j = 0; j < nc; ++j) {
        const float* c = crow(j);
        gv[0] += c[i];
        gv[1] += c[i + half];
      }
    }
#if KP_CX_UPD64
    gv[0] /= (double)P.b;
    gv[1] /= (double)P.b;
#else
    gv[0] *= inv_b;
    gv[1] *= inv_b;
#endif
    const float a = x[i], b = x[i + half];
    if (opt.reg_w != 0.f) {
#if KP_CX_UPD64
      const double mod = opt.reg_n2 ? (double)n2 : sqrt((double)a * a + (double)b * b);
      const double k3 = 3.0 * (double)opt.reg_w / (double)P.b * (double)(P.cnt_l + P.cnt_r) * mod;
#else
      const float mod = opt.reg_n2 ? n2 : sqrtf(a * a + b * b);
      const float k3 = 3.0f * opt.reg_w * inv_b * (float)(P.cnt_l + P.cnt_r) * mod;
#endif
      gv[0] += k3 * a;
      gv[1] += k3 * b;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int d = i + h * half;
      const float gd = (float)gv[h];
      float xd = h ? b : a;
      const size_t o = (size_t)slot * DP + d;
      if (opt.kind == KP_OPT_ADAGRAD) {
        float s1 = S1[o];
        s1 = s1 + gd * gd;
        const float stdv = sqrtf(s1) + opt.eps;
        xd = xd + (-opt.lr * gd) / stdv;
        S1[o] = s1;
      } else if (opt.kind == KP_OPT_ADAM) {
        float m1 = S1[o], v2 = S2[o];
        m1 = m1 + opt.one_minus_b1 * (gd - m1);
        v2 = v2 * opt.b2;
        v2 = v2 + (opt.one_minus_b2 * gd) * gd;
        const float den = sqrtf(v2) / opt.bc2_sqrt + opt.eps;
        xd = xd + (-opt.step_size * m1) / den;
        S1[o] = m1;
        S2[o] = v2;
      } else {
        xd = xd + (-opt.lr) * gd;
      }
      x[d] = xd;
    }
  }
}

// fp64 ranking queries (launch_rank_f64): q_s = x_s o R[p_s] from exact fp64 products of
// the fp32 operands; the target score q_s . E_o and the kelpie column q_s . x_s as one
// sequential fp64 FMA chain over d (the order kp_rank_f64_count scores every entity in)
__device__ __forceinline__ double cx_q64(const float* __restrict__ lhs, const float* __restrict__ rel, int d,
                                         int half) {
  if (d < half) return (double)lhs[d] * (double)rel[d] - (double)lhs[d + half] * (double)rel[d + half];
  if (d < 2 * half) {
    const int i = d - half;
    return (double)lhs[i] * (double)rel[d] + (double)lhs[d] * (double)rel[i];
  }
  return 0.0;
}

template <int DP>
__global__ void kp_cx_rankq64(const float* __restrict__ X, const float* __restrict__ R, const float* __restrict__ E,
                              int n_ent, int half, const int32_t* __restrict__ pred, int n_slots,
                              double* __restrict__ Q, double* __restrict__ t64, double* __restrict__ kcol64) {
  const int s = blockIdx.x;
  if (s >= n_slots) return;
  const float* x = X + (size_t)s * DP;
  const float* rel = R + (size_t)pred[3 * s + 1] * DP;
  double* q = Q + (size_t)s * DP;
  for (int d = threadIdx.x; d < DP; d += blockDim.x) q[d] = cx_q64(x, rel, d, half);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int o = pred[3 * s + 2];
    double z = 0.0, t = 0.0;
    for (int d = 0; d < DP; ++d) z = __fma_rn(q[d], (double)x[d], z);
    if (o < n_ent) {
      const float* eo = E + (size_t)o * DP;
      for (int d = 0; d < DP; ++d) t = __fma_rn(q[d], (double)eo[d], t);
    } else {
      t = z;  // the kelpie entity is its own object
    }
    kcol64[s] = z;
    t64[s] = t;
  }
}

__global__ void kp_cx_scoreq(const float* __restrict__ E, const float* __restrict__ R, int dp, int half,
                             const int32_t* __restrict__ heads, const int32_t* __restrict__ rels, int n,
                             float* __restrict__ Q) {
  int s = blockIdx.x;
  if (s >= n) return;
  const float* lhs = E + (size_t)heads[s] * dp;
  const float* rel = R + (size_t)rels[s] * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) Q[(size_t)s * dp + d] = cx_q(lhs, rel, d, half);
}

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
// step queries q_j = x_slot o R_rel (complex.py:65-72), one row per step query
template <int DP>
__global__ void kp_cx_stepq(const float* __restrict__ X, const float* __restrict__ R, int half,
                            const int4* __restrict__ stepq, int nq, float* __restrict__ Q) {
  const int j = blockIdx.x;
  if (j >= nq) return;
  const int4 sq = stepq[j];
  const float* x = X + (size_t)sq.x * DP;
  const float* rel = R + (size_t)sq.y * DP;
  for (int d = threadIdx.x; d < DP; d += blockDim.x) Q[(size_t)j * DP + d] = cx_q(x, rel, d, half);
}

template <int DB>
void launch_stepq(kp_ctx* c, const int4* stepq, const float* X, int nq, float* Q) {
  if (nq <= 0) return;
  hipLaunchKernelGGL((kp_cx_stepq<16 * DB>), dim3(nq), dim3(64), 0, c->stream, X, c->dR, c->dim / 2, stepq, nq, Q);
  KP_HIP(hipGetLastError());
}

// co-resident attention workgroups: LDS and registers allow two per CU for rows up
// to 208 floats, one for wider rows
// (kp_attn3: as many as the occupancy API reports)
template <int DB>
int attn_slots_db(kp_ctx* c) {
  if (c->attn_mode == 1) return c->n_cu * attn3_wpc<DB>(c);
  return c->n_cu * (DB <= 13 ? 2 : 1);
}

template <int DB>
void launch_attn(kp_ctx* c, bool with_o, const float* Q, int nq, const AttnPlan& plan, float* m, float* l,
                 float* O) {
  if (nq <= 0) return;
  if (c->attn_mode == 1) {
    if (with_o)
      launch_attn3<DB, ATT_SOFTMAX_O>(c, c->n_ent, Q, nq, plan, m, l, O, nullptr, 0.f);
    else
      launch_attn3<DB, ATT_SOFTMAX>(c, c->n_ent, Q, nq, plan, m, l, O, nullptr, 0.f);
    return;
  }
  const size_t shm = attn_lds_bytes(DB);
  if (with_o)
    hipLaunchKernelGGL((kp_attn<DB, ATT_SOFTMAX_O>), dim3(plan.n_wg), dim3(256), shm, c->stream, c->dE, c->n_ent, Q,
                       nq, plan.wk, m, l, O, nullptr, 0.f);
  else
    hipLaunchKernelGGL((kp_attn<DB, ATT_SOFTMAX>), dim3(plan.n_wg), dim3(256), shm, c->stream, c->dE, c->n_ent, Q,
                       nq, plan.wk, m, l, O, nullptr, 0.f);
  KP_HIP(hipGetLastError());
}

template <int DB>
void launch_update(kp_ctx* c, int n_act, const int4* act, const CxPlan* plans, const CxQuery* pq,
                   const int4* stepq, int nq, const int4* stept, int nt, const float* tsum, const float* qpair,
                   const float* lsef, const float* am, const float* al, const float* aO, int n_split, float* contrib,
                   float* X, float* S1, float* S2, const CxOpt& opt) {
  if (n_act <= 0) return;
  const int half = c->dim / 2;
  KP_REQUIRE(n_split >= 1 && n_split <= 64, "cx contrib: one attention split per lane");
  if (nq + nt > 0) {
    hipLaunchKernelGGL((kp_cx_contrib<16 * DB>), dim3((nq + nt + 3) / 4), dim3(256), 0, c->stream, half, stepq, nq,
                       stept, nt, pq, X, c->dR, tsum, qpair, lsef, am, al, aO, n_split, contrib);
    KP_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL((kp_cx_update<16 * DB>), dim3(n_act), dim3(256), 0, c->stream, half, act, plans, nq, contrib, X,
                     S1, S2, opt);
  KP_HIP(hipGetLastError());
}

template <int DB>
void launch_rankq64(kp_ctx* c, const float* X, const int32_t* pred, int n, double* Q, double* t64, double* kcol64) {
  if (n <= 0) return;
  hipLaunchKernelGGL((kp_cx_rankq64<16 * DB>), dim3(n), dim3(64), 0, c->stream, X, c->dR, c->dE, c->n_ent,
                     c->dim / 2, pred, n, Q, t64, kcol64);
  KP_HIP(hipGetLastError());
}

#define CX_DISPATCH(DBV, ...)   \
  switch (DBV) {                 \
    case 1: { constexpr int DB = 1; __VA_ARGS__; } break;   \
    case 2: { constexpr int DB = 2; __VA_ARGS__; } break;   \
    case 4: { constexpr int DB = 4; __VA_ARGS__; } break;   \
    case 8: { constexpr int DB = 8; __VA_ARGS__; } break;   \
    case 13: { constexpr int DB = 13; __VA_ARGS__; } break; \
    case 16: { constexpr int DB = 16; __VA_ARGS__; } break; \
    case 25: { constexpr int DB = 25; __VA_ARGS__; } break; \
    default: throw KpError{KP_ENOTSUP, "ComplEx: unsupported padded dimension"}; \
  }

}  // namespace

int cx_pick_db(int dim) {
  static const int dbs[] = {1, 2, 4, 8, 13, 16, 25};
  for (int db : dbs)
    if (16 * db >= dim) return db;
  return -1;
}

// KP_HOST_TIMES=1 (diagnostic): per call, on stderr, the host time before the first upload
// (checks and planning), up to the last launch enqueued, and waiting for the device
static const bool g_host_times = std::getenv("KP_HOST_TIMES") != nullptr;
static double host_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void complex_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* bt) {
  const double t_in = g_host_times ? host_ms() : 0.0;
  const int DBV = c->dp / 16;
  const int K = c->n_ent;  // kelpie id
  const int ns = bt->n_slots;
  const int hpbs = hp->batch_size;
  KP_REQUIRE(hpbs > 0 && hp->epochs >= 0, "ComplEx: bad batch_size/epochs");
  const int E = hp->epochs;
  // every id is checked before it indexes a host vector or a device table (as ConvE / TransE)
  KP_REQUIRE(ns >= 0 && bt->row_off[0] == 0, "ComplEx: bad row_off");
  for (int s = 0; s < ns; ++s) {
    KP_REQUIRE(bt->row_off[s + 1] >= bt->row_off[s], "ComplEx: bad row_off");
    KP_REQUIRE(bt->pred[3 * s] == K, "ComplEx: the ranked triple must start at the kelpie entity");
    KP_REQUIRE(bt->pred[3 * s + 1] >= 0 && bt->pred[3 * s + 1] < c->n_rel2, "ComplEx: ranked relation out of range");
    KP_REQUIRE(bt->pred[3 * s + 2] >= 0 && bt->pred[3 * s + 2] <= K, "ComplEx: ranked object out of range");
    KP_REQUIRE(bt->filt_off[s + 1] >= bt->filt_off[s], "ComplEx: bad filt_off");
  }
  for (int64_t i = 0; i < (int64_t)bt->row_off[ns]; ++i) {
    const int32_t* rw = bt->rows + 3 * i;
    KP_REQUIRE(rw[0] >= 0 && rw[0] <= K && rw[2] >= 0 && rw[2] <= K && rw[1] >= 0 && rw[1] < c->n_rel2,
               "ComplEx: row id out of range");
  }
  for (int64_t i = 0; i < (int64_t)bt->filt_off[ns]; ++i)
    KP_REQUIRE(bt->filt[i] >= 0 && bt->filt[i] <= K, "ComplEx: filter id out of range");

  std::vector<CxPlan> plans;
  std::vector<CxQuery> pqs;
  std::vector<CxTail> pts;
  std::vector<int32_t> targets;
  std::vector<int2> pairs;
  std::unordered_map<int64_t, int> pair_id;
  std::vector<int> plan_base(ns, 0), nsteps(ns, 0);

  std::vector<int> rel_slot(c->n_rel2, -1);
  std::vector<int> rel_cnt, rel_ck, rel_first;
  std::unordered_map<int, int> tail_slot;
  auto make_plan = [&](const int32_t* rows, const int32_t* idx, int n) {
    CxPlan P{};
    P.b = n;
    P.q_begin = (int)pqs.size();
    P.t_begin = (int)pts.size();
    std::vector<int> rels;
    tail_slot.clear();
    // pass 1: group
    std::vector<int> qtg_count;
    for (int k = 0; k < n; ++k) {
      const int32_t* rw = rows + 3 * (size_t)(idx ? idx[k] : k);
      const int h = rw[0], r = rw[1], t = rw[2];
      if (h == K) {
        if (rel_slot[r] < 0) {
          rel_slot[r] = (int)rels.size();
          rels.push_back(r);
          qtg_count.push_back(0);
          pqs.push_back(CxQuery{r, 0, 0, 0, 0, 0, 0, 0});
        }
        CxQuery& Q = pqs[P.q_begin + rel_slot[r]];
        Q.c += 1;
        P.cnt_l += 1;
        if (t == K) {
          Q.ck += 1;
          P.cnt_r += 1;
        } else {
          qtg_count[rel_slot[r]] += 1;
        }
      } else {
        KP_REQUIRE(t == K, "ComplEx: a training row does not involve the kelpie entity");
        P.cnt_r += 1;
        const int64_t key = (int64_t)h * c->n_rel2 + r;
        auto it = pair_id.find(key);
        int pid;
        if (it == pair_id.end()) {
          pid = (int)pairs.size();
          pair_id.emplace(key, pid);
          pairs.push_back(make_int2(h, r));
        } else {
          pid = it->second;
        }
        auto jt = tail_slot.find(pid);
        if (jt == tail_slot.end()) {
          tail_slot.emplace(pid, (int)pts.size());
          pts.push_back(CxTail{pid, 1});
        } else {
          pts[jt->second].c += 1;
        }
      }
    }
    // pass 2: frozen targets grouped per query
    int base = (int)targets.size();
    for (size_t j = 0; j < rels.size(); ++j) {
      pqs[P.q_begin + j].tg_begin = base;
      pqs[P.q_begin + j].tg_count = 0;
      base += qtg_count[j];
    }
    targets.resize(base);
    for (int k = 0; k < n; ++k) {
      const int32_t* rw = rows + 3 * (size_t)(idx ? idx[k] : k);
      if (rw[0] == K && rw[2] != K) {
        CxQuery& Q = pqs[P.q_begin + rel_slot[rw[1]]];
        targets[Q.tg_begin + Q.tg_count++] = rw[2];
      }
    }
    for (int r : rels) rel_slot[r] = -1;
    P.q_count = (int)rels.size();
    P.t_count = (int)pts.size() - P.t_begin;
    plans.push_back(P);
  };

  int T = 0;
  for (int s = 0; s < ns; ++s) {
    const int r0 = bt->row_off[s], r1 = bt->row_off[s + 1];
    const int R = r1 - r0;
    KP_REQUIRE(R >= 0, "ComplEx: bad row_off");
    const int32_t* rows = bt->rows + 3 * (size_t)r0;
    plan_base[s] = (int)plans.size();
    if (R == 0 || E == 0) {
      nsteps[s] = 0;
      continue;
    }
    const int nst = (R + hpbs - 1) / hpbs;
    const int bs = std::min(hpbs, R);
    nsteps[s] = nst;
    if (nst == 1) {
      make_plan(rows, nullptr, R);
    } else {
      const int64_t g0 = bt->rng_off[s], g1 = bt->rng_off[s + 1];
      KP_REQUIRE(g1 - g0 >= (int64_t)E * R, "ComplEx: missing randperm draws for a multi-step slot");
      for (int e = 0; e < E; ++e) {
        const int32_t* perm = bt->rng + g0 + (int64_t)e * R;
        for (int j = 0; j < R; ++j) KP_REQUIRE(perm[j] >= 0 && perm[j] < R, "ComplEx: randperm value out of range");
        for (int j = 0; j < nst; ++j) {
          const int st = j * hpbs;
          const int n = std::min(bs, R - st);
          make_plan(rows, perm + st, n);
        }
      }
    }
    T = std::max(T, E * nst);
  }

  // per-step active lists
  std::vector<int> act_off(T + 1, 0), q_off(T + 1, 0), t_off(T + 1, 0);
  std::vector<int4> acts;
  std::vector<int4> stepq, stept;
  int max_nq = 0, max_items = 0;
  for (int t = 0; t < T; ++t) {
    act_off[t] = (int)acts.size();
    q_off[t] = (int)stepq.size();
    t_off[t] = (int)stept.size();
    int qo = 0, to = 0;
    for (int s = 0; s < ns; ++s) {
      const int nst = nsteps[s];
      if (nst == 0 || t >= E * nst) continue;
      const int plan = plan_base[s] + (nst == 1 ? 0 : t);
      acts.push_back(make_int4(s, plan, qo, to));
      const CxPlan& P = plans[plan];
      for (int j = 0; j < P.q_count; ++j)
        stepq.push_back(make_int4(s, pqs[P.q_begin + j].rel, P.q_begin + j, 0));
      for (int j = 0; j < P.t_count; ++j) stept.push_back(make_int4(s, pts[P.t_begin + j].pair, pts[P.t_begin + j].c, 0));
      qo += P.q_count;
      to += P.t_count;
    }
    max_nq = std::max(max_nq, qo);
    max_items = std::max(max_items, qo + to);
  }
  act_off[T] = (int)acts.size();
  q_off[T] = (int)stepq.size();
  t_off[T] = (int)stept.size();

  const int DP = c->dp;
  const double t_plan = g_host_times ? host_ms() : 0.0;
  // ---- uploads
  float* dX = nullptr;
  {
    std::vector<float> xp((size_t)ns * DP, 0.f);
    for (int s = 0; s < ns; ++s)
      std::memcpy(&xp[(size_t)s * DP], bt->x0 + (size_t)s * c->dim, sizeof(float) * c->dim);
    dX = upload(c, c->ws[0], xp.data(), xp.size());
  }
  float* dS1 = reinterpret_cast<float*>(c->ws[1].ensure(sizeof(float) * (size_t)ns * DP));
  float* dS2 = reinterpret_cast<float*>(c->ws[2].ensure(sizeof(float) * (size_t)ns * DP));
  KP_HIP(hipMemsetAsync(dS1, 0, sizeof(float) * (size_t)ns * DP, c->stream));
  KP_HIP(hipMemsetAsync(dS2, 0, sizeof(float) * (size_t)ns * DP, c->stream));
  CxPlan* dPlans = upload(c, c->ws[3], plans.data(), plans.size());
  CxQuery* dPq = upload(c, c->ws[4], pqs.data(), pqs.size());
  int32_t* dTg = upload(c, c->ws[6], targets.data(), targets.size());
  int2* dPairs = upload(c, c->ws[7], pairs.data(), pairs.size());
  int4* dActs = upload(c, c->ws[8], acts.data(), acts.size());
  int4* dStepQ = upload(c, c->ws[9], stepq.data(), std::max<size_t>(1, stepq.size()));
  DevBuf& bStepT = c->ws[24];
  int4* dStepT = upload(c, bStepT, stept.data(), std::max<size_t>(1, stept.size()));
  float* dContrib = reinterpret_cast<float*>(c->ws[25].ensure(sizeof(float) * (size_t)std::max(1, max_items) * DP));
  const int npq = (int)pqs.size(), npairs = (int)pairs.size();
  float* dTsum = reinterpret_cast<float*>(c->ws[10].ensure(sizeof(float) * (size_t)std::max(npq, 1) * DP));
  float* dQpair = reinterpret_cast<float*>(c->ws[11].ensure(sizeof(float) * (size_t)std::max(npairs, 1) * DP));
  float* dLsef = reinterpret_cast<float*>(c->ws[12].ensure(sizeof(float) * (size_t)std::max(npairs, 1)));

  // the ranking's inputs and buffers now, ahead of the step loop: an upload from pageable
  // memory after the loop waited for the whole loop on the device, so the rank kernels
  // were enqueued only then (a host round trip per batch with the context idle)
  double* dQ64 = reinterpret_cast<double*>(c->ws[29].ensure(sizeof(double) * (size_t)ns * DP));
  double* dT64 = reinterpret_cast<double*>(c->ws[30].ensure(sizeof(double) * 2 * (size_t)ns));
  int32_t* dPred = upload(c, c->ws[18], bt->pred, (size_t)ns * 3);
  std::vector<int32_t> po(ns);
  for (int s = 0; s < ns; ++s) po[s] = bt->pred[3 * s + 2];
  int32_t* dPo = upload(c, c->ws[19], po.data(), po.size());
  int32_t* dFo = upload(c, c->ws[20], bt->filt_off, (size_t)ns + 1);
  int32_t* dF = upload(c, c->ws[21], bt->filt, (size_t)bt->filt_off[ns]);
  float* dTarget = reinterpret_cast<float*>(c->ws[22].ensure(sizeof(float) * (size_t)ns));
  int64_t* dRank = reinterpret_cast<int64_t*>(c->ws[23].ensure(sizeof(int64_t) * (size_t)ns));

  const int half = c->dim / 2;
  KP_HIP(hipEventRecord(c->ev0, c->stream));
  if (npq > 0) {
    hipLaunchKernelGGL(kp_cx_tsum, dim3(npq), dim3(128), 0, c->stream, c->dE, DP, dPq, npq, dTg, dTsum);
    KP_HIP(hipGetLastError());
  }
  // frozen-head pairs: q and frozen log-sum-exp
  int slots_attn = 0;
  CX_DISPATCH(DBV, slots_attn = attn_slots_db<DB>(c));
  const AttnPlan plan_pairs = attn_plan_ctx(c, std::max(npairs, 1), c->n_ent, slots_attn);
  const int split_pairs = plan_pairs.wk.n_parts;
  size_t att_rows = (size_t)std::max(npairs, 1) * split_pairs;
  std::vector<AttnPlan> step_plan(T);
  for (int t = 0; t < T; ++t) {
    const int nq = q_off[t + 1] - q_off[t];
    step_plan[t] = attn_plan_ctx(c, std::max(nq, 1), c->n_ent, slots_attn);
    att_rows = std::max(att_rows, (size_t)nq * step_plan[t].wk.n_parts);
  }
  float* dAm = reinterpret_cast<float*>(c->ws[13].ensure(sizeof(float) * att_rows));
  float* dAl = reinterpret_cast<float*>(c->ws[14].ensure(sizeof(float) * att_rows));
  float* dAO = reinterpret_cast<float*>(c->ws[15].ensure(sizeof(float) * att_rows * DP));
  float* dQs = reinterpret_cast<float*>(c->ws[26].ensure(sizeof(float) * (size_t)std::max(max_nq, 1) * DP));
  if (npairs > 0) {
    hipLaunchKernelGGL(kp_cx_qpair, dim3(npairs), dim3(128), 0, c->stream, c->dE, c->dR, DP, half, dPairs, npairs,
                       dQpair);
    KP_HIP(hipGetLastError());
    CX_DISPATCH(DBV, launch_attn<DB>(c, false, dQpair, npairs, plan_pairs, dAm, dAl, nullptr));
    // combine the splits into lsef on the device (no host round trip inside the batch)
    hipLaunchKernelGGL(kp_cx_lse_merge, dim3((npairs + 255) / 256), dim3(256), 0, c->stream, npairs, split_pairs, dAm,
                       dAl, dLsef);
    KP_HIP(hipGetLastError());
  }

  // ---- the epoch/step loop
  CxOpt opt{};
  opt.kind = hp->optimizer;
  opt.lr = hp->lr;
  opt.b1 = hp->beta1;
  opt.b2 = hp->beta2;
  opt.eps = hp->eps;
  opt.one_minus_b1 = (float)(1.0 - (double)hp->beta1);
  opt.one_minus_b2 = (float)(1.0 - (double)hp->beta2);
  opt.reg_w = hp->reg_weight;
  KP_REQUIRE(hp->reg_kind == KP_REG_N3 || hp->reg_kind == KP_REG_N2, "ComplEx: unknown regulariser");
  opt.reg_n2 = hp->reg_kind == KP_REG_N2;
  // loop-interval events, destroyed on every exit path (a KP_HIP / KP_REQUIRE below throws)
  struct LoopEvents {
    hipEvent_t a = nullptr, b = nullptr;
    ~LoopEvents() {
      if (a) (void)hipEventDestroy(a);
      if (b) (void)hipEventDestroy(b);
    }
  } lev;
  KP_HIP(hipEventCreate(&lev.a));
  KP_HIP(hipEventCreate(&lev.b));
  hipEvent_t h0 = lev.a, h1 = lev.b;
  KP_HIP(hipEventRecord(h0, c->stream));
  const double t_loop0 = g_host_times ? host_ms() : 0.0;
  double t_steps[4] = {0, 0, 0, 0};  // host time after enqueueing steps 0, 1, T/2, T-1
  int64_t hot_launches = 0;
  c->hot_pairs.clear();
  c->hot_iv.clear();
  for (int t = 0; t < T; ++t) {
    const int nq = q_off[t + 1] - q_off[t];
    const int na = act_off[t + 1] - act_off[t];
    const int sp = step_plan[t].wk.n_parts;
    hipEvent_t ea = nullptr, eb = nullptr;
    if (nq > 0 && c->time_hot) {
      ea = c->event(2 * hot_launches);
      eb = c->event(2 * hot_launches + 1);
    }
    CX_DISPATCH(DBV, launch_stepq<DB>(c, dStepQ + q_off[t], dX, nq, dQs));
    if (nq > 0 && c->time_hot) KP_HIP(hipEventRecord(ea, c->stream));
    CX_DISPATCH(DBV, launch_attn<DB>(c, true, dQs, nq, step_plan[t], dAm, dAl, dAO));
    if (nq > 0) {
      if (c->time_hot) {
        KP_HIP(hipEventRecord(eb, c->stream));
        c->hot_pairs.push_back({(double)nq, 0.0});
      }
      ++hot_launches;
    }
    const double step = (double)(t + 1);
    opt.step_size = (float)((double)hp->lr / (1.0 - std::pow((double)hp->beta1, step)));
    opt.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)hp->beta2, step));
    CX_DISPATCH(DBV, launch_update<DB>(c, na, dActs + act_off[t], dPlans, dPq, dStepQ + q_off[t], nq,
                                       dStepT + t_off[t], t_off[t + 1] - t_off[t], dTsum, dQpair, dLsef, dAm, dAl, dAO,
                                       sp, dContrib, dX, dS1, dS2, opt));
    if (g_host_times) {
      if (t == 0) t_steps[0] = host_ms();
      if (t == 1) t_steps[1] = host_ms();
      if (t == T / 2) t_steps[2] = host_ms();
      if (t == T - 1) t_steps[3] = host_ms();
    }
  }
  KP_HIP(hipEventRecord(h1, c->stream));

  // ---- ranking: scores of (kelpie, p, .) over E plus the kelpie column, in fp64
  // (launch_rank_f64: at the reference init the target's neighbours are ~1e-5 relative away)
  CX_DISPATCH(DBV, launch_rankq64<DB>(c, dX, dPred, ns, dQ64, dT64, dT64 + ns));
  launch_rank_f64(c, ns, dQ64, dT64, dT64 + ns, dPo, dFo, dF, dTarget, dRank);
  KP_HIP(hipEventRecord(c->ev1, c->stream));

  if (bt->out_x) {
    std::vector<float> xp((size_t)ns * DP);
    KP_HIP(hipMemcpyAsync(xp.data(), dX, sizeof(float) * xp.size(), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
    for (int s = 0; s < ns; ++s)
      std::memcpy(bt->out_x + (size_t)s * c->dim, &xp[(size_t)s * DP], sizeof(float) * c->dim);
  }
  KP_HIP(hipMemcpyAsync(bt->out_score, dTarget, sizeof(float) * ns, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipMemcpyAsync(bt->out_rank, dRank, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, c->stream));
  const double t_enq = g_host_times ? host_ms() : 0.0;
  KP_HIP(hipStreamSynchronize(c->stream));
  if (g_host_times)
    std::fprintf(stderr,
                 "[kp_cx] slots %d steps %d: plan %.2f ms, enqueue %.2f ms (uploads+pairs %.2f, step 0 %.2f, step 1 "
                 "%.2f, to T/2 %.2f, to T-1 %.2f), wait %.2f ms\n",
                 ns, T, t_plan - t_in, t_enq - t_plan, t_loop0 - t_plan, t_steps[0] - t_loop0, t_steps[1] - t_steps[0],
                 t_steps[2] - t_steps[1], t_steps[3] - t_steps[2], host_ms() - t_enq);
  float ms_all = 0.f, ms_loop = 0.f;
  KP_HIP(hipEventElapsedTime(&ms_all, c->ev0, c->ev1));
  KP_HIP(hipEventElapsedTime(&ms_loop, h0, h1));
  double hot = 0.0;
  for (size_t i = 0; i < c->hot_pairs.size(); ++i) {
    float ms = 0.f;
    KP_HIP(hipEventElapsedTime(&ms, c->event(2 * i), c->event(2 * i + 1)));
    c->hot_pairs[i].second = ms * 1e-3;
    hot += ms * 1e-3;
    kp_push_interval(c, c->event(2 * i), c->event(2 * i + 1));
  }
  c->timing.device_s = ms_all * 1e-3;
  c->timing.loop_s = ms_loop * 1e-3;
  c->timing.hot_s = hot;
  c->timing.hot_launches = hot_launches;
  double work = 0.0;
  for (auto& pr : c->hot_pairs) work += pr.first * (double)c->n_ent;
  c->timing.hot_work = work;
}

void complex_scores_dev(kp_ctx* c, int n, const int32_t* dh, const int32_t* dr, float* dS, int ld) {
  if (n <= 0) return;
  const int DP = c->dp;
  float* dQ = reinterpret_cast<float*>(c->ws[17].ensure(sizeof(float) * (size_t)n * DP));
  hipLaunchKernelGGL(kp_cx_scoreq, dim3(n), dim3(128), 0, c->stream, c->dE, c->dR, DP, c->dim / 2, dh, dr, n, dQ);
  KP_HIP(hipGetLastError());
  launch_score_gemm(c, dQ, n, dS, ld, 0);
}

void complex_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out) {
  if (n <= 0) return;
  int32_t* dh = upload(c, c->ws[18], heads, (size_t)n);
  int32_t* dr = upload(c, c->ws[19], rels, (size_t)n);
  float* dS = reinterpret_cast<float*>(c->ws[16].ensure(sizeof(float) * (size_t)n * c->n_ent));
  complex_scores_dev(c, n, dh, dr, dS, c->n_ent);
  KP_HIP(hipMemcpyAsync(out, dS, sizeof(float) * (size_t)n * c->n_ent, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
}

#ifdef KP_ATTN_STAMPS
extern "C" int kp_debug_attn_stamps(unsigned long long* out, int reset) {
  KP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(kpattn::g_attn_stamps), sizeof(unsigned long long) * 8));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    KP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kpattn::g_attn_stamps), z, sizeof(z)));
  }
  return 0;
}
#endif
