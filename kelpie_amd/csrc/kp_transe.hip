// kp_transe.hip -- TransE batched post-training (KelpieTransE +
// KelpiePairwiseRankingOptimizer) and ranking, for gfx950.
//
// Reference semantics (src/link_prediction/models/transe.py:45-99,
// src/link_prediction/optimization/pairwise_ranking_optimizer.py:139-203):
//   per epoch: np.random.shuffle(rows); positives = repeat(rows, ratio); only the
//   first R of the ratio*R repeated rows are stepped (SURVEY A-Q2), in batches
//   of batch_size; negatives corrupt the head (head_or_tail == 1) or the tail
//   with a random entity in [0, |E|] (the kelpie id included, A-Q3);
//   loss = mean(max(0, f+ - f- + margin)) + lambda * (L2(pos) + L2(neg)) / 2,
//   f = ||lhs + rel - rhs||_2, L2 = (mean lhs^2 + mean rel^2 + mean rhs^2) / 3;
//   Adam(lr) on the kelpie row only.
//
// One workgroup per slot runs every epoch on chip (x and the Adam moments in
// LDS); 16 groups of 16 lanes each take one (positive, negative) pair at a
// time, reduce their two squared norms with 16-lane shuffles and accumulate
// the single-row gradient (TransE) in registers.  The random
// draws arrive as inputs: per epoch [row order | negative entity | head_or_tail].
// Memory-bound: every pair gathers up to 4 entity rows and a relation row
// from the L2 / Infinity Cache.
#include <cmath>

#include "kp_common.hpp"

namespace {

struct TeSlot {
  int row_off, R;
  long long rng_off;
};

struct TeHp {
  int epochs, bs, ratio;
  float margin, lam, lr, b1, b2, eps, one_minus_b1, one_minus_b2;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

constexpr int TE_CH = 256;
constexpr int TE_PPG = 2;  // pairs in flight per 16-lane group (all their row loads issued before the math)

#ifdef KP_TE_STAMPS
// diagnostic build only: per-phase cycles of kp_te_posttrain summed over wave 0 of
// every workgroup: [staging, pairs, chunk sync, reduce + Adam]
__device__ unsigned long long g_te_stamps[8];
#define TE_STAMP(k) te_ts[k] = __builtin_amdgcn_s_memtime()
#else
#define TE_STAMP(k) (void)0
#endif  // stepped pairs whose descriptors are staged in LDS at a time

// one (positive, negative) pair: the two difference vectors of 16 lanes x VPL float4
template <int VPL>
struct TePair {
  float4 vp[VPL], vn[VPL];
  float sp, sn;
};

// Row loads of one pair.  Frozen rows come from global memory (global_load, the
// kelpie id K replaced by row 0) and the kelpie row from LDS, selected per value:
// one flat load per row would let a 16-lane group's pointer alias either space.
template <int VPL>
__device__ __forceinline__ void te_load(TePair<VPL>& P, const float* __restrict__ E,
                                        const float* __restrict__ Rt, const float* xs, int dp, int K, int4 dsc,
                                        int tn, int l16, int NF4) {
  const int h = dsc.x, r = dsc.y, t = dsc.z, hn = dsc.w;
  const float* Lp = E + (size_t)(h == K ? 0 : h) * dp;
  const float* Rp = E + (size_t)(t == K ? 0 : t) * dp;
  const float* Ln = E + (size_t)(hn == K ? 0 : hn) * dp;
  const float* Rn = E + (size_t)(tn == K ? 0 : tn) * dp;
  const float* rel = Rt + (size_t)r * dp;
  P.sp = 0.f;
  P.sn = 0.f;
  // branch-free: lanes past the row end load a clamped duplicate and are zeroed, so
  // every pair's loads sit in one basic block and can all be in flight together
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int f0 = l16 + 16 * u;
    const bool on = f0 < NF4;
    const int f = on ? f0 : NF4 - 1;
    const float4 xk = ld4(xs + 4 * f);
    float4 a = ld4(Lp + 4 * f), c = ld4(Rp + 4 * f), a2 = ld4(Ln + 4 * f), c2 = ld4(Rn + 4 * f);
    const float4 b = ld4(rel + 4 * f);
    if (h == K) a = xk;
    if (t == K) c = xk;
    if (hn == K) a2 = xk;
    if (tn == K) c2 = xk;
    const float4 vp = make_float4((a.x + b.x) - c.x, (a.y + b.y) - c.y, (a.z + b.z) - c.z, (a.w + b.w) - c.w);
    const float4 vn = make_float4((a2.x + b.x) - c2.x, (a2.y + b.y) - c2.y, (a2.z + b.z) - c2.z, (a2.w + b.w) - c2.w);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    P.vp[u] = on ? vp : z;
    P.vn[u] = on ? vn : z;
  }
}

template <int VPL>
__device__ __forceinline__ void te_accum(TePair<VPL>& P, const int4 dsc, int tn, int K, float margin, float4* g,
                                         int& cnt) {
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    P.sp += P.vp[u].x * P.vp[u].x + P.vp[u].y * P.vp[u].y + P.vp[u].z * P.vp[u].z + P.vp[u].w * P.vp[u].w;
    P.sn += P.vn[u].x * P.vn[u].x + P.vn[u].y * P.vn[u].y + P.vn[u].z * P.vn[u].z + P.vn[u].w * P.vn[u].w;
  }
  P.sp = row16_sum(P.sp);
  P.sn = row16_sum(P.sn);
  const int h = dsc.x, t = dsc.z, hn = dsc.w;
  const float fp = sqrtf(P.sp), fn = sqrtf(P.sn);
  const float z = (fp - fn) + margin;
  const bool act = z >= 0.f;  // clamp_min backward passes grad where self >= min
  const float sgn_p = (float)((h == K) - (t == K));
  const float sgn_n = (float)((hn == K) - (tn == K));
  const float cp = (act && fp > 0.f) ? sgn_p / fp : 0.f;
  const float cn = (act && fn > 0.f) ? -sgn_n / fn : 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    g[u].x += cp * P.vp[u].x + cn * P.vn[u].x;
    g[u].y += cp * P.vp[u].y + cn * P.vn[u].y;
    g[u].z += cp * P.vp[u].z + cn * P.vn[u].z;
    g[u].w += cp * P.vp[u].w + cn * P.vn[u].w;
  }
  cnt += (h == K) + (t == K) + (hn == K) + (tn == K);
}

template <int VPL>  // float4 per lane (16 lanes per row): DP <= 64 * VPL
__global__ __launch_bounds__(256, 2) void kp_te_posttrain(int n_ent, int dp, int d, const float* __restrict__ E,
                                                       const float* __restrict__ R,
                                                       const TeSlot* __restrict__ slots,
                                                       const int32_t* __restrict__ rows,
                                                       const int32_t* __restrict__ rng, TeHp hp,
                                                       float* __restrict__ X) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;                                            // [dp]
  float* red = sm + dp;                                      // [16][dp] per-group gradient partials
  int4* dsc = reinterpret_cast<int4*>(sm + 17 * dp);         // [TE_CH] (h, r, t, h_neg)
  int* dtn = reinterpret_cast<int*>(dsc + TE_CH);            // [TE_CH] t_neg
  __shared__ int cnt_s[16];
  const int tid = threadIdx.x;
  const int grp = tid >> 4, l16 = tid & 15;
  const TeSlot S = slots[blockIdx.x];
  const int K = n_ent;
  float* x = X + (size_t)blockIdx.x * dp;
  for (int i = tid; i < dp; i += 256) xs[i] = x[i];
  // Adam moments: thread i owns element i (and i+256)
  float m1[2] = {0.f, 0.f}, v2[2] = {0.f, 0.f};
  __syncthreads();
  const int32_t* rw = rows + 3 * (size_t)S.row_off;
  const int NF4 = dp / 4;
  double b1t = 1.0, b2t = 1.0;
#ifdef KP_TE_STAMPS
  unsigned long long te_ts[5] = {0, 0, 0, 0, 0}, te_acc[4] = {0, 0, 0, 0}, te_wait = 0, te_rounds = 0;
#endif
  for (int e = 0; e < hp.epochs; ++e) {
    const int32_t* order = rng + S.rng_off + (long long)e * 3 * S.R;
    const int32_t* ents = order + S.R;
    const int32_t* hot = order + 2 * S.R;
    for (int st = 0; st < S.R; st += hp.bs) {
      const int B = min(hp.bs, S.R - st);
      float4 g[VPL];
#pragma unroll
      for (int u = 0; u < VPL; ++u) g[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      int cnt = 0;
      for (int c0 = st; c0 < st + B; c0 += TE_CH) {
        TE_STAMP(0);
        const int n = min(TE_CH, st + B - c0);
        // ---- stage the chunk's pair descriptors (coalesced draws, row gathers from L2)
        for (int k = tid; k < n; k += 256) {
          const int j = c0 + k;
          const int ri = order[j / hp.ratio];
          const int h = rw[3 * ri], r = rw[3 * ri + 1], t = rw[3 * ri + 2];
          const int ent = ents[j];
          const bool corrupt_head = hot[j] == 1;
          dsc[k] = make_int4(h, r, t, corrupt_head ? ent : h);
          dtn[k] = corrupt_head ? t : ent;
        }
        __syncthreads();
        TE_STAMP(1);
        // ---- TE_PPG pairs per group in flight: all their row loads issued before the math
        for (int k0 = grp; k0 < n; k0 += 16 * TE_PPG) {
          TePair<VPL> P[TE_PPG];
          int4 dd[TE_PPG];
          int tt[TE_PPG];
#pragma unroll
          for (int u = 0; u < TE_PPG; ++u) {
            const int k = min(k0 + 16 * u, n - 1);  // past the chunk: reload a valid pair, not accumulated
            dd[u] = dsc[k];
            tt[u] = dtn[k];
            te_load<VPL>(P[u], E, R, xs, dp, K, dd[u], tt[u], l16, NF4);
          }
#ifdef KP_TE_STAMPS
          const unsigned long long r0 = __builtin_amdgcn_s_memtime();
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          const unsigned long long r1 = __builtin_amdgcn_s_memtime();
          te_wait += r1 - r0;
#endif
#pragma unroll
          for (int u = 0; u < TE_PPG; ++u)
            if (k0 + 16 * u < n) te_accum<VPL>(P[u], dd[u], tt[u], K, hp.margin, g, cnt);
#ifdef KP_TE_STAMPS
          te_rounds += 1;
#endif
        }
        TE_STAMP(2);
        __syncthreads();  // the next chunk overwrites the descriptors
      }
      TE_STAMP(3);
      // ---- reduce the 16 group partials
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        const int f = l16 + 16 * u;
        if (f < NF4) *reinterpret_cast<float4*>(red + grp * dp + 4 * f) = g[u];
      }
      if (l16 == 0) cnt_s[grp] = cnt;
      __syncthreads();
      int ctot = 0;
      for (int k = 0; k < 16; ++k) ctot += cnt_s[k];
      const float invB = 1.0f / (float)B;
      const float regc = hp.lam / (3.0f * (float)B * (float)d) * (float)ctot;
      b1t *= (double)hp.b1;
      b2t *= (double)hp.b2;
      const float step_size = (float)((double)hp.lr / (1.0 - b1t));
      const float bc2s = (float)sqrt(1.0 - b2t);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u;
        if (i < dp) {
          float gs = 0.f;
          for (int k = 0; k < 16; ++k) gs += red[k * dp + i];
          const float xi = xs[i];
          const float gi = gs * invB + regc * xi;
          m1[u] = m1[u] + hp.one_minus_b1 * (gi - m1[u]);
          v2[u] = v2[u] * hp.b2;
          v2[u] = v2[u] + (hp.one_minus_b2 * gi) * gi;
          const float den = sqrtf(v2[u]) / bc2s + hp.eps;
          const float xn = (i < d) ? xi + (-step_size * m1[u]) / den : 0.f;
          red[i] = xn;  // stage (group 0's slot is consumed already)
        }
      }
      __syncthreads();
      for (int i = tid; i < dp; i += 256) xs[i] = red[i];
      __syncthreads();
      TE_STAMP(4);
#ifdef KP_TE_STAMPS
      te_acc[0] += te_ts[1] - te_ts[0];
      te_acc[1] += te_ts[2] - te_ts[1];
      te_acc[2] += te_ts[3] - te_ts[2];
      te_acc[3] += te_ts[4] - te_ts[3];
#endif
    }
  }
  for (int i = tid; i < dp; i += 256) x[i] = xs[i];
#ifdef KP_TE_STAMPS
  if (tid == 0) {
    for (int k = 0; k < 2; ++k) atomicAdd(&g_te_stamps[k], te_acc[k]);
    atomicAdd(&g_te_stamps[4], 1ull);
    atomicAdd(&g_te_stamps[5], (unsigned long long)S.R);
    atomicMax(&g_te_stamps[6], te_acc[0] + te_acc[1] + te_acc[2] + te_acc[3]);
    atomicMax(&g_te_stamps[7], (unsigned long long)S.R);
    atomicAdd(&g_te_stamps[2], te_wait);    // (reuses the chunk-sync slot: load wait inside the pair loop)
    atomicAdd(&g_te_stamps[3], te_rounds);  // (reuses the reduce slot: rounds)
  }
#endif
}

// scores[q][e] = || (lhs_q + rel_q) - E_e ||_2 for e < n_ent (transe.py:48-65);
// lhs_q is a frozen row (heads[q] >= 0) or the slot's kelpie row X[q].
#define TS_Q 8
__global__ __launch_bounds__(256) void kp_te_scores(int n_ent, int dp, const float* __restrict__ E,
                                                    const float* __restrict__ R, int nq,
                                                    const int32_t* __restrict__ heads,
                                                    const int32_t* __restrict__ rels,
                                                    const float* __restrict__ X, float* __restrict__ out, int ld,
                                                    int kcol) {
  extern __shared__ __attribute__((aligned(16))) float tq[];  // [TS_Q][dp]
  const int q0 = blockIdx.y * TS_Q;
  for (int i = threadIdx.x; i < TS_Q * dp; i += blockDim.x) {
    const int q = q0 + i / dp, k = i % dp;
    float v = 0.f;
    if (q < nq) {
      const int h = heads[q];
      const float lhs = (h >= 0) ? E[(size_t)h * dp + k] : X[(size_t)q * dp + k];
      v = lhs + R[(size_t)rels[q] * dp + k];
    }
    tq[i] = v;
  }
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n_ent) {
    float acc[TS_Q];
#pragma unroll
    for (int q = 0; q < TS_Q; ++q) acc[q] = 0.f;
    const float* row = E + (size_t)e * dp;
    for (int k = 0; k < dp; k += 4) {
      const float4 v = ld4(row + k);
#pragma unroll
      for (int q = 0; q < TS_Q; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(tq + q * dp + k);
        const float a = t.x - v.x, b = t.y - v.y, c = t.z - v.z, w = t.w - v.w;
        acc[q] += a * a + b * b + c * c + w * w;
      }
    }
#pragma unroll
    for (int q = 0; q < TS_Q; ++q)
      if (q0 + q < nq) out[(size_t)(q0 + q) * ld + e] = sqrtf(acc[q]);
  }
  // kelpie column: || (x + r) - x ||
  if (kcol >= 0 && blockIdx.x == 0 && threadIdx.x < TS_Q) {
    const int q = q0 + threadIdx.x;
    if (q < nq) {
      float acc = 0.f;
      for (int k = 0; k < dp; ++k) {
        const float dlt = tq[threadIdx.x * dp + k] - X[(size_t)q * dp + k];
        acc += dlt * dlt;
      }
      out[(size_t)q * ld + kcol] = sqrtf(acc);
    }
  }
}

void launch_te_scores(kp_ctx* c, int nq, const int32_t* dh, const int32_t* dr, const float* dX, float* dOut, int ld,
                      int kcol) {
  if (nq <= 0) return;
  dim3 grid((c->n_ent + 255) / 256, (nq + TS_Q - 1) / TS_Q);
  const size_t shm = sizeof(float) * TS_Q * c->dp;
  hipLaunchKernelGGL(kp_te_scores, grid, dim3(256), shm, c->stream, c->n_ent, c->dp, c->dE, c->dR, nq, dh, dr, dX,
                     dOut, ld, kcol);
  KP_HIP(hipGetLastError());
}

}  // namespace

void transe_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* bt) {
  const int ns = bt->n_slots;
  const int DP = c->dp;
  KP_REQUIRE(hp->neg_ratio >= 1 && hp->batch_size >= 1 && hp->epochs >= 0, "TransE: bad hyper-parameters");
  std::vector<TeSlot> slots(ns);
  for (int s = 0; s < ns; ++s) {
    const int R = bt->row_off[s + 1] - bt->row_off[s];
    KP_REQUIRE(R >= 0, "TransE: bad row_off");
    slots[s] = TeSlot{bt->row_off[s], R, (long long)bt->rng_off[s]};
    KP_REQUIRE(bt->rng_off[s + 1] - bt->rng_off[s] >= (int64_t)hp->epochs * 3 * R,
               "TransE: missing per-epoch draws (order | entities | head_or_tail)");
  }
  const int total_rows = bt->row_off[ns];
  for (int i = 0; i < 3 * total_rows; ++i)
    KP_REQUIRE(bt->rows[i] >= 0 && bt->rows[i] <= ((i % 3) == 1 ? c->n_rel2 - 1 : c->n_ent),
               "TransE: row id out of range");
  std::vector<float> xp((size_t)ns * DP, 0.f);
  for (int s = 0; s < ns; ++s) std::memcpy(&xp[(size_t)s * DP], bt->x0 + (size_t)s * c->dim, sizeof(float) * c->dim);
  float* dX = upload(c, c->ws[0], xp.data(), xp.size());
  TeSlot* dSlots = upload(c, c->ws[1], slots.data(), slots.size());
  int32_t* dRows = upload(c, c->ws[2], bt->rows, (size_t)std::max(1, 3 * total_rows));
  const int64_t nrng = bt->rng_off[ns];
  int32_t* dRng = upload(c, c->ws[3], bt->rng, (size_t)std::max<int64_t>(1, nrng));

  TeHp h{};
  h.epochs = hp->epochs;
  h.bs = hp->batch_size;
  h.ratio = hp->neg_ratio;
  h.margin = hp->margin;
  h.lam = hp->reg_weight;
  h.lr = hp->lr;
  h.b1 = hp->beta1;
  h.b2 = hp->beta2;
  h.eps = hp->eps;
  h.one_minus_b1 = (float)(1.0 - (double)hp->beta1);
  h.one_minus_b2 = (float)(1.0 - (double)hp->beta2);

  KP_HIP(hipEventRecord(c->ev0, c->stream));
  hipEvent_t ea = c->event(0), eb = c->event(1);
  KP_HIP(hipEventRecord(ea, c->stream));
  const size_t shm = sizeof(float) * (size_t)17 * DP + sizeof(int4) * TE_CH + sizeof(int) * TE_CH;
  const int vpl = (DP + 63) / 64;
  switch (vpl) {
#define TE_CASE(V)                                                                                              \
  case V:                                                                                                       \
    hipLaunchKernelGGL(kp_te_posttrain<V>, dim3(ns), dim3(256), shm, c->stream, c->n_ent, DP, c->dim, c->dE, c->dR, \
                       dSlots, dRows, dRng, h, dX);                                                             \
    break;
    TE_CASE(1)
    TE_CASE(2)
    TE_CASE(3)
    TE_CASE(4)
    TE_CASE(5)
    TE_CASE(6)
    TE_CASE(7)
    TE_CASE(8)
#undef TE_CASE
    default:
      throw KpError{KP_ENOTSUP, "TransE: dimension > 512 not supported"};
  }
  KP_HIP(hipGetLastError());
  KP_HIP(hipEventRecord(eb, c->stream));

  // ---- rank: scores of (kelpie, p, .) = ||(x + R_p) - E_e||, minimizer
  const int ld = round_up(c->n_ent + 1, 4);
  std::vector<int32_t> heads(ns, -1), rels(ns), po(ns);
  for (int s = 0; s < ns; ++s) {
    rels[s] = bt->pred[3 * s + 1];
    po[s] = bt->pred[3 * s + 2];
    KP_REQUIRE(bt->pred[3 * s] == c->n_ent, "TransE: the ranked triple must start at the kelpie entity");
  }
  int32_t* dH = upload(c, c->ws[4], heads.data(), heads.size());
  int32_t* dRl = upload(c, c->ws[5], rels.data(), rels.size());
  int32_t* dPo = upload(c, c->ws[6], po.data(), po.size());
  int32_t* dFo = upload(c, c->ws[7], bt->filt_off, (size_t)ns + 1);
  int32_t* dF = upload(c, c->ws[8], bt->filt, (size_t)std::max(1, bt->filt_off[ns]));
  float* dScores = reinterpret_cast<float*>(c->ws[9].ensure(sizeof(float) * (size_t)ns * ld));
  float* dTarget = reinterpret_cast<float*>(c->ws[10].ensure(sizeof(float) * ns));
  int64_t* dRank = reinterpret_cast<int64_t*>(c->ws[11].ensure(sizeof(int64_t) * ns));
  launch_te_scores(c, ns, dH, dRl, dX, dScores, ld, c->n_ent);
  launch_rank_count(c, ns, dScores, ld, c->n_ent + 1, dPo, dFo, dF, 1, dTarget, dRank);
  KP_HIP(hipEventRecord(c->ev1, c->stream));
  if (bt->out_x) {
    KP_HIP(hipMemcpyAsync(xp.data(), dX, sizeof(float) * xp.size(), hipMemcpyDeviceToHost, c->stream));
  }
  KP_HIP(hipMemcpyAsync(bt->out_score, dTarget, sizeof(float) * ns, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipMemcpyAsync(bt->out_rank, dRank, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  if (bt->out_x)
    for (int s = 0; s < ns; ++s) std::memcpy(bt->out_x + (size_t)s * c->dim, &xp[(size_t)s * DP], sizeof(float) * c->dim);
  float ms_all = 0.f, ms_hot = 0.f;
  KP_HIP(hipEventElapsedTime(&ms_all, c->ev0, c->ev1));
  KP_HIP(hipEventElapsedTime(&ms_hot, ea, eb));
  double work = 0;
  for (int s = 0; s < ns; ++s) work += (double)hp->epochs * slots[s].R;
  c->timing.device_s = ms_all * 1e-3;
  c->timing.loop_s = ms_hot * 1e-3;
  c->timing.hot_s = ms_hot * 1e-3;
  c->timing.hot_launches = 1;
  c->timing.hot_work = work;  // stepped (positive, negative) pairs
}

void transe_scores_dev(kp_ctx* c, int n, const int32_t* d_heads, const int32_t* d_rels, float* d_out, int ld) {
  launch_te_scores(c, n, d_heads, d_rels, nullptr, d_out, ld, -1);
}

void transe_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out) {
  if (n <= 0) return;
  int32_t* dh = upload(c, c->ws[4], heads, (size_t)n);
  int32_t* dr = upload(c, c->ws[5], rels, (size_t)n);
  float* dS = reinterpret_cast<float*>(c->ws[9].ensure(sizeof(float) * (size_t)n * c->n_ent));
  transe_scores_dev(c, n, dh, dr, dS, c->n_ent);
  KP_HIP(hipMemcpyAsync(out, dS, sizeof(float) * (size_t)n * c->n_ent, hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
}

#ifdef KP_TE_STAMPS
extern "C" int kp_debug_te_stamps(unsigned long long* out, int reset) {
  KP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_te_stamps), sizeof(unsigned long long) * 8));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    KP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_te_stamps), z, sizeof(z)));
  }
  return 0;
}
#endif
