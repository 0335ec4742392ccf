// kp_rank.hip -- all-entity scoring (fp32 MFMA) and the filtered rank of
// PostTrainingEngine.get_triple_results (post_training_engine.py:101-125).
#include "kp_common.hpp"

// ----------------------------------------------------------------------------
// score GEMM:  out[q][e] = act( Q[q] . E[e] )  for e < n_ent
//   Q [nq][dp], E [n_ent][dp] (dp multiple of 16, zero padded), out row stride ld.
//   fp32 MFMA v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain).  Block tile
//   64 queries x 64 entities x BK 32, 4 waves; wave w owns queries [16w,16w+16)
//   x 64 entities (4 accumulators).  C layout: row (query) = 4*(l>>4)+r,
//   col (entity) = l&15 -> lanes store consecutive entities (coalesced).
//   act: 0 identity (ComplEx), 1 sigmoid (ConvE, conve.py:156).
// ----------------------------------------------------------------------------
#define SG_BM 64
#define SG_BN 64
#define SG_BK 32
#define SG_LD (SG_BK + 4)

__global__ __launch_bounds__(256) void kp_gemm_abt(const float* __restrict__ A, int lda, int M,
                                                   const float* __restrict__ B, int ldb, int N, int k_begin,
                                                   int k_end, float* __restrict__ out, int ldo,
                                                   const float* __restrict__ bias, int act) {
  __shared__ __attribute__((aligned(16))) float Qs[SG_BM * SG_LD];
  __shared__ __attribute__((aligned(16))) float Es[SG_BN * SG_LD];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int q0 = blockIdx.y * SG_BM;
  const int e0 = blockIdx.x * SG_BN;
  // split-K: blockIdx.z selects a K range and an output slab
  const int ksplit = gridDim.z;
  const int klen = (k_end - k_begin + ksplit - 1) / ksplit;
  const int kb = k_begin + blockIdx.z * ((klen + SG_BK - 1) / SG_BK * SG_BK);
  const int ke = min(k_end, kb + (klen + SG_BK - 1) / SG_BK * SG_BK);
  out += (size_t)blockIdx.z * M * ldo;
  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int k0 = kb; k0 < ke; k0 += SG_BK) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int f = tid + 256 * u;
      int row = f >> 3, c4 = (f & 7) * 4;
      float4 vq = make_float4(0.f, 0.f, 0.f, 0.f), ve = vq;
      int kk = k0 + c4;
      if (q0 + row < M && kk < ke) vq = *reinterpret_cast<const float4*>(A + (size_t)(q0 + row) * lda + kk);
      if (e0 + row < N && kk < ke) ve = *reinterpret_cast<const float4*>(B + (size_t)(e0 + row) * ldb + kk);
      *reinterpret_cast<float4*>(&Qs[row * SG_LD + c4]) = vq;
      *reinterpret_cast<float4*>(&Es[row * SG_LD + c4]) = ve;
    }
    __syncthreads();
    // k permuted within each 16-deep chunk: MFMA i of a chunk pairs lane group g with
    // k = kk + 4g + i on both operands, so a lane's A and B values for four MFMAs are
    // one 16-byte LDS read each (the sum over k is unchanged, only its order)
#pragma unroll
    for (int kk = 0; kk < SG_BK; kk += 16) {
      const f32x4 a4 = *reinterpret_cast<const f32x4*>(&Qs[(16 * w + c) * SG_LD + kk + 4 * g]);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(&Es[(16 * n + c) * SG_LD + kk + 4 * g]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i], b4[i], acc[n], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    int e = e0 + 16 * n + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int q = q0 + 16 * w + 4 * g + r;
      if (q < M && e < N) {
        float v = acc[n][r];
        if (bias && blockIdx.z == 0) v += bias[e];
        if (act == 1) v = 1.0f / (1.0f + expf(-v));  // torch.sigmoid in float32 (accurate exp)
        out[(size_t)q * ldo + e] = v;
      }
    }
  }
}

// ----------------------------------------------------------------------------
// filtered rank, one workgroup per slot.
//   scores[s][0..n_cols) (column n_cols-1 is the kelpie entity when present)
//   minimizer: v_e = 1e6 for e in F, v_o = target, rank = #{v_e <= target}
//   maximizer: v_e = -1e6 for e in F,             rank = #{v_e >= target}
//   (post_training_engine.py:110-119; an o in F is excluded for maximizers)
// ----------------------------------------------------------------------------
// mode RANK_TRIPLE_RESULTS: PostTrainingEngine.get_triple_results (post_training_engine.py:101-125):
//   minimizer: filtered -> 1e6, o restored, count <= target; maximizer: filtered ->
//   -1e6 (o NOT restored when filtered), count >= target.
// mode RANK_PREDICT_TAILS: Model.predict_tails (model.py:42-68): filtered -> +-1e6, o
//   restored, count <= / >= target.
// mode RANK_SORT_POSITION: ConvE.predict_tails (conve.py:160-184): filtered -> 0.0, o
//   restored, rank = 1 + #(v > target), the position of o in a descending sort when
//   no other entity ties with it (torch.sort's order among ties is unspecified).
__global__ __launch_bounds__(256) void kp_rank_count(int n_slots, const float* __restrict__ scores, int ld,
                                                     int n_cols, const int32_t* __restrict__ pred_o,
                                                     const int32_t* __restrict__ filt_off,
                                                     const int32_t* __restrict__ filt, int minimizer,
                                                     float* __restrict__ target_out,
                                                     int64_t* __restrict__ rank_out, int mode) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
  __shared__ int partial[4];
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int nwords = (n_cols + 31) >> 5;
  for (int i = tid; i < nwords; i += blockDim.x) bits[i] = 0u;
  __syncthreads();
  const int f0 = filt_off[s], f1 = filt_off[s + 1];
  for (int i = f0 + tid; i < f1; i += blockDim.x) {
    int e = filt[i];
    if (e >= 0 && e < n_cols) atomicOr(&bits[e >> 5], 1u << (e & 31));
  }
  __syncthreads();
  const float* row = scores + (size_t)s * ld;
  const int o = pred_o[s];
  const float target = row[o];
  int cnt = 0;
  if (minimizer) {
    for (int e = tid; e < n_cols; e += blockDim.x) {
      float v = row[e];
      if ((bits[e >> 5] >> (e & 31)) & 1u) v = 1e6f;
      if (e == o) v = target;
      cnt += (v <= target) ? 1 : 0;
    }
  } else if (mode == RANK_SORT_POSITION) {
    for (int e = tid; e < n_cols; e += blockDim.x) {
      float v = row[e];
      if ((bits[e >> 5] >> (e & 31)) & 1u) v = 0.0f;
      if (e == o) v = target;
      cnt += (v > target) ? 1 : 0;
    }
    if (tid == 0) cnt += 1;
  } else {
    for (int e = tid; e < n_cols; e += blockDim.x) {
      float v = row[e];
      if ((bits[e >> 5] >> (e & 31)) & 1u) v = -1e6f;
      if (mode == RANK_PREDICT_TAILS && e == o) v = target;
      cnt += (v >= target) ? 1 : 0;
    }
  }
  // block reduce
  for (int o2 = 32; o2 > 0; o2 >>= 1) cnt += __shfl_xor(cnt, o2, 64);
  if ((tid & 63) == 0) partial[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += partial[w];
    rank_out[s] = tot;
    target_out[s] = target;
  }
}

void launch_rank_count(kp_ctx* c, int n_slots, const float* d_scores, int ld, int n_cols,
                       const int32_t* d_pred_o, const int32_t* d_filt_off, const int32_t* d_filt,
                       int minimizer, float* d_target, int64_t* d_rank, int mode) {
  if (n_slots <= 0) return;
  size_t shm = (size_t)((n_cols + 31) / 32) * 4;
  KP_REQUIRE(shm <= 150 * 1024, "rank: too many entities for the LDS filter bitmap");
  hipLaunchKernelGGL(kp_rank_count, dim3(n_slots), dim3(256), shm, c->stream, n_slots, d_scores, ld, n_cols,
                     d_pred_o, d_filt_off, d_filt, minimizer, d_target, d_rank, mode);
  KP_HIP(hipGetLastError());
}

// ----------------------------------------------------------------------------
// fp64 filtered rank of a maximizer (ComplEx get_triple_results, post_training_engine.py:
// 101-125).  At the reference's random init the post-trained target sits among dense
// near-ties (scores ~1e-6, nearest neighbour ~1e-11 away), and an fp32 dot product over
// 400 terms with cancellation is off by ~1e-5 relative: enough to move the rank.  The
// reference's fp64 run is the exact version of the same computation, so the device
// scores in fp64 (exact products of the fp32 operands, one fp64 FMA chain over d per
// entity, the same order for the target) and compares in fp64.  No score matrix is
// written: each thread scores one entity for RQ slots and counts against their targets.
// ----------------------------------------------------------------------------
constexpr int RQ = 16;  // slots per workgroup row of the grid

// E^T [dp][ldt] (fp32, zero columns past n_ent), once per context
__global__ void kp_transpose_table(const float* __restrict__ E, int n_ent, int dp, float* __restrict__ ET, int ldt) {
  __shared__ float tile[32][33];
  const int e0 = blockIdx.x * 32, d0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int e = e0 + i, d = d0 + tx;
    tile[i][tx] = (e < n_ent && d < dp) ? E[(size_t)e * dp + d] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int d = d0 + i, e = e0 + tx;
    if (d < dp && e < ldt) ET[(size_t)d * ldt + e] = tile[tx][i];
  }
}

// per slot: the filter bitmap over the n_ent + 1 columns (kelpie last)
__global__ __launch_bounds__(256) void kp_rank_filter_bits(int n_slots, int nwords, const int32_t* __restrict__ filt_off,
                                                           const int32_t* __restrict__ filt, int n_cols,
                                                           uint32_t* __restrict__ bits) {
  const int s = blockIdx.x;
  uint32_t* b = bits + (size_t)s * nwords;
  for (int i = threadIdx.x; i < nwords; i += blockDim.x) b[i] = 0u;
  __syncthreads();
  for (int i = filt_off[s] + threadIdx.x; i < filt_off[s + 1]; i += blockDim.x) {
    const int e = filt[i];
    if (e >= 0 && e < n_cols) atomicOr(&b[e >> 5], 1u << (e & 31));
  }
}

// torch.sigmoid on a float32 logit (conve.py:157): 1 / (1 + exp(-x)) in float32.  It
// reaches 1.0 at x ~ 16.64, so when the target's fp32 score is 1.0 the reference's rank
// counts every saturated entity as a tie, however far apart the logits are; the device
// ranks on fp64 logits and counts those ties explicitly (saturated: the float32 sigmoid
// is 1.0).  Below saturation, equal float32 scores are rounding coincidences of either
// side's logits and are not counted (the full-size fixtures: counting them moved the
// rank deltas out of the reference's own spread).
__device__ __forceinline__ bool sigmoid_f32_saturated(double x) { return 1.0f / (1.0f + expf(-(float)x)) == 1.0f; }
__device__ __forceinline__ float sigmoid_f32(double x) { return 1.0f / (1.0f + expf(-(float)x)); }

// kelpie column and target: one thread per slot (counts the kelpie column, writes the
// fp32 target score)
// act RANK64_DOT: the scores are the fp64 values (ComplEx); RANK64_SIGMOID: the scores
// are sigmoid(logit) and the rank compares the monotone logits, with a saturated target
// (float32 score 1.0) tied by every saturated entity as the reference's fp32 scores tie
// them (ConvE); RANK64_DIST: a
// minimizer whose scores are L2 distances and the rank compares their squares (TransE:
// get_triple_results' minimizer branch, the target counting itself even when filtered);
// RANK64_DIST1: the same minimizer on L1 distances (TransE norm p = 1)
__global__ void kp_rank_f64_kelpie(int n_slots, int n_ent, int nwords, const uint32_t* __restrict__ bits,
                                   const int32_t* __restrict__ pred_o, const double* __restrict__ t64,
                                   const double* __restrict__ kcol64, int act, float* __restrict__ target_out,
                                   unsigned long long* __restrict__ rank) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const bool filtered = (bits[(size_t)s * nwords + (n_ent >> 5)] >> (n_ent & 31)) & 1u;
  if (act == RANK64_DIST || act == RANK64_DIST1)
    rank[s] = (pred_o[s] == n_ent || (!filtered && kcol64[s] <= t64[s])) ? 1ull : 0ull;
  else if (act == RANK64_SIGMOID)
    rank[s] = (!filtered && (kcol64[s] >= t64[s] || (sigmoid_f32_saturated(t64[s]) && sigmoid_f32_saturated(kcol64[s]))))
                  ? 1ull
                  : 0ull;
  else
    rank[s] = (!filtered && kcol64[s] >= t64[s]) ? 1ull : 0ull;
  target_out[s] = act == RANK64_SIGMOID ? sigmoid_f32(t64[s])
                  : act == RANK64_DIST  ? (float)sqrt(t64[s])
                                        : (float)t64[s];  // DOT, DIST1
}

// MODE: RANK64_DOT (dot products, maximizer), RANK64_SIGMOID (dot products = logits, with
// the saturated float32 sigmoid ties), RANK64_DIST (squared L2), RANK64_DIST1 (L1)
template <int MODE>
__global__ __launch_bounds__(256) void kp_rank_f64_count(int n_slots, int n_ent, int dp, const double* __restrict__ Q,
                                                         const double* __restrict__ t64,
                                                         const int32_t* __restrict__ pred_o, const float* __restrict__ ET,
                                                         int ldt, int nwords, const uint32_t* __restrict__ bits,
                                                         unsigned long long* __restrict__ rank) {
  __shared__ int part[4][RQ];
  const int s0 = blockIdx.y * RQ;
  const int e = blockIdx.x * 256 + threadIdx.x;  // < ldt: ET is zero-padded
  const int ns = min(RQ, n_slots - s0);
  double acc[RQ];
#pragma unroll
  for (int j = 0; j < RQ; ++j) acc[j] = 0.0;
  // the slot rows are wave-uniform: scalar loads, one fp64 FMA chain over d per (slot, entity)
  const double* q = Q + (size_t)s0 * dp;
  for (int d = 0; d < dp; ++d) {
    const double v = (double)ET[(size_t)d * ldt + e];
#pragma unroll
    for (int j = 0; j < RQ; ++j)
      if (j < ns) {
        if constexpr (MODE == RANK64_DIST) {
          const double df = q[(size_t)j * dp + d] - v;  // exact: fp32 operands, fp64 difference
          acc[j] = __fma_rn(df, df, acc[j]);
        } else if constexpr (MODE == RANK64_DIST1) {
          acc[j] += fabs(q[(size_t)j * dp + d] - v);
        } else {
          acc[j] = __fma_rn(q[(size_t)j * dp + d], v, acc[j]);
        }
      }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < RQ; ++j) {
    int hit = 0;
    if (j < ns && e < n_ent) {
      const int s = s0 + j;
      const bool filtered = (bits[(size_t)s * nwords + (e >> 5)] >> (e & 31)) & 1u;
      // the target counts itself whatever the rounding of its own score (a maximizer's
      // only if unfiltered: its filtered score is set back after the count)
      if constexpr (MODE == RANK64_DIST || MODE == RANK64_DIST1)
        hit = e == pred_o[s] || (!filtered && acc[j] <= t64[s]);
      else if constexpr (MODE == RANK64_SIGMOID)
        hit = !filtered && (e == pred_o[s] || acc[j] >= t64[s] ||
                            (sigmoid_f32_saturated(t64[s]) && sigmoid_f32_saturated(acc[j])));
      else
        hit = !filtered && (e == pred_o[s] || acc[j] >= t64[s]);
    }
    for (int o = 32; o > 0; o >>= 1) hit += __shfl_xor(hit, o, 64);
    if (lane == 0) part[w][j] = hit;
  }
  __syncthreads();
  if (threadIdx.x < ns) {
    const int j = threadIdx.x;
    const int tot = part[0][j] + part[1][j] + part[2][j] + part[3][j];
    if (tot) atomicAdd(&rank[s0 + j], (unsigned long long)tot);
  }
}

void launch_rank_f64(kp_ctx* c, int n_slots, const double* d_q64, const double* d_t64, const double* d_kcol64,
                     const int32_t* d_pred_o, const int32_t* d_filt_off, const int32_t* d_filt, float* d_target,
                     int64_t* d_rank, int act) {
  if (n_slots <= 0) return;
  const int ldt = (c->n_ent + 255) / 256 * 256;
  if (!c->eT_ready) {
    float* ET = reinterpret_cast<float*>(c->eT.ensure(sizeof(float) * (size_t)c->dp * ldt));
    hipLaunchKernelGGL(kp_transpose_table, dim3(ldt / 32, (c->dp + 31) / 32), dim3(256), 0, c->stream, c->dE,
                       c->n_ent, c->dp, ET, ldt);
    KP_HIP(hipGetLastError());
    c->eT_ready = true;
  }
  const int n_cols = c->n_ent + 1;
  const int nwords = (n_cols + 31) / 32;
  uint32_t* bits = reinterpret_cast<uint32_t*>(c->ws[28].ensure(sizeof(uint32_t) * (size_t)n_slots * nwords));
  unsigned long long* rank = reinterpret_cast<unsigned long long*>(d_rank);
  hipLaunchKernelGGL(kp_rank_filter_bits, dim3(n_slots), dim3(256), 0, c->stream, n_slots, nwords, d_filt_off, d_filt,
                     n_cols, bits);
  KP_HIP(hipGetLastError());
  hipLaunchKernelGGL(kp_rank_f64_kelpie, dim3((n_slots + 63) / 64), dim3(64), 0, c->stream, n_slots, c->n_ent, nwords,
                     bits, d_pred_o, d_t64, d_kcol64, act, d_target, rank);
  KP_HIP(hipGetLastError());
  const dim3 grid(ldt / 256, (n_slots + RQ - 1) / RQ);
  if (act == RANK64_DIST)
    hipLaunchKernelGGL(kp_rank_f64_count<RANK64_DIST>, grid, dim3(256), 0, c->stream, n_slots, c->n_ent, c->dp, d_q64,
                       d_t64, d_pred_o, c->eT.as<float>(), ldt, nwords, bits, rank);
  else if (act == RANK64_DIST1)
    hipLaunchKernelGGL(kp_rank_f64_count<RANK64_DIST1>, grid, dim3(256), 0, c->stream, n_slots, c->n_ent, c->dp, d_q64,
                       d_t64, d_pred_o, c->eT.as<float>(), ldt, nwords, bits, rank);
  else if (act == RANK64_SIGMOID)
    hipLaunchKernelGGL(kp_rank_f64_count<RANK64_SIGMOID>, grid, dim3(256), 0, c->stream, n_slots, c->n_ent, c->dp,
                       d_q64, d_t64, d_pred_o, c->eT.as<float>(), ldt, nwords, bits, rank);
  else
    hipLaunchKernelGGL(kp_rank_f64_count<RANK64_DOT>, grid, dim3(256), 0, c->stream, n_slots, c->n_ent, c->dp, d_q64,
                       d_t64, d_pred_o, c->eT.as<float>(), ldt, nwords, bits, rank);
  KP_HIP(hipGetLastError());
}

void launch_gemm_abt(kp_ctx* c, const float* A, int lda, int M, const float* B, int ldb, int N, int K, float* out,
                     int ldo, const float* bias, int act, int ksplit) {
  if (M <= 0 || N <= 0) return;
  KP_REQUIRE(K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0, "gemm: K and leading dims must be multiples of 4");
  dim3 grid((N + SG_BN - 1) / SG_BN, (M + SG_BM - 1) / SG_BM, std::max(1, ksplit));
  hipLaunchKernelGGL(kp_gemm_abt, grid, dim3(256), 0, c->stream, A, lda, M, B, ldb, N, 0, K, out, ldo, bias, act);
  KP_HIP(hipGetLastError());
}

void launch_score_gemm(kp_ctx* c, const float* dQ, int nq, float* d_out, int ld, int act) {
  launch_gemm_abt(c, dQ, c->dp, nq, c->dE, c->dp, c->n_ent, c->dp, d_out, ld, nullptr, act, 1);
}

// ----------------------------------------------------------------------------
// conversion-entity test of RelevanceEngine.select_entities_to_convert
// (engine.py:103-120), one workgroup per candidate head: keep iff the target's
// raw score lies strictly inside (-1e6, max of the filter-masked row) for
// maximizers, or inside (min, 1e6) for minimizers.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void kp_convertible_reduce(int n, const float* __restrict__ scores, int ld,
                                                             int n_ent, int obj,
                                                             const int32_t* __restrict__ filt_off,
                                                             const int32_t* __restrict__ filt, int minimizer,
                                                             uint8_t* __restrict__ keep) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
  __shared__ float part[4];
  const int i = blockIdx.x;
  const int tid = threadIdx.x;
  const int nwords = (n_ent + 31) >> 5;
  for (int k = tid; k < nwords; k += blockDim.x) bits[k] = 0u;
  __syncthreads();
  for (int k = filt_off[i] + tid; k < filt_off[i + 1]; k += blockDim.x) {
    int e = filt[k];
    if (e >= 0 && e < n_ent) atomicOr(&bits[e >> 5], 1u << (e & 31));
  }
  __syncthreads();
  const float* row = scores + (size_t)i * ld;
  const float t = row[obj];
  float ext = minimizer ? 3.0e38f : -3.0e38f;
  for (int e = tid; e < n_ent; e += blockDim.x) {
    float v = row[e];
    if ((bits[e >> 5] >> (e & 31)) & 1u) v = minimizer ? 1e6f : -1e6f;
    ext = minimizer ? fminf(ext, v) : fmaxf(ext, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    float other = __shfl_xor(ext, o, 64);
    ext = minimizer ? fminf(ext, other) : fmaxf(ext, other);
  }
  if ((tid & 63) == 0) part[tid >> 6] = ext;
  __syncthreads();
  if (tid == 0) {
    float e2 = part[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) e2 = minimizer ? fminf(e2, part[w]) : fmaxf(e2, part[w]);
    keep[i] = minimizer ? ((1e6f > t && t > e2) ? 1 : 0) : ((-1e6f < t && t < e2) ? 1 : 0);
  }
}

void launch_convertible_reduce(kp_ctx* c, int n, const float* d_scores, int ld, int obj, const int32_t* d_fo,
                               const int32_t* d_f, int minimizer, uint8_t* d_keep) {
  if (n <= 0) return;
  size_t shm = (size_t)((c->n_ent + 31) / 32) * 4;
  KP_REQUIRE(shm <= 150 * 1024, "convertible: too many entities for the LDS filter bitmap");
  hipLaunchKernelGGL(kp_convertible_reduce, dim3(n), dim3(256), shm, c->stream, n, d_scores, ld, c->n_ent, obj, d_fo,
                     d_f, minimizer, d_keep);
  KP_HIP(hipGetLastError());
}
