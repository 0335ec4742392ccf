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
//   f = ||lhs + rel - rhs||_p (p = 2, or 1: transe.py:46, tune.py:19),
//   L2 = (mean lhs^2 + mean rel^2 + mean rhs^2) / 3;
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
#include <cstdlib>

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

// component-wise select: a ternary on float4 aggregates can be lowered to a select of
// addresses, which sends both operands through scratch memory
__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
  return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

#ifdef KP_TE_STAMPS
// diagnostic build only (make stamps): per workgroup [slot, R, start, end] in wall_clock64 ticks (100 MHz),
// then s_memtime cycles [wave 0 fetch + load wait, wave 0 compute, sum over steps of the slowest wave's
// item loop, sum over steps of the whole step (wave 0)]
__device__ long long g_te_times[8 * 8192];
#endif

constexpr int TE_NB = 5;  // negatives per bundle held in registers (the reference's ratio; larger ratios loop)

// sum over the 64 lanes of 16-lane sums (row16_sum), returned wave-uniform: row_bcast15 /
// row_bcast31 fold the four rows into lane 63
// 16-lane row sums as DPP adds: bound_ctrl set (every source lane of these patterns is
// inside its row, so it changes nothing) lets the compiler fuse each move into the add
__device__ __forceinline__ float row16_sum_f(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  return v;
}

__device__ __forceinline__ float wave_fold_u(float v) {  // v: 16-lane sums (row16_sum)
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

constexpr int TE_RCH = 512;  // work-item records built in LDS per chunk

// Work-item record (three int4 in LDS), built by all threads once per step so that the
// per-item loop is loads + arithmetic only (wave-uniform fields read with broadcast LDS
// reads and readfirstlane; no index arithmetic, divisions or 64-bit multiplies):
//   r0 = {element offset of the positive's frozen side (0 if it is the kelpie id K),
//         element offset of the relation row, flags, #K occurrences over the item's pairs}
//   r1 = {element offsets of negatives 0..3}, r2 = {offset of negative 4, sign bits, -, -}
// flags: bit 0 h == K, bit 1 t == K, bits 4-7 #negatives, bits 8+q corrupted head,
// bits 16+q negative entity == K; sign bits: 2 bits per negative, sgn + 1 with
// sgn = (hn == K) - (tn == K) (TransE)
__device__ __forceinline__ void te_record(int4* rec, int it, int cpb, int mb, int ratio, int st, int B,
                                          const int32_t* order, const int32_t* ents, const int32_t* hot,
                                          const int32_t* rw, int dp, int K) {
  const int m = mb + it / cpb, c = it - (it / cpb) * cpb;
  const int ri = order[m];
  const int h = rw[3 * ri], r = rw[3 * ri + 1], t = rw[3 * ri + 2];
  const int fz = (h == K) ? t : h;
  const int j0 = max(m * ratio, st) + c * TE_NB;
  const int jhi = min(m * ratio + ratio, st + B);
  const int nb = max(0, min(TE_NB, jhi - j0));
  int flags = (h == K ? 1 : 0) | (t == K ? 2 : 0) | (nb << 4);
  int sgn = 0, cnt = 0;
  int off[TE_NB];
#pragma unroll
  for (int q = 0; q < TE_NB; ++q) {
    const int jj = min(j0 + q, jhi - 1);
    const int ent = ents[jj];
    const bool ch = hot[jj] == 1;
    off[q] = (ent == K ? 0 : ent) * dp;
    const int hn = ch ? ent : h, tn = ch ? t : ent;
    if (q < nb) {
      flags |= (ch ? 1 << (8 + q) : 0) | (ent == K ? 1 << (16 + q) : 0);
      sgn |= ((hn == K) - (tn == K) + 1) << (2 * q);
      cnt += (h == K) + (t == K) + (hn == K) + (tn == K);
    } else {
      sgn |= 1 << (2 * q);
    }
  }
  rec[0] = make_int4((fz == K ? 0 : fz) * dp, r * dp, flags, cnt);
  rec[1] = make_int4(off[0], off[1], off[2], off[3]);
  rec[2] = make_int4(off[4], sgn, 0, 0);
}

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// One item: the positive and its negatives.  x4[u] is this lane's float4 of the kelpie
// row (constant within a step), fo[u] its element offset clamped into the row, on[u]
// whether that float4 is inside the row (out-of-row lanes load duplicates and are
// dropped from the norms; their gradient lanes are never stored).  The kernel is
// bound by VALU issue (tools/te_times.py): the selects below are per-lane with
// wave-uniform masks; forcing them into scalar branches was measured 1.9x slower.
__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// L1 (norm p = 1): f = sum |v| and d f / d v = sgn(v) with sgn(0) = 0 (torch's p = 1 norm
// backward); the per-pair coefficient is then +-1 instead of +-1 / f
template <int VPL, bool L1>
__device__ __forceinline__ void te_item(const int4* rec, const float* __restrict__ E, const float* __restrict__ Rt,
                                        const float4* x4, const int* fo, const bool* on, float margin, float4* g,
                                        int& cnt) {
  const int4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
  const int a_off = rfl(r0.x), rel_off = rfl(r0.y), flags = rfl(r0.z);
  const int noff[TE_NB] = {rfl(r1.x), rfl(r1.y), rfl(r1.z), rfl(r1.w), rfl(r2.x)};
  const int sgnb = rfl(r2.y);
  const int nb = (flags >> 4) & 15;
  const bool hk = flags & 1, tk = flags & 2;
  float4 av[VPL], bb[VPL], bn[TE_NB][VPL];
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    av[u] = ld4(E + a_off + fo[u]);
    bb[u] = ld4(Rt + rel_off + fo[u]);
#pragma unroll
    for (int q = 0; q < TE_NB; ++q) bn[q][u] = ld4(E + noff[q] + fo[u]);
  }
  float4 rp[VPL], lb[VPL], vp[VPL];
  float sp = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    // every kelpie row holds K on one side (both for a self loop)
    const float4 lp = hk ? x4[u] : av[u];
    rp[u] = tk ? x4[u] : av[u];
    const float4 b = bb[u];
    lb[u] = make_float4(lp.x + b.x, lp.y + b.y, lp.z + b.z, lp.w + b.w);
    vp[u] = make_float4(lb[u].x - rp[u].x, lb[u].y - rp[u].y, lb[u].z - rp[u].z, lb[u].w - rp[u].w);
    const float s = L1 ? (fabsf(vp[u].x) + fabsf(vp[u].y)) + (fabsf(vp[u].z) + fabsf(vp[u].w))
                       : fmaf(vp[u].x, vp[u].x, fmaf(vp[u].y, vp[u].y, fmaf(vp[u].z, vp[u].z, vp[u].w * vp[u].w)));
    sp += on[u] ? s : 0.f;
  }
  float4 vn[TE_NB][VPL];
  float sn[TE_NB];
#pragma unroll
  for (int q = 0; q < TE_NB; ++q) {
    sn[q] = 0.f;
    const bool ch = flags & (1 << (8 + q));
    const bool ek = flags & (1 << (16 + q));
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const float4 bq = ek ? x4[u] : bn[q][u];
      const float4 b = bb[u];
      float4 v;
      if (ch)  // corrupted head: (e_n + rel) - rhs
        v = make_float4((bq.x + b.x) - rp[u].x, (bq.y + b.y) - rp[u].y, (bq.z + b.z) - rp[u].z, (bq.w + b.w) - rp[u].w);
      else  // corrupted tail: (lhs + rel) - e_n
        v = make_float4(lb[u].x - bq.x, lb[u].y - bq.y, lb[u].z - bq.z, lb[u].w - bq.w);
      const float s = L1 ? (fabsf(v.x) + fabsf(v.y)) + (fabsf(v.z) + fabsf(v.w))
                         : fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w)));
      vn[q][u] = L1 ? make_float4(sgnf(v.x), sgnf(v.y), sgnf(v.z), sgnf(v.w)) : v;
      sn[q] += on[u] ? s : 0.f;
    }
  }
  // TE_NB + 1 independent wave reductions, interleaved
  sp = row16_sum_f(sp);
#pragma unroll
  for (int q = 0; q < TE_NB; ++q) sn[q] = row16_sum_f(sn[q]);
  const float fp = L1 ? wave_fold_u(sp) : sqrtf(wave_fold_u(sp));
  int n_act = 0;
#pragma unroll
  for (int q = 0; q < TE_NB; ++q) {
    const float fn = L1 ? wave_fold_u(sn[q]) : sqrtf(wave_fold_u(sn[q]));
    if (q >= nb) continue;
    const bool act = (fp - fn) + margin >= 0.f;  // clamp_min backward passes grad where self >= min
    n_act += act ? 1 : 0;
    const int sgn_n = ((sgnb >> (2 * q)) & 3) - 1;
    if (act && sgn_n != 0 && fn > 0.f) {  // negatives without the kelpie entity: hinge only
      const float cn = L1 ? -(float)sgn_n : -(float)sgn_n / fn;
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        g[u].x = fmaf(cn, vn[q][u].x, g[u].x);
        g[u].y = fmaf(cn, vn[q][u].y, g[u].y);
        g[u].z = fmaf(cn, vn[q][u].z, g[u].z);
        g[u].w = fmaf(cn, vn[q][u].w, g[u].w);
      }
    }
  }
  const int sgn_p = (hk ? 1 : 0) - (tk ? 1 : 0);
  if (n_act > 0 && sgn_p != 0 && fp > 0.f) {
    const float cps = L1 ? (float)(n_act * sgn_p) : (float)n_act * ((float)sgn_p / fp);
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const float4 w = L1 ? make_float4(sgnf(vp[u].x), sgnf(vp[u].y), sgnf(vp[u].z), sgnf(vp[u].w)) : vp[u];
      g[u].x = fmaf(cps, w.x, g[u].x);
      g[u].y = fmaf(cps, w.y, g[u].y);
      g[u].z = fmaf(cps, w.z, g[u].z);
      g[u].w = fmaf(cps, w.w, g[u].w);
    }
  }
  cnt += rfl(r0.w);
}

// One workgroup per slot (slots issued longest first) runs every epoch on chip: x in
// LDS, its Adam moments in registers.
//
// Work unit = one wave-uniform *bundle*: the stepped positions j = m*ratio .. m*ratio +
// ratio - 1 share the positive row order[m] (np.repeat of the shuffled rows, A-Q2), so
// a wave loads the positive's frozen side (h or t; the other is the kelpie row x) and
// the relation ONCE, plus one fresh entity row per negative (a negative keeps the
// positive's uncorrupted side).  Descriptors are wave-uniform scalar loads; rows are
// float4 per lane (64 lanes per row).  The kelpie id K in any position selects x
// (loads stay branch-free: K reads row 0).  Squared norms are wave reductions; the
// single-row gradient (TransE) accumulates in registers; per step the
// 16 wave partials are summed in a fixed order in LDS and Adam updates x.
//
// Cost model: per stepped pair one fresh 4*d-byte negative row; the
// positive side and relation once per bundle.  A slot's epochs are one dependent chain,
// so its time is the latency of that chain: the slot's rows are staged in LDS once and
// each epoch's draws are loaded into registers during the previous epoch and stored to
// the other half of a double buffer in LDS (they do not depend on x), which leaves one
// row-gather round per bundle, two barriers and the Adam step per epoch.  NT = 1024
// threads per workgroup (1024: one per CU; 512 for diagnostics).
// STAGED = false (slots too long for the LDS buffers) reads the descriptors from memory.
template <int VPL, int NT, bool STAGED, bool L1>  // VPL float4 per lane: dp <= 256 * VPL
__global__ __launch_bounds__(NT) void kp_te_posttrain(int n_ent, int dp, int d, const float* __restrict__ E,
                                                          const float* __restrict__ Rt,
                                                          const TeSlot* __restrict__ slots,
                                                          const int32_t* __restrict__ slot_of_block,
                                                          const int32_t* __restrict__ rows,
                                                          const int32_t* __restrict__ rng, TeHp hp,
                                                          float* __restrict__ X) {
  constexpr int TE_NW = NT / 64;  // waves
  constexpr int PF = 4;           // prefetched draw words per thread (STAGED: 3 R <= PF * NT)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;        // [dp]
  float* red = sm + dp;  // [TE_NW][dp] per-wave gradient partials
  int* rws = reinterpret_cast<int*>(red + TE_NW * dp);  // STAGED: [3 R] the slot's rows
  int* drw = rws + 3 * (STAGED ? slots[slot_of_block[blockIdx.x]].R : 0);  // STAGED: [2][3 R] draws
  __shared__ int4 recs[3 * TE_RCH];  // work-item records of the current chunk
  __shared__ int cnt_s[TE_NW];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int slot = slot_of_block[blockIdx.x];
  const TeSlot S = slots[slot];
  const int K = n_ent;
  float* x = X + (size_t)slot * dp;
#ifdef KP_TE_STAMPS
  const long long t_start = wall_clock64();
  long long st_fetch = 0, st_comp = 0, st_red = 0, st_items = 0;
  __shared__ unsigned long long loop_max_s;
  if (tid == 0) loop_max_s = 0;
#endif
  for (int i = tid; i < dp; i += NT) xs[i] = x[i];
  float m1 = 0.f, v2 = 0.f;  // Adam moments of element tid (tid < dp)
  const int32_t* rwg = rows + 3 * (size_t)S.row_off;
  const int32_t* rngs = rng + S.rng_off;
  const int R3 = 3 * S.R;
  int pf[PF];
  if (STAGED) {
    for (int i = tid; i < R3; i += NT) {
      rws[i] = rwg[i];
      if (hp.epochs > 0) drw[i] = rngs[i];
    }
  }
  __syncthreads();
  const int32_t* rw = STAGED ? rws : rwg;
  const int NF4 = dp / 4;
  const int ratio = hp.ratio;
  int fo[VPL];
  bool on[VPL];
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int f = lane + 64 * u;
    on[u] = f < NF4;
    fo[u] = 4 * (f < NF4 ? f : NF4 - 1);
  }
  double b1t = 1.0, b2t = 1.0;
  for (int e = 0; e < hp.epochs; ++e) {
    const int32_t* order = STAGED ? drw + (e & 1) * R3 : rngs + (long long)e * R3;
    const int32_t* ents = order + S.R;
    const int32_t* hot = order + 2 * S.R;
    if (STAGED && e + 1 < hp.epochs) {  // next epoch's draws, landed during this epoch
      const int32_t* nx = rngs + (long long)(e + 1) * R3;
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int i = tid + k * NT;
        pf[k] = i < R3 ? nx[i] : 0;
      }
    }
    for (int st = 0; st < S.R; st += hp.bs) {
      const int B = min(hp.bs, S.R - st);
      float4 g[VPL];
#pragma unroll
      for (int u = 0; u < VPL; ++u) g[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      int cnt = 0;
      // work items: (bundle m, chunk of <= TE_NB of its negatives) over the bundles that
      // overlap the step's positions [st, st + B); records built per chunk of TE_RCH items
      const int cpb = (ratio + TE_NB - 1) / TE_NB;
      const int mb = st / ratio;
      const int n_items = ((st + B - 1) / ratio - mb + 1) * cpb;
#ifdef KP_TE_STAMPS
      const long long c_step = __builtin_amdgcn_s_memtime();
#endif
      float4 x4[VPL];
#pragma unroll
      for (int u = 0; u < VPL; ++u) x4[u] = ld4(xs + fo[u]);
      for (int c0 = 0; c0 < n_items; c0 += TE_RCH) {
        const int nc = min(TE_RCH, n_items - c0);
        if (c0 > 0) __syncthreads();  // the previous chunk's records are consumed
        for (int k = tid; k < nc; k += NT)
          te_record(recs + 3 * k, c0 + k, cpb, mb, ratio, st, B, order, ents, hot, rw, dp, K);
        __syncthreads();
        for (int k = wave; k < nc; k += TE_NW) {
#ifdef KP_TE_STAMPS
          const long long c1 = __builtin_amdgcn_s_memtime();
#endif
          te_item<VPL, L1>(recs + 3 * k, E, Rt, x4, fo, on, hp.margin, g, cnt);
#ifdef KP_TE_STAMPS
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          st_comp += __builtin_amdgcn_s_memtime() - c1;
#endif
        }
      }
#ifdef KP_TE_STAMPS
      const long long c3 = __builtin_amdgcn_s_memtime();
      if (lane == 0) atomicMax(&loop_max_s, (unsigned long long)(c3 - c_step));
#endif
      if (STAGED && e + 1 < hp.epochs && st + hp.bs >= S.R) {  // last step of the epoch
        int* nb_ = drw + ((e + 1) & 1) * R3;
#pragma unroll
        for (int k = 0; k < PF; ++k) {
          const int i = tid + k * NT;
          if (i < R3) nb_[i] = pf[k];
        }
      }
      // ---- sum the wave partials in a fixed order, then Adam on x
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        const int f = lane + 64 * u;
        if (f < NF4) *reinterpret_cast<float4*>(red + wave * dp + 4 * f) = g[u];
      }
      if (lane == 0) cnt_s[wave] = cnt;
      __syncthreads();
      b1t *= (double)hp.b1;
      b2t *= (double)hp.b2;
      if (tid < dp) {
        int ctot = 0;
        for (int k = 0; k < TE_NW; ++k) ctot += cnt_s[k];
        const float invB = 1.0f / (float)B;
        const float regc = hp.lam / (3.0f * (float)B * (float)d) * (float)ctot;
        const float step_size = (float)((double)hp.lr / (1.0 - b1t));
        const float bc2s = (float)sqrt(1.0 - b2t);
        float gs = 0.f;
        for (int k = 0; k < TE_NW; ++k) gs += red[k * dp + tid];
        const float xi = xs[tid];
        const float gi = gs * invB + regc * xi;
        m1 = m1 + hp.one_minus_b1 * (gi - m1);
        v2 = v2 * hp.b2;
        v2 = v2 + (hp.one_minus_b2 * gi) * gi;
        const float den = sqrtf(v2) / bc2s + hp.eps;
        xs[tid] = (tid < d) ? xi + (-step_size * m1) / den : 0.f;
      }
      __syncthreads();
#ifdef KP_TE_STAMPS
      st_red += __builtin_amdgcn_s_memtime() - c_step;
      st_items += (long long)loop_max_s;
      __syncthreads();
      if (tid == 0) loop_max_s = 0;
#endif
    }
  }
  for (int i = tid; i < dp; i += NT) x[i] = xs[i];
#ifdef KP_TE_STAMPS
  if (tid == 0 && blockIdx.x < 8192) {
    long long* o = g_te_times + 8 * blockIdx.x;
    o[0] = slot;
    o[1] = S.R;
    o[2] = t_start;
    o[3] = wall_clock64();
    o[4] = st_fetch;
    o[5] = st_comp;
    o[6] = st_red;
    o[7] = st_items;
  }
#endif
}

// scores[q][e] = || (lhs_q + rel_q) - E_e ||_p for e < n_ent (transe.py:48-65), p = 2
// or 1 (l1); lhs_q is a frozen row (heads[q] >= 0) or the slot's kelpie row X[q].
#define TS_Q 8
__global__ __launch_bounds__(256) void kp_te_scores(int n_ent, int dp, const float* __restrict__ E,
                                                    const float* __restrict__ R, int nq,
                                                    const int32_t* __restrict__ heads,
                                                    const int32_t* __restrict__ rels,
                                                    const float* __restrict__ X, float* __restrict__ out, int ld,
                                                    int kcol, int l1) {
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
        acc[q] += l1 ? (fabsf(a) + fabsf(b)) + (fabsf(c) + fabsf(w)) : a * a + b * b + c * c + w * w;
      }
    }
#pragma unroll
    for (int q = 0; q < TS_Q; ++q)
      if (q0 + q < nq) out[(size_t)(q0 + q) * ld + e] = l1 ? acc[q] : sqrtf(acc[q]);
  }
  // kelpie column: || (x + r) - x ||
  if (kcol >= 0 && blockIdx.x == 0 && threadIdx.x < TS_Q) {
    const int q = q0 + threadIdx.x;
    if (q < nq) {
      float acc = 0.f;
      for (int k = 0; k < dp; ++k) {
        const float dlt = tq[threadIdx.x * dp + k] - X[(size_t)q * dp + k];
        acc += l1 ? fabsf(dlt) : dlt * dlt;
      }
      out[(size_t)q * ld + kcol] = l1 ? acc : sqrtf(acc);
    }
  }
}

void launch_te_scores(kp_ctx* c, int nq, const int32_t* dh, const int32_t* dr, const float* dX, float* dOut, int ld,
                      int kcol) {
  if (nq <= 0) return;
  dim3 grid((c->n_ent + 255) / 256, (nq + TS_Q - 1) / TS_Q);
  const size_t shm = sizeof(float) * TS_Q * c->dp;
  hipLaunchKernelGGL(kp_te_scores, grid, dim3(256), shm, c->stream, c->n_ent, c->dp, c->dE, c->dR, nq, dh, dr, dX,
                     dOut, ld, kcol, c->te_norm == 1 ? 1 : 0);
  KP_HIP(hipGetLastError());
}

// fp64 ranking queries (launch_rank_f64, RANK64_DIST / RANK64_DIST1): the translation
// q = x + R_p of the post-trained row in fp64 (exact: two fp32 operands), its squared
// distance (L1: its |.| sum) to the target and to the kelpie row as one sequential fp64
// chain over d, the order
// kp_rank_f64_count scores every entity in.  An fp32 norm over 200 terms is ~1e-7
// relative off, enough to swap near-tied entities (FB15k-237 necessary fixtures).
__global__ void kp_te_rankq64(const float* __restrict__ X, const float* __restrict__ R,
                              const float* __restrict__ E, int n_ent, int dp, const int32_t* __restrict__ pred,
                              int n_slots, double* __restrict__ Q, double* __restrict__ t64,
                              double* __restrict__ kcol64, int l1) {
  const int s = blockIdx.x;
  if (s >= n_slots) return;
  const float* x = X + (size_t)s * dp;
  const float* r = R + (size_t)pred[3 * s + 1] * dp;
  double* q = Q + (size_t)s * dp;
  for (int d = threadIdx.x; d < dp; d += blockDim.x) q[d] = (double)x[d] + (double)r[d];
  __syncthreads();
  if (threadIdx.x == 0) {
    const int o = pred[3 * s + 2];
    double z = 0.0, t = 0.0;
    for (int d = 0; d < dp; ++d) {
      const double df = q[d] - (double)x[d];
      z = l1 ? z + fabs(df) : __fma_rn(df, df, z);
    }
    if (o < n_ent) {
      const float* eo = E + (size_t)o * dp;
      for (int d = 0; d < dp; ++d) {
        const double df = q[d] - (double)eo[d];
        t = l1 ? t + fabs(df) : __fma_rn(df, df, t);
      }
    } else {
      t = z;  // the kelpie entity is its own object
    }
    kcol64[s] = z;
    t64[s] = t;
  }
}

}  // namespace

void transe_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* bt) {
  const int ns = bt->n_slots;
  const int DP = c->dp;
  const bool l1 = c->te_norm == 1;
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

  // longest slots first: a slot's epochs are one dependent chain on one CU
  std::vector<int32_t> order(ns);
  for (int s = 0; s < ns; ++s) order[s] = s;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return slots[a].R > slots[b].R; });
  int32_t* dOrder = upload(c, c->ws[12], order.data(), order.size());
  KP_REQUIRE(DP <= 512, "TransE: dimension > 512 not supported");
  int max_r = 0;
  for (int s = 0; s < ns; ++s) max_r = std::max(max_r, slots[s].R);
  // one 1024-thread workgroup per CU: a long slot is bound by the row gathers one CU keeps
  // in flight (measured: 18.6 us per epoch at R 200-400 vs 23.6 with two 512-thread
  // workgroups per CU sharing it, tools/te_times.py); short slots queue behind
  int nt = DP > 256 ? 512 : 1024;  // two float4 per lane need > 128 VGPRs: 8 waves per workgroup
  if (const char* env = std::getenv("KELPIE_TE_NT")) nt = std::atoi(env) == 1024 ? 1024 : 512;  // diagnostics
  const bool staged = 3 * max_r <= 4 * nt && (size_t)9 * max_r * sizeof(int) <= 48 * 1024;
  const int nw = nt / 64;
  const size_t shm = sizeof(float) * (size_t)(1 + nw) * DP + (staged ? sizeof(int) * (size_t)9 * max_r : 0);

  KP_HIP(hipEventRecord(c->ev0, c->stream));
  hipEvent_t ea = c->event(0), eb = c->event(1);
  KP_HIP(hipEventRecord(ea, c->stream));
  const int vpl = (DP + 255) / 256;
#define TE_LAUNCH(V, T, ST, L)                                                                                   \
  hipLaunchKernelGGL((kp_te_posttrain<V, T, ST, L>), dim3(ns), dim3(T), shm, c->stream, c->n_ent, DP, c->dim, c->dE, \
                     c->dR, dSlots, dOrder, dRows, dRng, h, dX)
#define TE_NORM(V, T, ST)     \
  if (l1)                     \
    TE_LAUNCH(V, T, ST, true); \
  else                        \
    TE_LAUNCH(V, T, ST, false)
#define TE_STAGE(V, T)      \
  if (staged) {             \
    TE_NORM(V, T, true);    \
  } else {                  \
    TE_NORM(V, T, false);   \
  }
  if (vpl == 1) {
    if (nt == 1024) {
      TE_STAGE(1, 1024);
    } else {
      TE_STAGE(1, 512);
    }
  } else {
    TE_STAGE(2, 512);
  }
#undef TE_STAGE
#undef TE_NORM
#undef TE_LAUNCH
  KP_HIP(hipGetLastError());
  KP_HIP(hipEventRecord(eb, c->stream));

  // ---- rank: scores of (kelpie, p, .) = ||(x + R_p) - E_e||_p, minimizer
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
  float* dTarget = reinterpret_cast<float*>(c->ws[10].ensure(sizeof(float) * ns));
  int64_t* dRank = reinterpret_cast<int64_t*>(c->ws[11].ensure(sizeof(int64_t) * ns));
  if (c->te_rank64) {
    int32_t* dPred = upload(c, c->ws[13], bt->pred, (size_t)ns * 3);
    double* dQ64 = reinterpret_cast<double*>(c->ws[29].ensure(sizeof(double) * (size_t)ns * DP));
    double* dT64 = reinterpret_cast<double*>(c->ws[30].ensure(sizeof(double) * 2 * (size_t)ns));
    hipLaunchKernelGGL(kp_te_rankq64, dim3(ns), dim3(64), 0, c->stream, dX, c->dR, c->dE, c->n_ent, DP, dPred, ns,
                       dQ64, dT64, dT64 + ns, l1 ? 1 : 0);
    KP_HIP(hipGetLastError());
    launch_rank_f64(c, ns, dQ64, dT64, dT64 + ns, dPo, dFo, dF, dTarget, dRank, l1 ? RANK64_DIST1 : RANK64_DIST);
  } else {
    float* dScores = reinterpret_cast<float*>(c->ws[9].ensure(sizeof(float) * (size_t)ns * ld));
    launch_te_scores(c, ns, dH, dRl, dX, dScores, ld, c->n_ent);
    launch_rank_count(c, ns, dScores, ld, c->n_ent + 1, dPo, dFo, dF, 1, dTarget, dRank);
  }
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
  c->hot_iv.clear();
  kp_push_interval(c, ea, eb);
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
extern "C" int kp_debug_te_times(long long* out, int n) {
  KP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_te_times), sizeof(long long) * 8 * (size_t)std::min(n, 8192)));
  return 0;
}
#endif
