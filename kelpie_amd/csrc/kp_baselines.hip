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
//     workspace, blocked by 32-column panels held in LDS (float64 VALU; D^3/3
//     multiply-adds).
#include <cmath>
#include <utility>

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
// with b = z_t as column Dp of the workspace (Dp = D rounded up to CR_NB, the system
// bordered by an identity block, b by zeros; row stride ld = Dp + 1); right-looking blocked
// Gaussian elimination with partial pivoting, out = z_p . ((1 - sig) y).  The border never
// pivots into the first D columns (its entries there are 0, a tie with 0 means singular)
// and its multipliers are 0, so the first D unknowns are those of the D x D system.
//   row swaps exchange entries of a logical -> workspace row map in LDS, no data moves;
//   per panel of CR_NB columns: the panel rows k0..Dp in registers, one row per thread,
//   factorised there (pivot = first row of maximal |a| (idamax) by a DPP wave argmax and
//   one barrier per column over the waves' best rows in LDS; multipliers; rank-1 update,
//   whose first column is the next pivot search's input), then L to LDS;
//   U12 = L11^-1 A12 over the trailing columns and b (one column per thread, its 32 loads
//   issued together), then A22 -= L21 U12 (8 rows x 64 columns per wave item, loads first,
//   L21 broadcast from LDS);
//   back substitution by CR_NB-row blocks staged in LDS: the block's rows on one wave
//   (shuffles), then every row above it updated by the block's y.
// Every element sees the operations of the unblocked column-by-column elimination in the
// same order (row swaps travel with the multipliers; subtractions in pivot order;
// -ffp-contract=off), so the result equals it bit for bit; the blocking only removes the
// per-column barriers and L2 round trips of the trailing matrix.
// one DPP step of a wave argmax over (|a|, row): the larger value, the smaller row on ties
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void argmax_dpp(double& v, int& vi) {
  const long long b = __double_as_longlong(v);
  const int lo = (int)b, hi = (int)(b >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xF, false);
  const int oi = __builtin_amdgcn_update_dpp(vi, vi, CTRL, ROW_MASK, 0xF, false);
  const double ov = __longlong_as_double(((long long)ohi << 32) | (unsigned)olo);
  if (ov > v || (ov == v && oi < vi)) {
    v = ov;
    vi = oi;
  }
}

// wave argmax: quad xor 1 and 2, row rotations by 4 and 8, then row_bcast15 / row_bcast31
// fold the four rows into lane 63, read back uniformly
__device__ __forceinline__ void wave_argmax(double& v, int& vi) {
  argmax_dpp<0xB1, 0xF>(v, vi);
  argmax_dpp<0x4E, 0xF>(v, vi);
  argmax_dpp<0x124, 0xF>(v, vi);
  argmax_dpp<0x128, 0xF>(v, vi);
  argmax_dpp<0x142, 0xA>(v, vi);
  argmax_dpp<0x143, 0xC>(v, vi);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  v = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  vi = __builtin_amdgcn_readlane(vi, 63);
}

// f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N - 1>): a loop whose
// index is a compile-time constant in every copy (register arrays stay in registers)
template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int CR_NB = 32;
constexpr int CR_PS = CR_NB + 1;  // panel row stride (doubles): odd, row-per-lane access is conflict-free
#ifndef KP_CR_T
#define KP_CR_T 512
#endif
#ifndef KP_CR_ROWS
#define KP_CR_ROWS 8
#endif
#ifndef KP_CR_SEG
#define KP_CR_SEG 32
#endif
constexpr int CR_T = KP_CR_T;      // threads per workgroup (one panel row / one trailing column each)
constexpr int CR_R = KP_CR_ROWS;   // rows per trailing-update chunk
constexpr int CR_SEG = KP_CR_SEG;  // rows per trailing-update item
// diagnostic: per-phase s_memtime totals of workgroup 0, printed at its end (KP_CR_STAMPS,
// diagnostic builds only)
#ifdef KP_CR_STAMPS
#ifndef KP_DIAGNOSTIC_BUILD
#error "KP_CR_STAMPS is a diagnostic define: build it with tools/build_variant.sh -DKP_DIAGNOSTIC_BUILD"
#endif
#define CR_ST(k)                                                 \
  do {                                                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_last;                                   \
    st_last = t_;                                                \
  } while (0)
#else
#define CR_ST(k) (void)0
#endif
static_assert(CR_T >= 512 && CR_T % 64 == 0 && CR_NB % CR_SEG == 0 && CR_SEG % CR_R == 0, "one thread per panel row (Dp <= 512)");

__global__ __launch_bounds__(CR_T) void kp_criage_solve(int D, int dp, const int32_t* __restrict__ items,
                                                        const float* __restrict__ Z, const float* __restrict__ E,
                                                        const double* __restrict__ H, double* __restrict__ Aws,
                                                        double* __restrict__ out, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double crl[];  // panel [D][CR_PS]; later b, partial sums
  __shared__ double wv[2][CR_T / 64];
  __shared__ int wi[2][CR_T / 64];
  __shared__ double wrow[2][CR_T / 64][32];  // each wave's best row (its panel columns), by column parity
  __shared__ double jrow[2][32];             // row j, which the pivot row displaces
  __shared__ int phys[512];  // logical row -> workspace row: row swaps move no data
  __shared__ float red[4];
  __shared__ float sig_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef KP_CR_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last = __builtin_amdgcn_s_memtime();
#endif
  const int Dp = (D + CR_NB - 1) / CR_NB * CR_NB;
  const int ld = Dp + 1;
  const int32_t* it = items + 4 * (size_t)blockIdx.x;
  const float* zp = Z + (size_t)it[0] * dp;
  const float* zt = Z + (size_t)it[1] * dp;
  const double* He = H + (size_t)it[2] * D * D;
  const float* ee = E + (size_t)it[3] * dp;
  double* A = Aws + (size_t)blockIdx.x * Dp * ld;
  // sig = sigmoid(e . z_t) in float32: 256 partial sums, four waves, fixed combination order
  if (tid < 256) {
    float part = 0.f;
    for (int j = tid; j < D; j += 256) part += ee[j] * zt[j];
    part = wsum(part);
    if (lane == 0) red[wave] = part;
  }
  __syncthreads();
  if (tid == 0) {
    const float dot = (red[0] + red[1]) + (red[2] + red[3]);
    sig_s = 1.0f / (1.0f + expf(-dot));
  }
  __syncthreads();
  const float sig = sig_s;
  const float c = sig * (1.0f - sig);
  for (int i = wave; i < Dp; i += CR_T / 64) {
    if (i < D) {
      const float zi = zt[i];
      for (int j = lane; j < Dp; j += 64)
        A[(size_t)i * ld + j] = j < D ? He[(size_t)i * D + j] + (double)(c * (zi * zt[j])) : 0.0;
      if (lane == 0) A[(size_t)i * ld + Dp] = (double)zi;
    } else {
      for (int j = lane; j < ld; j += 64) A[(size_t)i * ld + j] = j == i ? 1.0 : 0.0;
    }
  }
  for (int i = tid; i < Dp; i += CR_T) phys[i] = i;
  __syncthreads();
  CR_ST(0);
  bool singular = false;
  constexpr int w = CR_NB;
  for (int k0 = 0; k0 < Dp && !singular; k0 += CR_NB) {
    const int m = Dp - k0;
    // the panel: thread i holds logical row k0 + i in registers.  `me` is tid made opaque
    // per panel, so the compiler does not hoist the 64 per-column row tests (tid == j,
    // tid > j) out of the panel loop into spilled mask registers
    int me = tid;
    asm volatile("" : "+v"(me));
    const bool own = me < m;
    double P[CR_NB];
    if (own) {
      const double* src = A + (size_t)phys[k0 + tid] * ld + k0;
#pragma unroll
      for (int t = 0; t < w; ++t) P[t] = src[t];
    }
    CR_ST(1);
    double v = own ? fabs(P[0]) : -1.0;
    int vi = own ? me : 0x7fffffff;
    static_for<CR_NB>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // pivot: first row of maximal |a| (idamax); this column's candidates were
      // computed by the previous column's update
      // one barrier per column: each wave publishes its best (value, row) and that row's
      // data, thread j its own row, in the buffer of this column's parity (a thread can
      // only reach column j + 2's writes after every thread passed column j + 1's barrier)
      constexpr int buf = j & 1;
      wave_argmax(v, vi);
      if (lane == 0) {
        wv[buf][wave] = v;
        wi[buf][wave] = vi;
      }
      if (me == vi) {
#pragma unroll
        for (int t = 0; t < w; ++t) wrow[buf][wave][t] = P[t];
      }
      if (me == j) {
#pragma unroll
        for (int t = 0; t < w; ++t) jrow[buf][t] = P[t];
      }
      __syncthreads();
      CR_ST(2);
      double best = wv[buf][0];
      int p = wi[buf][0];
#pragma unroll
      for (int q = 1; q < CR_T / 64; ++q)
        if (wv[buf][q] > best || (wv[buf][q] == best && wi[buf][q] < p)) {
          best = wv[buf][q];
          p = wi[buf][q];
        }
      // exactly singular: LAPACK's getrf reports it, numpy.linalg.inv raises (uniform; the
      // remaining columns only pass their barriers)
      singular = singular || best == 0.0;
      if (singular) p = j;
      const double* prow = wrow[buf][p >> 6];
      if (p != j && me == 0) {
        const int t = phys[k0 + j];
        phys[k0 + j] = phys[k0 + p];
        phys[k0 + p] = t;
      }
      CR_ST(3);
      if (p != j && me == j) {
#pragma unroll
        for (int t = 0; t < w; ++t) P[t] = prow[t];
      }
      if (p != j && me == p) {
#pragma unroll
        for (int t = 0; t < w; ++t) P[t] = jrow[buf][t];
      }
      v = -1.0;
      vi = 0x7fffffff;
      if (!singular && own && me > j) {
        const double l = P[j] / prow[j];
        P[j] = l;
        if constexpr (j + 1 < w) {
          P[j + 1] -= l * prow[j + 1];
          v = fabs(P[j + 1]);
          vi = me;
        }
#pragma unroll
        for (int t = j + 2; t < w; ++t) P[t] -= l * prow[t];
      }
      CR_ST(4);
    });
    if (singular) break;
    // L11 / L21 to the LDS panel; U11 rows back to the workspace (the back substitution reads them)
    if (own) {
#pragma unroll
      for (int t = 0; t < w; ++t) crl[tid * CR_PS + t] = P[t];
    }
    if (tid < w) {
      double* dst = A + (size_t)phys[k0 + tid] * ld + k0;
#pragma unroll
      for (int t = 0; t < w; ++t) dst[t] = P[t];
    }
    __syncthreads();
    // U12 = L11^-1 A12 over the trailing columns and b, one column per thread (nc <= 513)
    const int c0 = k0 + w, nc = ld - c0;
    if (tid < nc) {
      double* Ac = A + c0 + tid;
      double u[CR_NB];
#pragma unroll
      for (int j = 0; j < w; ++j) u[j] = Ac[(unsigned)(phys[k0 + j] * ld)];
#pragma unroll
      for (int j = 1; j < w; ++j) {
#pragma unroll
        for (int i = 0; i < j; ++i) u[j] -= crl[j * CR_PS + i] * u[i];
        __builtin_amdgcn_sched_barrier(0);  // one row's L11 reads at a time (register pressure)
      }
      // the map re-read (memory clobber) rather than 32 offsets held across the solve
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < w; ++j) Ac[(unsigned)(phys[k0 + j] * ld)] = u[j];
    }
    __syncthreads();
    CR_ST(5);
    // A22 -= L21 U12: items of CR_SEG rows x 64 columns, one per wave at a time; U12's
    // column loaded once per item, the rows in chunks of CR_R with the next chunk's loads
    // issued before the current chunk's arithmetic
    const int r0 = k0 + w, nr = Dp - r0;
    if (nr > 0) {
      const int rg = nr / CR_SEG, cg = (nc + 63) / 64;
      for (int item = wave; item < rg * cg; item += CR_T / 64) {
        const int ri = item / cg, ci = item - ri * cg;
        const int col = c0 + ci * 64 + lane;
        if (col < ld) {
          double u[CR_NB];
#pragma unroll
          for (int t = 0; t < w; ++t) u[t] = A[(unsigned)(phys[k0 + t] * ld + col)];
          const int rb = r0 + CR_SEG * ri;
          double a[2][CR_R];
          unsigned off[2][CR_R];
#pragma unroll
          for (int q = 0; q < CR_R; ++q) {
            off[0][q] = (unsigned)(phys[rb + q] * ld + col);
            a[0][q] = A[off[0][q]];
          }
          static_for<CR_SEG / CR_R>([&](auto cc) {
            constexpr int ch = decltype(cc)::value, cur = ch & 1, nxt = cur ^ 1;
            if constexpr (ch + 1 < CR_SEG / CR_R) {
#pragma unroll
              for (int q = 0; q < CR_R; ++q) {
                off[nxt][q] = (unsigned)(phys[rb + (ch + 1) * CR_R + q] * ld + col);
                a[nxt][q] = A[off[nxt][q]];
              }
            }
#pragma unroll
            for (int q = 0; q < CR_R; ++q) {
              const double* L = crl + (rb - k0 + ch * CR_R + q) * CR_PS;
#pragma unroll
              for (int t0 = 0; t0 < w; t0 += 8) {
#pragma unroll
                for (int t = t0; t < t0 + 8; ++t) a[cur][q] -= L[t] * u[t];
                __builtin_amdgcn_sched_barrier(0);  // eight L21 reads in flight at a time (register pressure)
              }
            }
#pragma unroll
            for (int q = 0; q < CR_R; ++q) A[off[cur][q]] = a[cur][q];
          });
        }
      }
    }
    __syncthreads();
    CR_ST(6);
  }
  if (singular) {
    if (tid == 0) {
      out[blockIdx.x] = NAN;
      status[blockIdx.x] = 1;
    }
    return;
  }
  // back substitution: y_i = b_i / U_ii, then b_j -= U_ji y_i for j < i, i descending;
  // U's columns [lo, hi) of rows [0, hi) staged in LDS per block
  double* bsh = crl;
  double* ub = crl + 768;
  for (int i = tid; i < Dp; i += CR_T) bsh[i] = A[(size_t)phys[i] * ld + Dp];
  for (int hi = Dp; hi > 0; hi -= CR_NB) {
    const int lo = hi - CR_NB;
    for (int r = tid >> 5; r < hi; r += CR_T / 32) ub[r * CR_PS + (tid & 31)] = A[(size_t)phys[r] * ld + lo + (tid & 31)];
    __syncthreads();
    if (wave == 0) {
      const int row = lo + lane;
      double b = lane < w ? bsh[row] : 0.0;
      for (int i = hi - 1; i >= lo; --i) {
        if (row == i) b = b / ub[row * CR_PS + (i - lo)];
        const double yi = __shfl(b, i - lo, 64);
        if (row < i) b -= ub[row * CR_PS + (i - lo)] * yi;
      }
      if (lane < w) bsh[row] = b;
    }
    __syncthreads();
    for (int row = tid; row < lo; row += CR_T) {
      const double* Ur = ub + row * CR_PS;
      double b = bsh[row];
      for (int i = hi - 1; i >= lo; --i) b -= Ur[i - lo] * bsh[i];
      bsh[row] = b;
    }
    __syncthreads();
  }
  CR_ST(7);
#ifdef KP_CR_STAMPS
  if (blockIdx.x == 0 && tid == 0)
    printf("[cr stamps] build %llu panel-load %llu pivot %llu swap %llu elim %llu u12 %llu trailing %llu backsub %llu\n",
           st_acc[0], st_acc[1], st_acc[2], st_acc[3], st_acc[4], st_acc[5], st_acc[6], st_acc[7]);
#endif
  double* rv = crl + 512;
  const double om = (double)(1.0f - sig);
  if (tid < 256) {
    double acc = 0.0;
    for (int j = tid; j < D; j += 256) acc += (double)zp[j] * (om * bsh[j]);
    rv[tid] = acc;
  }
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
  // candidates in chunks: one float64 D x (D + 1) system per workgroup
  const int Dp = (D + CR_NB - 1) / CR_NB * CR_NB;
  const size_t sys = (size_t)Dp * (Dp + 1);
  const int chunk = std::max(1, std::min(n, (int)(((size_t)4 << 30) / (sys * sizeof(double)))));
  double* dA = reinterpret_cast<double*>(ba.ensure(sizeof(double) * (size_t)chunk * sys));
  const size_t lds = sizeof(double) * ((size_t)768 + (size_t)Dp * CR_PS);
  for (int i0 = 0; i0 < n; i0 += chunk) {
    const int m = std::min(chunk, n - i0);
    int32_t* dIt = upload(c, bit, it4.data() + 4 * (size_t)i0, (size_t)4 * m);
    double* dO = reinterpret_cast<double*>(bo.ensure(sizeof(double) * (size_t)m));
    int32_t* dS = reinterpret_cast<int32_t*>(bs.ensure(sizeof(int32_t) * (size_t)m));
    hipLaunchKernelGGL(kp_criage_solve, dim3(m), dim3(CR_T), lds, c->stream, D, c->dp, dIt, dZ, c->dE, dH, dA, dO,
                       dS);
    KP_HIP(hipGetLastError());
    KP_HIP(hipMemcpyAsync(out + i0, dO, sizeof(double) * m, hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipMemcpyAsync(status + i0, dS, sizeof(int32_t) * m, hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
  }
  for (DevBuf* b : {&bsrc, &bz, &bt, &bte, &bx, &bw, &boff, &bh, &bit, &ba, &bo, &bs}) b->release();
}
