// kp_gemm3.hip -- C = A B^T on bf16 MFMA with three-piece operands ("bf16x3", as
// kp_attn3): ConvE's two FC GEMMs inside the post-training step loop
// (conve.py:143-146 forward: flat [pairs x 9728] . fc.weight^T; its transpose backward
// [pairs x 200] . fc.weight).  Same contract as kp_gemm_abt (kp_rank.hip):
//   out[z][m][n] = act(sum_{k in split z} A[m][k] B[n][k] + (z == 0 ? bias[n] : 0)),
// but B (and A, unless A_F32) arrive as split images: every fp32 value x as three bf16 pieces
// x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1), stored piece-major
// ([3][rows][ld], split3_rows).  The FC weights are split once per context (conve_fc3);
// the backward's 200-wide A once per step (every one of its 152 column tiles reads it);
// the forward's 9728-wide A by the workgroups as they stage it (A_F32, below).  A product takes the six bf16 x bf16 terms of mfma3 (the
// dropped three are below 2^-24 |a||b|), so the result agrees with the fp32 GEMM to fp32
// rounding (not bitwise: the accumulation order differs).  Per 32-deep k step and 16 x 16
// block: 6 v_mfma_f32_16x16x32_bf16 of 16 cycles against 8 v_mfma_f32_16x16x4f32 of 32.
//
// Tile 64 x 64 x 32, four waves; wave w owns rows [16 w, 16 w + 16) x 64 columns (four
// accumulators).  LDS: two stages x two operands x three pieces x 64 rows at a 96-byte
// row stride (the 16-lane groups of ds_read_b128 then hit 64 distinct banks); the next k
// tile's global loads (16 B per piece per thread) are issued before the current tile's
// MFMAs and stored to the other stage after them: one barrier per k tile.
#include "kp_common.hpp"
#include "kp_attn3.hpp"

namespace {

using kpattn::bf16x8;

constexpr int G3_BK = 32;
constexpr int G3_RS = 48;                // LDS row stride in bf16 (96 B)
constexpr int G3_PS = 64 * G3_RS;        // one piece of one operand tile (bf16)
constexpr int G3_STAGE = 2 * 3 * G3_PS;  // A and B pieces of one stage

// A_F32: A arrives as fp32 [M][lda] and each workgroup splits its own A tiles while staging
// them (the ConvE forward, whose 9728-wide activations four column tiles read: a split
// image would cost more HBM traffic than the redundant split costs VALU)
// NST: LDS stages (2: 73,728 B, two workgroups per CU; 1: 36,864 B, four, with a second
// barrier per k tile)
template <bool A_F32, int NST>
__global__ __launch_bounds__(256) void kp_gemm3_abt(const void* __restrict__ Av, int lda, int M,
                                                    const __bf16* __restrict__ B3, int ldb, int N, int k_begin,
                                                    int k_end, float* __restrict__ out, int ldo,
                                                    const float* __restrict__ bias, int act) {
  extern __shared__ __attribute__((aligned(16))) __bf16 g3s[];  // [stage][A p0 p1 p2 | B p0 p1 p2][64][G3_RS]
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int m0 = blockIdx.y * 64;
  const int n0 = blockIdx.x * 64;
  const int ksplit = gridDim.z;
  const int klen = (k_end - k_begin + ksplit - 1) / ksplit;
  const int kb = k_begin + blockIdx.z * ((klen + G3_BK - 1) / G3_BK * G3_BK);
  const int ke = min(k_end, kb + (klen + G3_BK - 1) / G3_BK * G3_BK);
  out += (size_t)blockIdx.z * M * ldo;
  const size_t pa = (size_t)M * lda, pb = (size_t)N * ldb;  // piece strides of the images
  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // staging: thread tid takes row tid >> 2, k columns 8 (tid & 3) .. + 7 of every piece
  const int srow = tid >> 2, sk = 8 * (tid & 3);
  const bool arow = m0 + srow < M, brow = n0 + srow < N;
  const size_t arow_off = (size_t)(arow ? m0 + srow : 0) * lda + sk;
  const __bf16* bp = B3 + (size_t)(brow ? n0 + srow : 0) * ldb + sk;
  uint4 ga[3], gb[3];
  float4 gf[2];
  auto gload = [&](int k0) {
    const bool kin = k0 + sk < ke;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int p = 0; p < 3; ++p) gb[p] = (brow && kin) ? *reinterpret_cast<const uint4*>(bp + p * pb + k0) : z;
    if constexpr (A_F32) {
      const float* ap = reinterpret_cast<const float*>(Av) + arow_off + k0;
      const float4 zf = make_float4(0.f, 0.f, 0.f, 0.f);
      gf[0] = (arow && kin) ? *reinterpret_cast<const float4*>(ap) : zf;
      gf[1] = (arow && kin) ? *reinterpret_cast<const float4*>(ap + 4) : zf;
    } else {
      const __bf16* ap = reinterpret_cast<const __bf16*>(Av) + arow_off + k0;
#pragma unroll
      for (int p = 0; p < 3; ++p) ga[p] = (arow && kin) ? *reinterpret_cast<const uint4*>(ap + p * pa) : z;
    }
  };
  auto lstore = [&](int st) {
    __bf16* sa = g3s + st * G3_STAGE + srow * G3_RS + sk;
    if constexpr (A_F32) {
      const float f[8] = {gf[0].x, gf[0].y, gf[0].z, gf[0].w, gf[1].x, gf[1].y, gf[1].z, gf[1].w};
      bf16x8 h, m, l;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 a, b, d;
        kpattn::split3(f[j], a, b, d);
        h[j] = a;
        m[j] = b;
        l[j] = d;
      }
      ga[0] = __builtin_bit_cast(uint4, h);
      ga[1] = __builtin_bit_cast(uint4, m);
      ga[2] = __builtin_bit_cast(uint4, l);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      *reinterpret_cast<uint4*>(sa + p * G3_PS) = ga[p];
      *reinterpret_cast<uint4*>(sa + (3 + p) * G3_PS) = gb[p];
    }
  };

  if (kb < ke) {
    gload(kb);
    if (NST == 2) lstore(0);
  }
  if (NST == 2) __syncthreads();
  int st = 0;
  for (int k0 = kb; k0 < ke; k0 += G3_BK) {
    const bool more = k0 + G3_BK < ke;
    if (NST == 1) {
      lstore(0);
      __syncthreads();
    }
    if (more) gload(k0 + G3_BK);
    const __bf16* sa = g3s + st * G3_STAGE;
    const __bf16* sb = sa + 3 * G3_PS;
    // A operand: row 16 w + c, k = 8 g .. 8 g + 7; B operand: row 16 n + c of B, same k
    bf16x8 a[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(sa + p * G3_PS + (16 * w + c) * G3_RS + 8 * g);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      bf16x8 b[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) b[p] = *reinterpret_cast<const bf16x8*>(sb + p * G3_PS + (16 * n + c) * G3_RS + 8 * g);
      acc[n] = kpattn::mfma3(a, b, acc[n]);
    }
    if (NST == 2 && more) lstore(st ^ 1);
    __syncthreads();
    if (NST == 2) st ^= 1;
  }
  // C block n: lane (g, c) holds rows 16 w + 4 g + r, column 16 n + c
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = n0 + 16 * n + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = m0 + 16 * w + 4 * g + r;
      if (q < M && e < N) {
        float v = acc[n][r];
        if (bias && blockIdx.z == 0) v += bias[e];
        if (act == 1) v = 1.0f / (1.0f + __expf(-v));
        out[(size_t)q * ldo + e] = v;
      }
    }
  }
}

// X [rows][ld] -> pieces [3][rows][ld] over columns [0, cols): one thread per 4 values
__global__ void kp_split3_rows(const float* __restrict__ X, int rows, int cols, int ld, __bf16* __restrict__ out) {
  const int q = cols / 4;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)rows * q) return;
  const int r = (int)(i / q), c4 = 4 * (int)(i % q);
  const size_t o = (size_t)r * ld + c4, ps = (size_t)rows * ld;
  const float4 v = *reinterpret_cast<const float4*>(X + o);
  const float f[4] = {v.x, v.y, v.z, v.w};
  typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
  bf4 h, m, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    __bf16 a, b, d;
    kpattn::split3(f[j], a, b, d);
    h[j] = a;
    m[j] = b;
    l[j] = d;
  }
  *reinterpret_cast<bf4*>(out + o) = h;
  *reinterpret_cast<bf4*>(out + ps + o) = m;
  *reinterpret_cast<bf4*>(out + 2 * ps + o) = l;
}

}  // namespace

void launch_gemm3_abt(kp_ctx* c, const void* A, bool a_f32, int lda, int M, const uint16_t* B3, int ldb, int N,
                      int K, float* out, int ldo, const float* bias, int act, int ksplit) {
  if (M <= 0 || N <= 0) return;
  KP_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && K <= lda && K <= ldb,
             "gemm3: K and leading dims must be multiples of 8, K within them");
  dim3 grid((N + 63) / 64, (M + 63) / 64, std::max(1, ksplit));
  static const bool one_stage = std::getenv("KP_FC_STAGES") && std::atoi(std::getenv("KP_FC_STAGES")) == 1;
  const __bf16* b3 = reinterpret_cast<const __bf16*>(B3);
  const size_t lds = (one_stage ? 1 : 2) * G3_STAGE * sizeof(__bf16);
#define KP_G3(AF, NS) \
  hipLaunchKernelGGL((kp_gemm3_abt<AF, NS>), grid, dim3(256), lds, c->stream, A, lda, M, b3, ldb, N, 0, K, out, ldo, bias, act)
  if (a_f32) {
    if (one_stage) KP_G3(true, 1); else KP_G3(true, 2);
  } else {
    if (one_stage) KP_G3(false, 1); else KP_G3(false, 2);
  }
#undef KP_G3
  KP_HIP(hipGetLastError());
}

void split3_rows(kp_ctx* c, const float* X, int rows, int cols, int ld, uint16_t* out) {
  if (rows <= 0 || cols <= 0) return;
  KP_REQUIRE(cols % 4 == 0 && ld % 4 == 0 && cols <= ld, "split3_rows: columns and stride must be multiples of 4");
  const long long n = (long long)rows * (cols / 4);
  hipLaunchKernelGGL(kp_split3_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, X, rows, cols, ld,
                     reinterpret_cast<__bf16*>(out));
  KP_HIP(hipGetLastError());
}
