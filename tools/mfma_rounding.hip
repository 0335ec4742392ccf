// Accumulation rounding of v_mfma_f32_16x16x32_bf16 (diagnostic, GPU box):
//   hipcc --offload-arch=gfx950 -O2 -o build/mfma_rounding tools/mfma_rounding.hip && ./build/mfma_rounding
// One wave accumulates ITER MFMAs of positive bf16 products into one f32 accumulator (the
// shape of kp_attn3's O phase: weights ~1 times table entries ~1e-3, ~1e5 terms) and the
// same chain with fmaf on the VALU.  The host sums the exact products in fp64 and emulates an
// f32 round-to-nearest-even chain.  A signed error growing ~linearly with ITER against both
// says the MFMA accumulation truncates (biased); a random-walk error says it rounds to nearest.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// a ~ 1.0 .. 1.03 (softmax weights), b ~ 2^-11 .. 2^-10 (entries)
__host__ __device__ inline uint16_t a_bits(int it, int k) { return (uint16_t)(0x3F80u + (hash32(it * 64 + k) & 3u)); }
__host__ __device__ inline uint16_t b_bits(int it, int k) {
  return (uint16_t)(0x3A00u + (hash32(0x9e3779b9u ^ (uint32_t)(it * 64 + k)) & 0x7Fu));
}
static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

__global__ void run(int iters, float* out) {
  const int lane = threadIdx.x;
  const int g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float chain = 0.f;
  for (int it = 0; it < iters; ++it) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * g + j;
      uint16_t ab = a_bits(it, k), bb = b_bits(it, k);
      a[j] = __builtin_bit_cast(__bf16, ab);
      b[j] = __builtin_bit_cast(__bf16, bb);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    if (lane == 0) {
      for (int k = 0; k < 32; ++k) {
        uint32_t ua = (uint32_t)a_bits(it, k) << 16, ub = (uint32_t)b_bits(it, k) << 16;
        chain = fmaf(__uint_as_float(ua), __uint_as_float(ub), chain);
      }
    }
  }
  if (lane == 0) {
    out[0] = acc[0];
    out[1] = chain;
  }
}

int main() {
  float* d;
  hipMalloc(&d, 8);
  for (int iters : {1000, 10000, 100000}) {
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, iters, d);
    float h[2];
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    double exact = 0.0;
    float rne = 0.f;
    for (int it = 0; it < iters; ++it) {
      double s = 0.0;
      for (int k = 0; k < 32; ++k) {
        const double p = (double)bf2f(a_bits(it, k)) * (double)bf2f(b_bits(it, k));
        s += p;
        rne = fmaf(bf2f(a_bits(it, k)), bf2f(b_bits(it, k)), rne);
      }
      exact += s;
    }
    printf("iters %6d (%7d products): exact %.9e  mfma %.9e (rel %+.3e)  valu-fmaf %.9e (rel %+.3e)  host-fmaf %+.3e\n",
           iters, 32 * iters, exact, h[0], (h[0] - exact) / exact, h[1], (h[1] - exact) / exact,
           (rne - exact) / exact);
  }
  hipFree(d);
  return 0;
}
