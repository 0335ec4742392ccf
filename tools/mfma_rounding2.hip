// Rounding of ONE v_mfma_f32_16x16x32_bf16 (diagnostic, GPU box):
//   hipcc --offload-arch=gfx950 -O2 -o mfma_rounding2 tools/mfma_rounding2.hip && ./mfma_rounding2
// Random bf16 operands (mixed signs, 8-bit exponent spread) and a random f32 C.  For each
// output the host computes the exact C + sum of 32 products in fp64, its correctly rounded
// f32, and reports the error of the MFMA result in units of the result's ulp: mean signed
// error (bias), mean |error|, max |error|, and the fraction of outputs not equal to the
// correctly rounded value.  Case "pos": all products positive (the O-phase shape).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void run(int trials, const uint16_t* A, const uint16_t* B, const float* C, float* D) {
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = __builtin_bit_cast(__bf16, A[(size_t)t * 512 + lane * 8 + j]);
      b[j] = __builtin_bit_cast(__bf16, B[(size_t)t * 512 + lane * 8 + j]);
    }
    f32x4 c;
    for (int r = 0; r < 4; ++r) c[r] = C[(size_t)t * 256 + lane * 4 + r];
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(size_t)t * 256 + lane * 4 + r] = d[r];
  }
}

static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int trials = 4096;
  std::mt19937 gen(1);
  for (int cs = 0; cs < 3; ++cs) {
    const bool pos = cs >= 1;
    const float cscale = cs == 2 ? 64.f : 1.f;  // a C much larger than the products
    std::vector<uint16_t> A((size_t)trials * 512), B((size_t)trials * 512);
    std::vector<float> C((size_t)trials * 256), D((size_t)trials * 256);
    std::uniform_real_distribution<float> u(0.5f, 1.0f);
    std::uniform_int_distribution<int> ex(-4, 4), sg(0, 1);
    auto mk = [&](bool positive) {
      float v = std::ldexp(u(gen), ex(gen));
      if (!positive && sg(gen)) v = -v;
      uint32_t bits;
      memcpy(&bits, &v, 4);
      return (uint16_t)(bits >> 16);
    };
    for (auto& x : A) x = mk(pos);
    for (auto& x : B) x = mk(pos);
    for (auto& x : C) x = cscale * (pos ? 1.f : (sg(gen) ? 1.f : -1.f)) * std::ldexp(u(gen), 4);
    uint16_t *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(run, dim3(256), dim3(64), 0, 0, trials, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    double bias = 0, mabs = 0, mx = 0;
    long long neq = 0, n = 0;
    for (int t = 0; t < trials; ++t)
      for (int lane = 0; lane < 64; ++lane)
        for (int r = 0; r < 4; ++r) {
          // D[i][j]: lane = j + 16 * (i / 4), r = i % 4 ; A[i][k]: lane i + 16 * (k / 8), elt k % 8;
          // B[k][j]: lane j + 16 * (k / 8), elt k % 8
          const int j = lane & 15, i = 4 * (lane >> 4) + r;
          double s = C[(size_t)t * 256 + lane * 4 + r];
          for (int k = 0; k < 32; ++k)
            s += (double)bf2f(A[(size_t)t * 512 + (i + 16 * (k / 8)) * 8 + k % 8]) *
                 (double)bf2f(B[(size_t)t * 512 + (j + 16 * (k / 8)) * 8 + k % 8]);
          const float cr = (float)s;
          const float got = D[(size_t)t * 256 + lane * 4 + r];
          const double ulp = std::ldexp(1.0, std::ilogb(cr) - 23);
          const double e = ((double)got - s) / ulp;
          bias += e;
          mabs += std::fabs(e);
          mx = std::max(mx, std::fabs(e));
          neq += got != cr;
          ++n;
        }
    printf("%-12s outputs %lld: bias %+.4f ulp, mean|err| %.4f ulp, max %.3f ulp, != correctly rounded %.4f\n",
           cs == 0 ? "mixed-sign" : (cs == 1 ? "positive" : "pos,big C"), n, bias / n, mabs / n, mx,
           (double)neq / n);
    hipFree(dA);
    hipFree(dB);
    hipFree(dC);
    hipFree(dD);
  }
  return 0;
}
