// Probe (diagnostics): bias of a chain of S v_mfma_f32_32x32x16_bf16 accumulations
// (one output tile accumulated over S k-steps of random bf16 operands), and the
// same chain with the accumulator's sign flipped every F steps (operands of the
// flipped steps negated, accumulator negated at each flip; sign restored at the end).
// Prints the mean signed error and rms error of D relative to rms(D).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void chain(const __bf16* A, const __bf16* B, float* D, int S, int F) {
  const int lane = threadIdx.x, blk = blockIdx.x;
  A += (size_t)blk * S * 512; B += (size_t)blk * S * 512; D += blk * 1024;
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  bool neg = false;
  for (int s = 0; s < S; ++s) {
    if (F > 0 && s > 0 && s % F == 0) {
      neg = !neg;
      for (int r = 0; r < 16; ++r) c[r] = -c[r];
    }
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * (lane >> 5) + e;
      const float av = (float)A[s * 512 + (lane & 31) * 16 + k];
      a[e] = (__bf16)(neg ? -av : av);
      b[e] = B[s * 512 + k * 32 + (lane & 31)];
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    D[i * 32 + (lane & 31)] = neg ? -c[r] : c[r];
  }
}

int main() {
  const int NB = 512;
  std::mt19937 rng(11);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (int S : {16, 64, 256}) {
    std::vector<__bf16> A((size_t)NB * S * 512), B((size_t)NB * S * 512);
    std::vector<float> Af(A.size()), Bf(B.size()), D(NB * 1024);
    for (size_t i = 0; i < A.size(); ++i) {
      Af[i] = (float)(__bf16)nd(rng); A[i] = (__bf16)Af[i];
      Bf[i] = (float)(__bf16)nd(rng); B[i] = (__bf16)Bf[i];
    }
    std::vector<double> ex(NB * 1024, 0.0);
    for (int blk = 0; blk < NB; ++blk)
      for (int s = 0; s < S; ++s)
        for (int i = 0; i < 32; ++i)
          for (int k = 0; k < 16; ++k) {
            const double a = Af[((size_t)blk * S + s) * 512 + i * 16 + k];
            const float* bp = &Bf[((size_t)blk * S + s) * 512 + k * 32];
            double* e = &ex[blk * 1024 + i * 32];
            for (int j = 0; j < 32; ++j) e[j] += a * bp[j];
          }
    __bf16 *dA, *dB;
    float* dD;
    (void)hipMalloc(&dA, A.size() * 2); (void)hipMalloc(&dB, B.size() * 2); (void)hipMalloc(&dD, D.size() * 4);
    (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    for (int F : {0, 1, 2, 4, 8}) {
      hipLaunchKernelGGL(chain, dim3(NB), dim3(64), 0, 0, dA, dB, dD, S, F);
      (void)hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
      double se = 0, se2 = 0, sd2 = 0;
      for (int i = 0; i < NB * 1024; ++i) {
        const double e = D[i] - ex[i];
        se += e; se2 += e * e; sd2 += ex[i] * ex[i];
      }
      const double n = NB * 1024.0, rd = std::sqrt(sd2 / n);
      printf("S=%3d flip every %d: mean err %+.3e  rms err %.3e  (x rms(D); 2^-24 = 5.96e-08)\n", S, F,
             se / n / rd, std::sqrt(se2 / n) / rd);
    }
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dD);
  }
  return 0;
}
