// Probe (diagnostics): statistics of v_mfma_f32_32x32x16_bf16's rounding on random
// data -- mean signed error of D = C + A*B in units of ulp(D), split by the sign of D,
// for accumulators of the products' own size and 2^8 / 2^16 larger.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// A [32][16], B [16][32], C/D [32][32] row-major, one MFMA per 64-thread block
__global__ void probe(const __bf16* A, const __bf16* B, const float* C, float* D) {
  const int lane = threadIdx.x, blk = blockIdx.x;
  A += blk * 512; B += blk * 512; C += blk * 1024; D += blk * 1024;
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * (lane >> 5) + e;
    a[e] = A[(lane & 31) * 16 + k];
    b[e] = B[k * 32 + (lane & 31)];
  }
  f32x16 c;
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    c[r] = C[i * 32 + (lane & 31)];
  }
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    D[i * 32 + (lane & 31)] = c[r];
  }
}

static float bf(float x) { return (float)(__bf16)x; }

int main() {
  const int NB = 4096;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<__bf16> A(NB * 512), B(NB * 512);
  std::vector<float> Af(NB * 512), Bf(NB * 512), C(NB * 1024), D(NB * 1024);
  for (int i = 0; i < NB * 512; ++i) {
    Af[i] = bf(nd(rng)); A[i] = (__bf16)Af[i];
    Bf[i] = bf(nd(rng)); B[i] = (__bf16)Bf[i];
  }
  __bf16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  for (float cs : {0.f, 1.f, 256.f, 65536.f}) {
    for (auto& c : C) c = cs * nd(rng);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    double sp = 0, sn = 0, ap = 0, an = 0, np = 0, nn = 0, srne = 0;
    for (int blk = 0; blk < NB; ++blk)
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          long double ex = C[blk * 1024 + i * 32 + j];
          for (int k = 0; k < 16; ++k)
            ex += (long double)Af[blk * 512 + i * 16 + k] * (long double)Bf[blk * 512 + k * 32 + j];
          const float d = D[blk * 1024 + i * 32 + j];
          const double ulp = std::ldexp(1.0, std::ilogb(d == 0 ? 1e-30f : d) - 23);
          const double e = (double)((long double)d - ex) / ulp;
          srne += ((float)ex == d);
          if (ex > 0) { sp += e; ap += std::fabs(e); np += 1; }
          else { sn += e; an += std::fabs(e); nn += 1; }
        }
    printf("|C|~%-8g D>0: mean err %+.4f ulp (mean|err| %.4f)  D<0: mean err %+.4f ulp (mean|err| %.4f)  "
           "equal to RNE(exact): %.2f%%\n", cs, sp / np, ap / np, sn / nn, an / nn,
           100.0 * srne / (NB * 1024.0));
  }
  return 0;
}
