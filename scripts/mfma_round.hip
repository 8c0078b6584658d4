// Probe: rounding of v_mfma_f32_32x32x16_bf16's fp32 accumulation (diagnostics).
// Each case puts 16 bf16 values in row 0 of A (k = 0..15), ones in column 0 of B,
// and C[0][0] = c0; prints D[0][0] - exact next to the round-to-nearest result.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void probe(const float* av, const float* c0, float* out) {
  const int lane = threadIdx.x;
  // A 32x16: lane l holds row l%32, k = 8*(l/32) .. +7;  B 16x32: lane l holds col l%32, same k
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * (lane >> 5) + e;
    a[e] = (__bf16)((lane & 31) == 0 ? av[k] : 0.f);
    b[e] = (__bf16)((lane & 31) == 0 ? 1.f : 0.f);
  }
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  if (lane == 0) c[0] = c0[0];
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  if (lane == 0) out[0] = c[0];
}

int main() {
  struct Case { const char* name; float c0; float a[16]; };
  const float u = ldexpf(1.f, -24);
  Case cs[] = {
      {"1 + 2^-24 + 2^-26 (RNE up)", 0.f, {1.f, u, u / 4}},
      {"1 - 2^-26 (RNE 1, RTZ 1-2^-24)", 0.f, {1.f, -u / 4}},
      {"C=1 + 2^-24 + 2^-26", 1.f, {u, u / 4}},
      {"C=1 - 2^-26", 1.f, {-u / 4}},
      {"C=1 + 0.75*2^-23", 1.f, {u, u / 2}},
      {"C=-1 - 0.75*2^-23", -1.f, {-u, -u / 2}},
      {"C=1 - 0.75*2^-24", 1.f, {-u / 2, -u / 4}},
      {"1 + 2^-30 + 2^-30 (x16)", 0.f, {1.f, ldexpf(1, -30), ldexpf(1, -30), ldexpf(1, -30),
                                       ldexpf(1, -30), ldexpf(1, -30), ldexpf(1, -30),
                                       ldexpf(1, -30), ldexpf(1, -30), ldexpf(1, -30),
                                       ldexpf(1, -30), ldexpf(1, -30), ldexpf(1, -30),
                                       ldexpf(1, -30), ldexpf(1, -30), ldexpf(1, -30)}},
      {"C=2^20 + 1 + 0.5 + 0.25", ldexpf(1, 20), {1.f, 0.5f, 0.25f}},
      {"C=2^23 + 0.75", ldexpf(1, 23), {0.5f, 0.25f}},
      {"C=-2^23 - 0.75", -ldexpf(1, 23), {-0.5f, -0.25f}},
  };
  float *da, *dc, *dout;
  hipMalloc(&da, 64);
  hipMalloc(&dc, 4);
  hipMalloc(&dout, 4);
  for (auto& c : cs) {
    hipMemcpy(da, c.a, 64, hipMemcpyHostToDevice);
    hipMemcpy(dc, &c.c0, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, dc, dout);
    float r;
    hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost);
    long double ex = c.c0;
    for (int k = 0; k < 16; ++k) ex += (long double)c.a[k];
    const float rne = (float)ex;
    printf("%-34s mfma %.10e  exact %.12Le  rne %.10e  %s\n", c.name, r, ex, rne,
           r == rne ? "RNE" : (fabsl((long double)r) < fabsl(ex) ? "toward-zero" : "away"));
  }
  return 0;
}
