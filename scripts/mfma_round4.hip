// Probe (diagnostics): split-bf16 (3 planes, 6 products) accumulation chains with
// ONE B (the "weights") shared by every block and fresh random A (the "voxels") per
// block, as in the conv: per output column, the mean error over all rows/blocks
// (the coherent part) vs the rms error, relative to rms(D).  Orders: small products
// first (the conv's current order) and hh first; and the f32 MFMA for reference.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x; float r = x - (float)h;
  m = (__bf16)r; r = r - (float)m;
  l = (__bf16)r;
}

// mode 0: small first (mm, hl, lh, hm, mh, hh); 1: hh first; 2: f32 MFMA 32x32x2
__global__ void chain(const float* A, const float* B, float* D, int S, int mode) {
  const int lane = threadIdx.x, blk = blockIdx.x;
  A += (size_t)blk * S * 512; D += blk * 1024;
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  for (int s = 0; s < S; ++s) {
    if (mode == 2) {
      for (int kk = 0; kk < 8; ++kk) {  // 16 k as 8 steps of k = 2
        f32x2 a = {A[s * 512 + (lane & 31) * 16 + 2 * kk + (lane >> 5)], 0.f};
        float av = A[s * 512 + (lane & 31) * 16 + 2 * kk + (lane >> 5)];
        float bv = B[s * 512 + (2 * kk + (lane >> 5)) * 32 + (lane & 31)];
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, c, 0, 0, 0);
        (void)a;
      }
      continue;
    }
    bf16x8 a[3], b[3];
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * (lane >> 5) + e;
      __bf16 h, m, l;
      split3(A[s * 512 + (lane & 31) * 16 + k], h, m, l);
      a[0][e] = h; a[1][e] = m; a[2][e] = l;
      split3(B[s * 512 + k * 32 + (lane & 31)], h, m, l);
      b[0][e] = h; b[1][e] = m; b[2][e] = l;
    }
    if (mode == 1) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
    if (mode == 0) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    D[i * 32 + (lane & 31)] = c[r];
  }
}

int main() {
  const int NB = 2048, S = 54;  // 54 k-steps of 16 = 27 taps x 32 channels
  std::mt19937 rng(5);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> A((size_t)NB * S * 512), B((size_t)S * 512), D(NB * 1024);
  const float amean = getenv("AMEAN") ? atof(getenv("AMEAN")) : 0.f;
  for (auto& v : A) v = nd(rng) + amean;
  for (auto& v : B) v = nd(rng) * 0.05f;
  std::vector<double> ex(NB * 1024, 0.0);
  for (int blk = 0; blk < NB; ++blk)
    for (int s = 0; s < S; ++s)
      for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 16; ++k) {
          const double a = A[((size_t)blk * S + s) * 512 + i * 16 + k];
          for (int j = 0; j < 32; ++j) ex[blk * 1024 + i * 32 + j] += a * (double)B[s * 512 + k * 32 + j];
        }
  float *dA, *dB, *dD;
  (void)hipMalloc(&dA, A.size() * 4); (void)hipMalloc(&dB, B.size() * 4); (void)hipMalloc(&dD, D.size() * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  const char* names[] = {"split6 small-first", "split6 hh-first", "f32 mfma"};
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(chain, dim3(NB), dim3(64), 0, 0, dA, dB, dD, S, mode);
    (void)hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    double se2 = 0, sd2 = 0, col2 = 0;
    std::vector<double> colm(32, 0.0);
    for (int i = 0; i < NB * 1024; ++i) {
      const double e = D[i] - ex[i];
      se2 += e * e; sd2 += ex[i] * ex[i];
      colm[i % 32] += e;
    }
    const double n = NB * 1024.0, rd = std::sqrt(sd2 / n);
    for (auto v : colm) col2 += (v / (n / 32)) * (v / (n / 32));
    double mall = 0;
    for (auto v : colm) mall += v;
    mall /= n;
    // correlation of the column-mean error with the column sum of B
    std::vector<double> bs(32, 0.0);
    for (int s2 = 0; s2 < S; ++s2)
      for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 32; ++j) bs[j] += B[s2 * 512 + k * 32 + j];
    double sxy = 0, sxx = 0, syy = 0;
    for (int j = 0; j < 32; ++j) {
      const double xm = colm[j] / (n / 32);
      sxy += xm * bs[j]; sxx += xm * xm; syy += bs[j] * bs[j];
    }
    printf("%-20s rms err %.3e  column-mean error: rms %.3e, overall mean %+.3e, corr with colsum(B) %+.2f (x rms(D))\n",
           names[mode], std::sqrt(se2 / n) / rd, std::sqrt(col2 / 32) / rd, mall / rd,
           sxy / std::sqrt(sxx * syy + 1e-300));
  }
  return 0;
}
