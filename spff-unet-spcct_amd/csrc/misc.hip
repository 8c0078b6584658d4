// Layout conversion, MaxPool3d((1,2,2)) forward/backward and small utilities.
// Reference: MaxPool3d(P=(1,2,2)) models.py:661-665 (pool only in H,W: F6).
#include "spff_internal.h"
#include <math.h>

namespace spff {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// x [B][C][D][H][W] (reference layout) -> y [B][D][H][W][ldy], channels C..ldy-1 = 0
__global__ void k_ncdhw_to_ndhwc(const float* __restrict__ x, float* __restrict__ y, int B,
                                 int64_t S, int C, int ldy) {
  const int64_t V = (int64_t)B * S;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = v / S, sp = v % S;
    float* o = y + v * ldy;
    for (int c = 0; c < ldy; ++c) o[c] = c < C ? x[(b * C + c) * S + sp] : 0.f;
  }
}

hipError_t ncdhw_to_ndhwc(const float* x, float* y, Vol vol, int C, int ldy, hipStream_t s) {
  const int64_t S = (int64_t)vol.D * vol.H * vol.W;
  const int64_t V = vol.B * S;
  int grid = (int)std::min<int64_t>((V + 255) / 256, 8192);
  hipLaunchKernelGGL(k_ncdhw_to_ndhwc, dim3(grid), dim3(256), 0, s, x, y, vol.B, S, C, ldy);
  return hipGetLastError();
}

// ---------------------------------------------------------------- maxpool --
// Tie rule = PyTorch CPU max_pool: scan (dh,dw) in row-major order, replace on
// strictly greater or NaN, so the FIRST max wins.  idx = dh*2 + dw.
__global__ void k_maxpool_fwd(const float* __restrict__ x, float* __restrict__ y,
                              uint8_t* __restrict__ idx, Vol in, int C) {
  const int Ho = in.H / 2, Wo = in.W / 2, C4 = C / 4;
  const int64_t total = (int64_t)in.B * in.D * Ho * Wo * C4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    int64_t t = i / C4;
    const int wo = (int)(t % Wo); t /= Wo;
    const int ho = (int)(t % Ho); t /= Ho;  // t = b*D + d
    const int64_t vin = (t * in.H + 2 * ho) * in.W + 2 * wo;
    float best[4];
    uint8_t bi[4] = {0, 0, 0, 0};
    {
      const float4 v = *reinterpret_cast<const float4*>(x + vin * C + c);
      best[0] = v.x; best[1] = v.y; best[2] = v.z; best[3] = v.w;
    }
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const int64_t vv = vin + (k >> 1) * in.W + (k & 1);
      const float4 v = *reinterpret_cast<const float4*>(x + vv * C + c);
      const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (vs[j] > best[j] || isnan(vs[j])) { best[j] = vs[j]; bi[j] = (uint8_t)k; }
    }
    const int64_t vo = i / C4;
    *reinterpret_cast<float4*>(y + vo * C + c) = make_float4(best[0], best[1], best[2], best[3]);
    *reinterpret_cast<uchar4*>(idx + vo * C + c) = make_uchar4(bi[0], bi[1], bi[2], bi[3]);
  }
}

hipError_t maxpool_fwd(const float* x, float* y, uint8_t* idx, Vol in, int C, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int64_t total = (int64_t)in.B * in.D * (in.H / 2) * (in.W / 2) * (C / 4);
  int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid), dim3(256), 0, s, x, y, idx, in, C);
  return hipGetLastError();
}

// dx[v_in][c] = dskip[v_in*ld + c] + (argmax hit ? dp[v_out][c] : 0)
__global__ void k_maxpool_bwd_add(const float* __restrict__ dp, const uint8_t* __restrict__ idx,
                                  const float* __restrict__ dskip, int ldskip,
                                  float* __restrict__ dx, Vol in, int C) {
  const int Ho = in.H / 2, Wo = in.W / 2, C4 = C / 4;
  const int64_t total = (int64_t)in.B * in.D * in.H * in.W * C4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const int64_t v = i / C4;
    int64_t t = v;
    const int w = (int)(t % in.W); t /= in.W;
    const int h = (int)(t % in.H); t /= in.H;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (dskip) {
      const float* p = dskip + v * ldskip + c;
      o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3];
    }
    const int ho = h >> 1, wo = w >> 1;
    if (ho < Ho && wo < Wo) {
      const int64_t vo = (t * Ho + ho) * Wo + wo;
      const uint8_t k = (uint8_t)((h & 1) * 2 + (w & 1));
      const uchar4 ix = *reinterpret_cast<const uchar4*>(idx + vo * C + c);
      const float4 g = *reinterpret_cast<const float4*>(dp + vo * C + c);
      if (ix.x == k) o[0] += g.x;
      if (ix.y == k) o[1] += g.y;
      if (ix.z == k) o[2] += g.z;
      if (ix.w == k) o[3] += g.w;
    }
    *reinterpret_cast<float4*>(dx + v * C + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

hipError_t maxpool_bwd_add(const float* dp, const uint8_t* idx, const float* dskip, int ldskip,
                           float* dx, Vol in, int C, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int64_t total = (int64_t)in.B * in.D * in.H * in.W * (C / 4);
  int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(k_maxpool_bwd_add, dim3(grid), dim3(256), 0, s, dp, idx, dskip, ldskip, dx,
                     in, C);
  return hipGetLastError();
}

__global__ void k_scale(float* x, int64_t n, const float* scale) {
  const float a = *scale;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= a;
}

hipError_t scale_by_dev(float* x, int64_t n, const float* scale, hipStream_t s) {
  int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_scale, dim3(grid), dim3(256), 0, s, x, n, scale);
  return hipGetLastError();
}

}  // namespace spff
