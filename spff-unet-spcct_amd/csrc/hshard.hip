// Height sharding of the registry layout [B, 1, 5, H, W] ("in the
// registry layout (D = 5), shard H instead, in multiples of 8 rows"): rank r owns
// global rows [r H_l, (r + 1) H_l) at level 0 (H_l a multiple of 8, so the three
// (1,2,2) pools and the up-convolutions stay rank-local).  Every 3x3x3 conv of a
// height-sharded plan runs on a row-padded copy of its input:
//
//   xp[b][d][hp][w][c], hp in [0, H + 2), pitch ldp (multiple of 8, zero channels
//   beyond the conv's input channels):  rows 1 .. H = the local rows (the two-source
//   [up | skip] view and the fused lrelu(IN(y1)) input activation applied here),
//   rows 0 and H + 1 = the neighbours' boundary rows (zero at the global ends),
//
// the conv kernels see a volume of H + 2 rows whose first and last output rows are
// discarded (k_hunpad); for the weight gradient dy is padded with zero rows, so
// those rows contribute nothing.  The boundary rows travel through a staging slab
// [recv_lo | send_lo | send_hi | recv_hi] (each B D W ldp floats) with the caller's
// spff_coll.halo at d_local = 2, the same callback depth sharding uses.
// HBM-bound copies: one read and one write of the conv input / output per conv.
#include "spff_internal.h"

#include <algorithm>

namespace spff {

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// one thread per (padded voxel, 4-channel group)
__global__ __launch_bounds__(256) void k_hpad(Src2 x, int cin, float* __restrict__ xp,
                                              float* __restrict__ send, int B, int D, int H,
                                              int W, int ldp) {
  const int q4 = ldp >> 2;
  const int64_t nrow = (int64_t)W * q4;
  const int64_t total = (int64_t)B * D * (H + 2) * nrow;
  const int64_t S = (int64_t)B * D * W * ldp;  // one staging slice
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % q4) * 4;
    const int64_t vp = i / q4;  // ((b D + d)(H + 2) + hp) W + w
    const int w = (int)(vp % W);
    const int64_t r = vp / W;
    const int hp = (int)(r % (H + 2));
    const int64_t bd = r / (H + 2);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (hp >= 1 && hp <= H && c < cin) {
      const int64_t vi = (bd * H + hp - 1) * W + w;  // local voxel
      const int b = (int)(bd / D);
      if (c < x.split) {
        v = ld4(x.p0 + vi * x.ld0 + c);
        if (x.al) {
          float t4[4] = {v.x, v.y, v.z, v.w};
          const float* ap = x.al + (int64_t)b * x.ld0 + c;
          const float* dp = x.de + (int64_t)b * x.ld0 + c;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = t4[j] * ap[j] + dp[j];
            t4[j] = fmaxf(t, 0.01f * t);  // lrelu(t, 0.01), as the fused conv load
          }
          v = make_float4(t4[0], t4[1], t4[2], t4[3]);
        }
      } else {
        v = ld4(x.p1 + vi * x.ld1 + (c - x.split));
      }
      if (c + 4 > cin) {  // zero the pad channels of a partial group
        if (c + 1 >= cin) v.y = 0.f;
        if (c + 2 >= cin) v.z = 0.f;
        if (c + 3 >= cin) v.w = 0.f;
      }
    }
    st4(xp + vp * ldp + c, v);
    if (send && (hp == 1 || hp == H)) {
      const int64_t si = (bd * W + w) * ldp + c;
      if (hp == 1) st4(send + si, v);
      if (hp == H) st4(send + S + si, v);
    }
  }
}

// rows 0 and H + 1 of xp from the received boundary rows (zero at a global end)
__global__ __launch_bounds__(256) void k_hfill(float* __restrict__ xp, const float* __restrict__ lo,
                                               const float* __restrict__ hi, int B, int D, int H,
                                               int W, int ldp, int zlo, int zhi) {
  const int q4 = ldp >> 2;
  const int64_t slice = (int64_t)B * D * W * q4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 2 * slice;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool top = i >= slice;
    const int64_t j = top ? i - slice : i;
    const int c = (int)(j % q4) * 4;
    const int64_t vw = j / q4;  // (b D + d) W + w
    const int w = (int)(vw % W);
    const int64_t bd = vw / W;
    const int hp = top ? H + 1 : 0;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!(top ? zhi : zlo)) v = ld4((top ? hi : lo) + vw * ldp + c);
    st4(xp + ((bd * (H + 2) + hp) * W + w) * ldp + c, v);
  }
}

// y (Dst2, local rows) <- rows 1 .. H of the padded conv output yp (pitch C)
__global__ __launch_bounds__(256) void k_hunpad(const float* __restrict__ yp, Dst2 y, int C,
                                                int B, int D, int H, int W) {
  const int q4 = C >> 2;
  const int64_t total = (int64_t)B * D * H * W * q4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % q4) * 4;
    const int64_t v = i / q4;  // ((b D + d) H + h) W + w
    const int w = (int)(v % W);
    const int64_t r = v / W;
    const int h = (int)(r % H);
    const int64_t bd = r / H;
    const float4 val = ld4(yp + ((bd * (H + 2) + h + 1) * W + w) * C + c);
    if (c < y.split)
      st4(y.p0 + v * y.ld0 + c, val);
    else
      st4(y.p1 + v * y.ld1 + (c - y.split), val);
  }
}

int grid_for(int64_t work) {
  return (int)std::min<int64_t>((work + 255) / 256, 8192);
}

}  // namespace

size_t hpad_floats(Vol v, int ldp) { return (size_t)v.B * v.D * (v.H + 2) * v.W * ldp; }
size_t hstage_floats(Vol v, int ldp) { return (size_t)4 * v.B * v.D * v.W * ldp; }

hipError_t hpad(const Src2& x, int cin, float* xp, float* stage, Vol v, int ldp, hipStream_t s) {
  if (ldp % 8 || cin > ldp || x.ld0 % 4 || x.ld1 % 4 || (x.split < cin && x.split % 4))
    return hipErrorInvalidValue;
  const int64_t work = (int64_t)v.B * v.D * (v.H + 2) * v.W * (ldp / 4);
  float* send = stage ? stage + (int64_t)v.B * v.D * v.W * ldp : nullptr;
  hipLaunchKernelGGL(k_hpad, dim3(grid_for(work)), dim3(256), 0, s, x, cin, xp, send, v.B, v.D,
                     v.H, v.W, ldp);
  return hipGetLastError();
}

hipError_t hfill(float* xp, const float* stage, Vol v, int ldp, int zlo, int zhi, hipStream_t s) {
  const int64_t S = (int64_t)v.B * v.D * v.W * ldp;
  hipLaunchKernelGGL(k_hfill, dim3(grid_for(2 * S / 4)), dim3(256), 0, s, xp, stage, stage + 3 * S,
                     v.B, v.D, v.H, v.W, ldp, zlo, zhi);
  return hipGetLastError();
}

hipError_t hunpad(const float* yp, const Dst2& y, int C, Vol v, hipStream_t s) {
  if (C % 4 || y.ld0 % 4 || y.ld1 % 4 || (y.split < C && y.split % 4)) return hipErrorInvalidValue;
  const int64_t work = nvox(v) * (C / 4);
  hipLaunchKernelGGL(k_hunpad, dim3(grid_for(work)), dim3(256), 0, s, yp, y, C, v.B, v.D, v.H,
                     v.W);
  return hipGetLastError();
}

}  // namespace spff
