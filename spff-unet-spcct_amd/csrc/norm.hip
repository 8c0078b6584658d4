// InstanceNorm3d(affine, eps=1e-5) + LeakyReLU(0.01) forward/backward and the
// per-(b, c, d) hw-reductions the gate algebra needs (reference models.py:168-181,
// 1453-1469).  All HBM-bound: one float4 (4 channels) per lane, channel-last
// [B][D][H][W][C] rows, per-thread register accumulation over voxels, then a
// fixed-order LDS tree -> deterministic sums, no float atomics.
//
// Naming: y = raw conv output, al = gamma*rstd, de = beta - mean*al (so the
// normalised+affine value is r = y*al + de, exactly the CPU batch-norm
// transform form), a = lrelu(r).
#include "spff_internal.h"

#include <algorithm>
#include <cmath>

#ifndef SPFF_RED_CH
#define SPFF_RED_CH 16
#endif
#ifndef SPFF_EW_GX
#define SPFF_EW_GX 4  // blocks per (b,d) slab: fewer, longer streams measured fastest (64 -> 4: -20 %)
#endif
#ifndef SPFF_EW_MINWG
// Floor on a whole launch's workgroups: with few (b,d) slabs (the registry's D = 5 depth)
// SPFF_EW_GX blocks per slab leave most of the 256 CUs idle (B D 4 = 40 workgroups), so the
// blocks per slab grow until the launch has this many.  The 128^3 patch (B D = 256) keeps 4.
#define SPFF_EW_MINWG 1024
#endif

namespace spff {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
// voxel lanes per 256-thread block for C/4 channel quads: the largest power of two
// <= 256 / (C/4), so the fixed-order LDS tree halves evenly (C = 12, 24, 48, ...
// of the SwinUNETR path leave a few threads idle; powers of two use all 256)
__host__ __device__ inline int red_vpp(int tpv) {
  int v = 256 / tpv, p = 1;
  while (2 * p <= v) p *= 2;
  return p;
}
// elementwise block size: a multiple of C/4, so a thread's channel quad is fixed
// over its grid-stride loop (256 for power-of-two C)
static inline int ew_bs(int C) { return (C / 4) * (256 / (C / 4)); }
#ifndef SPFF_NT
#define SPFF_NT 1  // streaming passes: bit 0 nontemporal loads (kept: -0.22 ms/step A/B), bit 1 stores (slower)
#endif
typedef float nt_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_s(const float* p) {
  if constexpr ((SPFF_NT & 1) != 0) {
    const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void st_s(float* p, const float4& v) {
  if constexpr ((SPFF_NT & 2) != 0) {
    const nt_f4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<nt_f4*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
// neg = negative slope: 0.01 for LeakyReLU (SPFF), 0 for ReLU (3DUNet)
__device__ __forceinline__ float lrelu(float r, float neg) { return r > 0.f ? r : neg * r; }
__device__ __forceinline__ float slope(float r, float neg) { return r > 0.f ? 1.f : neg; }
// g + the pooled gradient routed to (h, w) of slab bd by its argmax byte (PoolAdd), as
// k_maxpool_bwd_add adds it; odd extents: the last row / column has no pooled parent
__device__ __forceinline__ float4 pool_add(float4 g, const PoolAdd& pa, int64_t bd, int hw,
                                           const Vol& vol, int C, int c) {
  const int h = hw / vol.W, w = hw - h * vol.W;
  const int Ho = vol.H >> 1, Wo = vol.W >> 1, ho = h >> 1, wo = w >> 1;
  if (ho < Ho && wo < Wo) {
    const int64_t vo = (bd * Ho + ho) * Wo + wo;
    const uint8_t k = (uint8_t)((h & 1) * 2 + (w & 1));
    const uchar4 ix = *reinterpret_cast<const uchar4*>(pa.idx + vo * C + c);
    const float4 d = *reinterpret_cast<const float4*>(pa.dp + vo * C + c);
    if (ix.x == k) g.x += d.x;
    if (ix.y == k) g.y += d.y;
    if (ix.z == k) g.z += d.z;
    if (ix.w == k) g.w += d.w;
  }
  return g;
}

namespace {
struct RedPlan {
  int tpv, vpp, chunk, nsplit, HW;
};
RedPlan red_plan(Vol vol, int C) {
  RedPlan p;
  p.HW = vol.H * vol.W;
  p.tpv = C / 4;
  p.vpp = red_vpp(p.tpv);
  p.chunk = p.vpp * SPFF_RED_CH;
  p.nsplit = cdiv(p.HW, p.chunk);
  return p;
}
}  // namespace

#ifndef SPFF_RED_BATCH
#define SPFF_RED_BATCH 4  // voxel rows loaded back to back per thread before accumulating
#endif

template <int OP, int NQ>
__device__ __forceinline__ void red_accum(const RedArgs& a, const float (&ys)[4], const float (&gs)[4],
                                          const float (&p0)[4], const float (&p1)[4],
                                          const float (&p2)[4], const float (&p3)[4],
                                          const float (&mu)[4], const float (&rs)[4],
                                          float (&acc)[NQ][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (OP == RED_SUM) {
      acc[0][j] += ys[j];
    } else if (OP == RED_SQDEV) {
      const float t = ys[j] - p0[j];
      acc[0][j] += t * t;
    } else if (OP == RED_ACT) {
      acc[0][j] += lrelu(ys[j] * p0[j] + p1[j], a.neg);
    } else if (OP == RED_BWD_TAIL) {
      acc[0][j] += gs[j];
      acc[NQ - 1][j] += gs[j] * lrelu(ys[j] * p0[j] + p1[j], a.neg);
    } else if (OP == RED_BWD_TAIL6) {
      const float r = ys[j] * p0[j] + p1[j];
      const float sl = slope(r, a.neg), gsl = gs[j] * sl;
      const float xh = (ys[j] - mu[j]) * rs[j];
      acc[0][j] += gs[j];
      acc[1][j] += gs[j] * lrelu(r, a.neg);
      acc[2][j] += gsl;
      acc[3][j] += sl;
      acc[4][j] += gsl * xh;
      acc[5][j] += sl * xh;
    } else {  // RED_BWD_IN
      const float r = ys[j] * p0[j] + p1[j];
      const float dr = (gs[j] * p2[j] + p3[j]) * slope(r, a.neg);
      const float xh = (ys[j] - mu[j]) * rs[j];
      acc[0][j] += dr;
      acc[NQ - 1][j] += dr * xh;
    }
  }
}

// One block per (split, b*D + d): the thread (vo, cq) streams channel quad cq of voxels
// hb + vo, hb + vo + vpp, ... of the slab's chunk, SPFF_RED_BATCH rows loaded back to
// back (several 16-B loads in flight per thread: the single-load loop held ~half the
// bytes in flight the HBM needs), then the fixed-order reduction over vo: for power-of-
// two quads per voxel (C = 4 .. 256) xor-shuffles inside each wave and the 4 wave sums
// added in wave order through LDS (one barrier); otherwise (SwinUNETR's C = 12, 24, 48,
// the 3DUNet's C = 512) the LDS tree.
template <int OP, int NQ>
__global__ __launch_bounds__(256) void k_slab_reduce(RedArgs a, Vol vol, int C, float* __restrict__ ws,
                                                     int nsplit, int chunk) {
  constexpr bool TWO = OP == RED_BWD_TAIL || OP == RED_BWD_IN || OP == RED_BWD_TAIL6;
  constexpr int NB = SPFF_RED_BATCH;
  const int bd = blockIdx.y;  // b*D + d
  const int split = blockIdx.x;
  const int b = bd / vol.D, d = bd % vol.D;
  const int HW = vol.H * vol.W;
  const int tpv = C >> 2, vpp = red_vpp(tpv);
  const int cq = threadIdx.x % tpv, vo = threadIdx.x / tpv;
  const int c = 4 * cq;
  float acc[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[q][j] = 0.f;
  if (vo < vpp) {
    float p0[4], p1[4], p2[4], p3[4];  // per-channel params
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int bc = b * C + c + j;
      p0[j] = 0.f; p1[j] = 0.f; p2[j] = 1.f; p3[j] = 0.f;
      if (OP == RED_SQDEV) p0[j] = a.mean[bc];
      if (OP == RED_ACT || OP == RED_BWD_TAIL || OP == RED_BWD_IN || OP == RED_BWD_TAIL6) {
        p0[j] = a.al[bc];
        p1[j] = a.de[bc];
      }
      if (OP == RED_BWD_IN) {
        if (a.A) { p2[j] = a.A[(int64_t)bc * vol.D + d]; p3[j] = a.Bc[(int64_t)bc * vol.D + d]; }
      }
    }
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, rs[4] = {0.f, 0.f, 0.f, 0.f};
    if (OP == RED_BWD_IN || OP == RED_BWD_TAIL6) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { mu[j] = a.mean[b * C + c + j]; rs[j] = a.rstd[b * C + c + j]; }
    }
    const int hb = split * chunk, he = min(HW, hb + chunk);
    const int64_t base = (int64_t)bd * HW;
    for (int hw0 = hb + vo; hw0 < he; hw0 += NB * vpp) {
      float4 yv[NB], gv[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int hw = hw0 + k * vpp;
        const int64_t off = (base + (hw < he ? hw : hw0)) * C + c;
        yv[k] = ld_s(a.y + off);
        if (TWO) gv[k] = ld_s(a.g + off);
        if (TWO && a.pa.dp) gv[k] = pool_add(gv[k], a.pa, bd, hw < he ? hw : hw0, vol, C, c);
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (hw0 + k * vpp >= he) break;
        const float ys[4] = {yv[k].x, yv[k].y, yv[k].z, yv[k].w};
        float gs[4] = {0.f, 0.f, 0.f, 0.f};
        if (TWO) { gs[0] = gv[k].x; gs[1] = gv[k].y; gs[2] = gv[k].z; gs[3] = gv[k].w; }
        red_accum<OP, NQ>(a, ys, gs, p0, p1, p2, p3, mu, rs, acc);
      }
    }
  }
  __shared__ float red[256 * 4 * (NQ > 4 ? NQ : 4)];
  if ((tpv & (tpv - 1)) == 0 && tpv <= 64) {
    // xor-shuffle tree over the wave's 64 / tpv voxel lanes (vpp = 256 / tpv, so every
    // thread is active and the waves hold equal voxel-lane counts), then the waves in order
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[q][j];
        for (int o = tpv; o < 64; o <<= 1) v += __shfl_xor(v, o);
        acc[q][j] = v;
      }
    if (lane < tpv) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[((wv * NQ + q) * tpv + lane) * 4 + j] = acc[q][j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NQ * tpv * 4; i += 256) {
      const int j = i & 3, cqq = (i >> 2) % tpv, q = (i >> 2) / tpv;
      float t = 0.f;
      for (int w = 0; w < 4; ++w) t += red[((w * NQ + q) * tpv + cqq) * 4 + j];
      ws[(((int64_t)bd * nsplit + split) * C + 4 * cqq + j) * NQ + q] = t;
    }
    return;
  }
  // fixed-order LDS tree over the vpp voxel lanes
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = acc[q][j];
    __syncthreads();
    for (int st = vpp / 2; st >= 1; st >>= 1) {
      if (vo < st) {
#pragma unroll
        for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] += red[(threadIdx.x + st * tpv) * 4 + j];
      }
      __syncthreads();
    }
    if (vo == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ws[(((int64_t)bd * nsplit + split) * C + c + j) * NQ + q] = red[threadIdx.x * 4 + j];
    }
    __syncthreads();
  }
}

// combine splits: out[b][c][d][q] = sum_split ws[bd][split][c][q]; with out2, q >= 2 go to
// out2[b][c][d][q - 2] (nq - 2 wide) and out holds q 0, 1
__global__ void k_slab_combine(const float* __restrict__ ws, float* __restrict__ out, Vol vol,
                               int C, int nq, int nsplit, float* __restrict__ out2) {
  const int total = vol.B * vol.D * C * nq;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int q = i % nq;
    const int c = (i / nq) % C;
    const int bd = i / (nq * C);
    const int b = bd / vol.D, d = bd % vol.D;
    float s = 0.f;
#pragma unroll 4
    for (int k = 0; k < nsplit; ++k) s += ws[(((int64_t)bd * nsplit + k) * C + c) * nq + q];
    const int64_t slab = ((int64_t)b * C + c) * vol.D + d;
    if (!out2) out[slab * nq + q] = s;
    else if (q < 2) out[slab * 2 + q] = s;
    else out2[slab * (nq - 2) + (q - 2)] = s;
  }
}

__global__ void k_in_sums_from_tail(const float* __restrict__ t4, const float* __restrict__ A,
                                    const float* __restrict__ Bc, float* __restrict__ out,
                                    int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 t = reinterpret_cast<const float4*>(t4)[i];
    const float a = A[i], bc = Bc[i];
    out[2 * i] = a * t.x + bc * t.y;
    out[2 * i + 1] = a * t.z + bc * t.w;
  }
}
hipError_t in_sums_from_tail(const float* t4, const float* A, const float* Bc, float* out,
                             int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_in_sums_from_tail,
                     dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, t4,
                     A, Bc, out, n);
  return hipGetLastError();
}

size_t slab_reduce_ws_bytes(Vol vol, int C, int nq) {
  RedPlan p = red_plan(vol, C);
  return (size_t)vol.B * vol.D * p.nsplit * C * nq * sizeof(float);
}

hipError_t slab_reduce(RedOp op, const RedArgs& a, Vol vol, int C, float* out, float* ws,
                       hipStream_t s, float* out2) {
  if ((op == RED_BWD_TAIL6) != (out2 != nullptr)) return hipErrorInvalidValue;
  if (C % 4 || C > 1024) return hipErrorInvalidValue;
  RedPlan p = red_plan(vol, C);
  dim3 grid(p.nsplit, vol.B * vol.D);
  int nq = 1;
  switch (op) {
    case RED_SUM: hipLaunchKernelGGL((k_slab_reduce<RED_SUM, 1>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
    case RED_SQDEV: hipLaunchKernelGGL((k_slab_reduce<RED_SQDEV, 1>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
    case RED_ACT: hipLaunchKernelGGL((k_slab_reduce<RED_ACT, 1>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
    case RED_BWD_TAIL: nq = 2; hipLaunchKernelGGL((k_slab_reduce<RED_BWD_TAIL, 2>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
    case RED_BWD_IN: nq = 2; hipLaunchKernelGGL((k_slab_reduce<RED_BWD_IN, 2>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
    case RED_BWD_TAIL6: nq = 6; hipLaunchKernelGGL((k_slab_reduce<RED_BWD_TAIL6, 6>), grid, dim3(256), 0, s, a, vol, C, ws, p.nsplit, p.chunk); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int total = vol.B * vol.D * C * nq;
  hipLaunchKernelGGL(k_slab_combine, dim3(std::min(cdiv(total, 256), 4096)), dim3(256), 0, s, ws,
                     out, vol, C, nq, p.nsplit, out2);
  return hipGetLastError();
}

// ------------------------------------------------------------ finalizers --
__global__ void k_in_mean(const float* __restrict__ sums, float* __restrict__ mean, Vol vol, int C) {
  const int bc = blockIdx.x * blockDim.x + threadIdx.x;
  if (bc >= vol.B * C) return;
  double s = 0.0;
  for (int d = 0; d < vol.D; ++d) s += sums[(int64_t)bc * vol.D + d];
  mean[bc] = (float)(s / ((double)vol.D * vol.H * vol.W));
}

__global__ void k_in_rstd(const float* __restrict__ sq, const float* __restrict__ gamma,
                          const float* __restrict__ beta, const float* __restrict__ mean,
                          float* __restrict__ rstd, float* __restrict__ al, float* __restrict__ de,
                          Vol vol, int C) {
  const int bc = blockIdx.x * blockDim.x + threadIdx.x;
  if (bc >= vol.B * C) return;
  const int c = bc % C;
  double s = 0.0;
  for (int d = 0; d < vol.D; ++d) s += sq[(int64_t)bc * vol.D + d];
  const double var = s / ((double)vol.D * vol.H * vol.W);
  const float rs = (float)(1.0 / sqrt(var + 1e-5));
  rstd[bc] = rs;
  const float a = gamma[c] * rs;
  al[bc] = a;
  de[bc] = beta[c] - mean[bc] * a;
}

hipError_t in_mean(const float* sums, float* mean, Vol vol, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_in_mean, dim3(cdiv(vol.B * C, 256)), dim3(256), 0, s, sums, mean, vol, C);
  return hipGetLastError();
}

hipError_t in_rstd(const float* sq, const float* gamma, const float* beta, const float* mean,
                   float* rstd, float* al, float* de, Vol vol, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_in_rstd, dim3(cdiv(vol.B * C, 256)), dim3(256), 0, s, sq, gamma, beta,
                     mean, rstd, al, de, vol, C);
  return hipGetLastError();
}

// one wave per channel c: lanes take strided depths, fp64 shuffle tree per
// sample, samples summed in order (deterministic; short dependent chains --
// the per-(b, c, d) sums are tiny and this kernel is latency-bound)
__global__ __launch_bounds__(256) void k_in_bwd_stats(const float* __restrict__ sums,
                                                      float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta,
                                                      float* __restrict__ k1,
                                                      float* __restrict__ k2, Vol vol, int C) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const double N = (double)vol.D * vol.H * vol.W;
  double tg = 0.0, tb = 0.0;
  for (int b = 0; b < vol.B; ++b) {
    const int64_t bc = (int64_t)b * C + c;
    double s0 = 0.0, s1 = 0.0;
    for (int d = lane; d < vol.D; d += 64) {
      const float2 v = *reinterpret_cast<const float2*>(sums + (bc * vol.D + d) * 2);
      s0 += v.x;
      s1 += v.y;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
    if (lane == 0) {
      k1[bc] = (float)(s0 / N);
      k2[bc] = (float)(s1 / N);
    }
    tb += s0;
    tg += s1;
  }
  if (lane == 0) {
    if (dgamma) dgamma[c] = (float)tg;
    if (dbeta) dbeta[c] = (float)tb;
  }
}

hipError_t in_bwd_stats(const float* sums, const float* gamma, float* dgamma, float* dbeta,
                        float* k1, float* k2, Vol vol, int C, hipStream_t s) {
  (void)gamma;
  hipLaunchKernelGGL(k_in_bwd_stats, dim3(cdiv(C, 4)), dim3(256), 0, s, sums, dgamma, dbeta, k1,
                     k2, vol, C);
  return hipGetLastError();
}

// ---------------------------------------------- depth-sharded finalizers --
// A sharded plan's per-(b,c,d) sums cover its own D-slab only: they are
// reduced over d into fp64 partials, summed over the shard group (spff_coll
// allreduce) and then finalised with the GLOBAL voxel count.
__global__ void k_in_partial(const float* __restrict__ sums, double* __restrict__ part, Vol vol,
                             int C, int nq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (bc, q)
  if (i >= vol.B * C * nq) return;
  const int q = i % nq;
  const int64_t bc = i / nq;
  double s = 0.0;
  for (int d = 0; d < vol.D; ++d) s += sums[(bc * vol.D + d) * nq + q];
  part[i] = s;
}
__global__ void k_in_mean_fin(const double* __restrict__ part, float* __restrict__ mean, int BC,
                              double N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < BC) mean[i] = (float)(part[i] / N);
}
__global__ void k_in_rstd_fin(const double* __restrict__ part, const float* __restrict__ gamma,
                              const float* __restrict__ beta, const float* __restrict__ mean,
                              float* __restrict__ rstd, float* __restrict__ al,
                              float* __restrict__ de, int BC, int C, double N) {
  const int bc = blockIdx.x * blockDim.x + threadIdx.x;
  if (bc >= BC) return;
  const int c = bc % C;
  const float rs = (float)(1.0 / sqrt(part[bc] / N + 1e-5));
  rstd[bc] = rs;
  const float a = gamma[c] * rs;
  al[bc] = a;
  de[bc] = beta[c] - mean[bc] * a;
}
// gamma / beta gradients from the LOCAL partials (summed by the gradient all-reduce)
__global__ void k_in_bwd_dgb(const double* __restrict__ part, float* __restrict__ dgamma,
                             float* __restrict__ dbeta, int B, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double tg = 0.0, tb = 0.0;
  for (int b = 0; b < B; ++b) {
    tb += part[((int64_t)b * C + c) * 2 + 0];
    tg += part[((int64_t)b * C + c) * 2 + 1];
  }
  if (dgamma) dgamma[c] = (float)tg;
  if (dbeta) dbeta[c] = (float)tb;
}
__global__ void k_in_bwd_fin(const double* __restrict__ part, float* __restrict__ k1,
                             float* __restrict__ k2, int BC, double N) {
  const int bc = blockIdx.x * blockDim.x + threadIdx.x;
  if (bc >= BC) return;
  k1[bc] = (float)(part[2 * bc + 0] / N);
  k2[bc] = (float)(part[2 * bc + 1] / N);
}

hipError_t in_partial(const float* sums, double* part, Vol vol, int C, int nq, hipStream_t s) {
  hipLaunchKernelGGL(k_in_partial, dim3(cdiv(vol.B * C * nq, 256)), dim3(256), 0, s, sums, part,
                     vol, C, nq);
  return hipGetLastError();
}
hipError_t in_mean_fin(const double* part, float* mean, int BC, double N, hipStream_t s) {
  hipLaunchKernelGGL(k_in_mean_fin, dim3(cdiv(BC, 256)), dim3(256), 0, s, part, mean, BC, N);
  return hipGetLastError();
}
hipError_t in_rstd_fin(const double* part, const float* gamma, const float* beta,
                       const float* mean, float* rstd, float* al, float* de, int B, int C,
                       double N, hipStream_t s) {
  hipLaunchKernelGGL(k_in_rstd_fin, dim3(cdiv(B * C, 256)), dim3(256), 0, s, part, gamma, beta,
                     mean, rstd, al, de, B * C, C, N);
  return hipGetLastError();
}
hipError_t in_bwd_dgb(const double* part, float* dgamma, float* dbeta, int B, int C,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_in_bwd_dgb, dim3(cdiv(C, 64)), dim3(64), 0, s, part, dgamma, dbeta, B, C);
  return hipGetLastError();
}
hipError_t in_bwd_fin(const double* part, float* k1, float* k2, int BC, double N, hipStream_t s) {
  hipLaunchKernelGGL(k_in_bwd_fin, dim3(cdiv(BC, 256)), dim3(256), 0, s, part, k1, k2, BC, N);
  return hipGetLastError();
}

// ------------------------------------------------- BatchNorm3d finalizers --
// nn.BatchNorm3d(C) (reference Cicek3DUNet, models.py:718-724): the same
// per-(b,c,d) hw-sums, reduced over b AND d (N = B*D*H*W per channel).  The
// per-channel results are written replicated over b ([B][C]) so act_apply /
// in_bwd_apply / slab_reduce run unchanged.  fp64 accumulation over (b,d), as
// ATen's CPU batch norm accumulates in double.
__global__ void k_bn_mean(const float* __restrict__ sums, float* __restrict__ mean, Vol vol,
                          int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int b = 0; b < vol.B; ++b)
    for (int d = 0; d < vol.D; ++d) s += sums[((int64_t)b * C + c) * vol.D + d];
  const float m = (float)(s / ((double)vol.B * vol.D * vol.H * vol.W));
  for (int b = 0; b < vol.B; ++b) mean[b * C + c] = m;
}

// train: rstd/al/de from the squared-deviation sums; running stats updated
// in place (momentum m, unbiased variance), batch_norm_cpu_update_stats order
__global__ void k_bn_rstd(const float* __restrict__ sq, const float* __restrict__ gamma,
                          const float* __restrict__ beta, const float* __restrict__ mean,
                          float* __restrict__ rstd, float* __restrict__ al, float* __restrict__ de,
                          float* __restrict__ rmean, float* __restrict__ rvar, double mom,
                          double eps, Vol vol, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int b = 0; b < vol.B; ++b)
    for (int d = 0; d < vol.D; ++d) s += sq[((int64_t)b * C + c) * vol.D + d];
  const double N = (double)vol.B * vol.D * vol.H * vol.W;
  const double var = s / N;
  const float rs = (float)(1.0 / sqrt(var + eps));
  const float mu = mean[c];
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float a = g * rs;
  for (int b = 0; b < vol.B; ++b) {
    rstd[b * C + c] = rs;
    al[b * C + c] = a;
    de[b * C + c] = bt - mu * a;
  }
  if (rmean) {
    rmean[c] = (float)(mom * (double)mu + (1.0 - mom) * (double)rmean[c]);
    const double uv = N > 1.0 ? s / (N - 1.0) : var;
    rvar[c] = (float)(mom * uv + (1.0 - mom) * (double)rvar[c]);
  }
}

// eval: normalise with the running statistics
__global__ void k_bn_eval(const float* __restrict__ rmean, const float* __restrict__ rvar,
                          const float* __restrict__ gamma, const float* __restrict__ beta,
                          float* __restrict__ mean, float* __restrict__ rstd,
                          float* __restrict__ al, float* __restrict__ de, double eps, int B,
                          int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float rs = (float)(1.0 / sqrt((double)rvar[c] + eps));
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float a = g * rs;
  for (int b = 0; b < B; ++b) {
    mean[b * C + c] = rmean[c];
    rstd[b * C + c] = rs;
    al[b * C + c] = a;
    de[b * C + c] = bt - rmean[c] * a;
  }
}

// backward: from per-(b,c,d) [sum dr, sum dr*xhat] -> dgamma, dbeta and the
// batch means k1 = mean dr, k2 = mean dr*xhat (replicated over b)
__global__ void k_bn_bwd_stats(const float* __restrict__ sums, float* __restrict__ dgamma,
                               float* __restrict__ dbeta, float* __restrict__ k1,
                               float* __restrict__ k2, Vol vol, int C, int eval) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  for (int b = 0; b < vol.B; ++b)
    for (int d = 0; d < vol.D; ++d) {
      const int64_t i = (((int64_t)b * C + c) * vol.D + d) * 2;
      s0 += sums[i];
      s1 += sums[i + 1];
    }
  const double N = (double)vol.B * vol.D * vol.H * vol.W;
  for (int b = 0; b < vol.B; ++b) {
    k1[b * C + c] = eval ? 0.f : (float)(s0 / N);
    k2[b * C + c] = eval ? 0.f : (float)(s1 / N);
  }
  if (dgamma) dgamma[c] = (float)s1;
  if (dbeta) dbeta[c] = (float)s0;
}

// ---- SyncBatchNorm: the same per-channel fp64 sums, over the data-parallel group ----
__global__ void k_bn_partial(const float* __restrict__ sums, double* __restrict__ part, Vol vol,
                             int C, int nq) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  for (int q = 0; q < nq; ++q) {
    double s = 0.0;
    for (int b = 0; b < vol.B; ++b)
      for (int d = 0; d < vol.D; ++d) s += sums[(((int64_t)b * C + c) * vol.D + d) * nq + q];
    part[(int64_t)q * C + c] = s;
  }
}
__global__ void k_bn_mean_fin(const double* __restrict__ part, float* __restrict__ mean, int B,
                              int C, double N) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float m = (float)(part[c] / N);
  for (int b = 0; b < B; ++b) mean[b * C + c] = m;
}
__global__ void k_bn_rstd_fin(const double* __restrict__ part, const float* __restrict__ gamma,
                              const float* __restrict__ beta, const float* __restrict__ mean,
                              float* __restrict__ rstd, float* __restrict__ al,
                              float* __restrict__ de, float* __restrict__ rmean,
                              float* __restrict__ rvar, double mom, double eps, int B, int C,
                              double N) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double s = part[c];
  const double var = s / N;
  const float rs = (float)(1.0 / sqrt(var + eps));
  const float mu = mean[c];
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float a = g * rs;
  for (int b = 0; b < B; ++b) {
    rstd[b * C + c] = rs;
    al[b * C + c] = a;
    de[b * C + c] = bt - mu * a;
  }
  if (rmean) {
    rmean[c] = (float)(mom * (double)mu + (1.0 - mom) * (double)rmean[c]);
    const double uv = N > 1.0 ? s / (N - 1.0) : var;
    rvar[c] = (float)(mom * uv + (1.0 - mom) * (double)rvar[c]);
  }
}
__global__ void k_bn_bwd_dgb_part(const double* __restrict__ part, float* __restrict__ dgamma,
                                  float* __restrict__ dbeta, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] = (float)part[C + c];
  if (dbeta) dbeta[c] = (float)part[c];
}
__global__ void k_bn_bwd_fin(const double* __restrict__ part, float* __restrict__ k1,
                             float* __restrict__ k2, int B, int C, double N) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float a = (float)(part[c] / N), b2 = (float)(part[C + c] / N);
  for (int b = 0; b < B; ++b) {
    k1[b * C + c] = a;
    k2[b * C + c] = b2;
  }
}
hipError_t bn_partial(const float* sums, double* part, Vol vol, int C, int nq, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_partial, dim3(cdiv(C, 64)), dim3(64), 0, s, sums, part, vol, C, nq);
  return hipGetLastError();
}
hipError_t bn_mean_fin(const double* part, float* mean, int B, int C, double N, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_mean_fin, dim3(cdiv(C, 64)), dim3(64), 0, s, part, mean, B, C, N);
  return hipGetLastError();
}
hipError_t bn_rstd_fin(const double* part, const float* gamma, const float* beta,
                       const float* mean, float* rstd, float* al, float* de, float* rmean,
                       float* rvar, double mom, double eps, int B, int C, double N, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_rstd_fin, dim3(cdiv(C, 64)), dim3(64), 0, s, part, gamma, beta, mean,
                     rstd, al, de, rmean, rvar, mom, eps, B, C, N);
  return hipGetLastError();
}
hipError_t bn_bwd_dgb_part(const double* part, float* dgamma, float* dbeta, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_bwd_dgb_part, dim3(cdiv(C, 64)), dim3(64), 0, s, part, dgamma, dbeta, C);
  return hipGetLastError();
}
hipError_t bn_bwd_fin(const double* part, float* k1, float* k2, int B, int C, double N,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_bn_bwd_fin, dim3(cdiv(C, 64)), dim3(64), 0, s, part, k1, k2, B, C, N);
  return hipGetLastError();
}

hipError_t bn_mean(const float* sums, float* mean, Vol vol, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_mean, dim3(cdiv(C, 64)), dim3(64), 0, s, sums, mean, vol, C);
  return hipGetLastError();
}
hipError_t bn_rstd(const float* sq, const float* gamma, const float* beta, const float* mean,
                   float* rstd, float* al, float* de, float* rmean, float* rvar, double mom,
                   double eps, Vol vol, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_rstd, dim3(cdiv(C, 64)), dim3(64), 0, s, sq, gamma, beta, mean, rstd,
                     al, de, rmean, rvar, mom, eps, vol, C);
  return hipGetLastError();
}
hipError_t bn_eval(const float* rmean, const float* rvar, const float* gamma, const float* beta,
                   float* mean, float* rstd, float* al, float* de, double eps, int B, int C,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_bn_eval, dim3(cdiv(C, 64)), dim3(64), 0, s, rmean, rvar, gamma, beta, mean,
                     rstd, al, de, eps, B, C);
  return hipGetLastError();
}
hipError_t bn_bwd_stats(const float* sums, float* dgamma, float* dbeta, float* k1, float* k2,
                        Vol vol, int C, hipStream_t s, int eval) {
  hipLaunchKernelGGL(k_bn_bwd_stats, dim3(cdiv(C, 64)), dim3(64), 0, s, sums, dgamma, dbeta, k1,
                     k2, vol, C, eval);
  return hipGetLastError();
}

// ------------------------------------------------------------ elementwise --
// grid.y = b*D + d ; grid.x strides over the (h,w,c/4) float4s of that slab.
// The stride (gridDim.x * ew_bs(C)) is a multiple of C/4 (C/4 <= 64),
// so a thread's channel quad is fixed: its per-(b,c[,d]) parameters are loaded
// once into registers, and the loop is pure float4 streaming.
__global__ __launch_bounds__(256) void k_act_apply(const float* __restrict__ y, float* __restrict__ out,
                                                   const float* __restrict__ al, const float* __restrict__ de,
                                                   const float* __restrict__ P, const float* __restrict__ Q,
                                                   Vol vol, int C, float neg, unsigned* __restrict__ amax) {
  const int bd = blockIdx.y, b = bd / vol.D, d = bd % vol.D;
  const int n4 = vol.H * vol.W * (C >> 2);
  const int64_t base = (int64_t)bd * vol.H * vol.W * C;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (i0 % (C >> 2)) * 4;
  float pa[4], pd[4], pp[4], pq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bc = b * C + c + j;
    pa[j] = al[bc];
    pd[j] = de[bc];
    pp[j] = P ? P[(int64_t)bc * vol.D + d] : 1.f;
    pq[j] = P ? Q[(int64_t)bc * vol.D + d] : 0.f;
  }
  float m = 0.f;
  for (int i = i0; i < n4; i += gridDim.x * blockDim.x) {
    const float4 v = ld_s(y + base + 4 * (int64_t)i);
    float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = lrelu(r[j] * pa[j] + pd[j], neg) * pp[j] + pq[j];
      m = fmaxf(m, fabsf(r[j]));
    }
    st_s(out + base + 4 * (int64_t)i, make_float4(r[0], r[1], r[2], r[3]));
  }
  if (amax) block_amax(m, amax);
}

// Blocks per slab: SPFF_EW_GX, raised to reach SPFF_EW_MINWG workgroups in all, at most
// one float4 per thread.  Any count keeps a thread's channel quad fixed (see above).
static int ew_gx(int n4, int C, int slabs) {
  const int want = std::max(SPFF_EW_GX, cdiv(SPFF_EW_MINWG, std::max(slabs, 1)));
  return std::max(1, std::min(cdiv(n4, ew_bs(C)), want));
}

static dim3 ew_grid(Vol vol, int C) {
  const int n4 = vol.H * vol.W * (C / 4);
  return dim3(ew_gx(n4, C, vol.B * vol.D), vol.B * vol.D);
}

hipError_t act_apply(const float* y, float* out, const float* al, const float* de, const float* P,
                     const float* Q, Vol vol, int C, hipStream_t s, float neg, unsigned* amax) {
  hipLaunchKernelGGL(k_act_apply, ew_grid(vol, C), dim3(ew_bs(C)), 0, s, y, out, al, de, P, Q, vol, C,
                     neg, amax);
  return hipGetLastError();
}

// An encoder block's output apply fused with the MaxPool3d((1,2,2)) that consumes it
// (models.py:661-665): per 2 x 2 window and channel quad, the four out = lrelu(y2 al + de)
// P + Q are written (the decoder's skip source) and their max and first-max index
// (k = 2 dh + dw, scan order, NaN wins: k_maxpool_fwd's rule) -- the pool never re-reads
// the block output.  H and W even (the caller falls back to act_apply + maxpool_fwd).
// grid.y = b D + d, grid.x strides over the slab's pooled (ho, wo, c/4).
__global__ __launch_bounds__(256) void k_act_apply_pool(
    const float* __restrict__ y, float* __restrict__ out, const float* __restrict__ al,
    const float* __restrict__ de, const float* __restrict__ P, const float* __restrict__ Q,
    float* __restrict__ pooled, uint8_t* __restrict__ idx, Vol vol, int C, float neg,
    unsigned* __restrict__ amax) {
  const int bd = blockIdx.y, b = bd / vol.D, d = bd % vol.D;
  const int Ho = vol.H / 2, Wo = vol.W / 2, C4 = C >> 2;
  const int n4 = Ho * Wo * C4;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (i0 % C4) * 4;
  float pa[4], pd[4], pp[4], pq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bc = b * C + c + j;
    pa[j] = al[bc];
    pd[j] = de[bc];
    pp[j] = P ? P[(int64_t)bc * vol.D + d] : 1.f;
    pq[j] = P ? Q[(int64_t)bc * vol.D + d] : 0.f;
  }
  float m = 0.f;  // max |out| (>= max |pooled|: the pool selects elements of out)
  for (int i = i0; i < n4; i += gridDim.x * blockDim.x) {
    const int q = i / C4, wo = q % Wo, ho = q / Wo;
    const int64_t vin = ((int64_t)bd * vol.H + 2 * ho) * vol.W + 2 * wo;
    float best[4];
    uint8_t bi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t vv = vin + (k >> 1) * vol.W + (k & 1);
      const float4 v = ld_s(y + vv * C + c);
      float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        r[j] = lrelu(r[j] * pa[j] + pd[j], neg) * pp[j] + pq[j];
        m = fmaxf(m, fabsf(r[j]));
        if (k == 0) {
          best[j] = r[j];
        } else if (r[j] > best[j] || isnan(r[j])) {
          best[j] = r[j];
          bi[j] = (uint8_t)k;
        }
      }
      st_s(out + vv * C + c, make_float4(r[0], r[1], r[2], r[3]));
    }
    const int64_t vo = ((int64_t)bd * Ho + ho) * Wo + wo;
    *reinterpret_cast<float4*>(pooled + vo * C + c) = make_float4(best[0], best[1], best[2], best[3]);
    *reinterpret_cast<uchar4*>(idx + vo * C + c) = make_uchar4(bi[0], bi[1], bi[2], bi[3]);
  }
  if (amax) block_amax(m, amax);
}

hipError_t act_apply_pool(const float* y, float* out, const float* al, const float* de,
                          const float* P, const float* Q, float* pooled, uint8_t* idx, Vol vol,
                          int C, hipStream_t s, float neg, unsigned* amax) {
  if ((vol.H | vol.W) & 1 || C % 4) return hipErrorInvalidValue;
  const int n4 = (vol.H / 2) * (vol.W / 2) * (C / 4);
  const dim3 grid(ew_gx(n4, C, vol.B * vol.D), vol.B * vol.D);
  hipLaunchKernelGGL(k_act_apply_pool, grid, dim3(ew_bs(C)), 0, s, y, out, al, de, P, Q, pooled,
                     idx, vol, C, neg, amax);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_in_bwd_apply(
    const float* __restrict__ y, const float* g, float* dy, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ al, const float* __restrict__ de,
    const float* __restrict__ gamma, const float* __restrict__ A, const float* __restrict__ Bc,
    const float* __restrict__ k1, const float* __restrict__ k2, Vol vol, int C, float neg,
    unsigned* __restrict__ amax, PoolAdd pa) {
  const int bd = blockIdx.y, b = bd / vol.D, d = bd % vol.D;
  const int n4 = vol.H * vol.W * (C >> 2);
  const int64_t base = (int64_t)bd * vol.H * vol.W * C;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (i0 % (C >> 2)) * 4;
  float pal[4], pde[4], pmu[4], prs[4], psc[4], pk1[4], pk2[4], pA[4], pB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bc = b * C + c + j;
    pal[j] = al[bc]; pde[j] = de[bc]; pmu[j] = mean[bc]; prs[j] = rstd[bc];
    psc[j] = rstd[bc] * gamma[c + j]; pk1[j] = k1[bc]; pk2[j] = k2[bc];
    pA[j] = A ? A[(int64_t)bc * vol.D + d] : 1.f;
    pB[j] = A ? Bc[(int64_t)bc * vol.D + d] : 0.f;
  }
  float m = 0.f;
  for (int i = i0; i < n4; i += gridDim.x * blockDim.x) {
    const float4 yv = ld_s(y + base + 4 * (int64_t)i);
    float4 gv = ld_s(g + base + 4 * (int64_t)i);
    if (pa.dp) gv = pool_add(gv, pa, bd, i / (C >> 2), vol, C, c);
    const float ys[4] = {yv.x, yv.y, yv.z, yv.w};
    const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float r = ys[j] * pal[j] + pde[j];
      const float dr = (gs[j] * pA[j] + pB[j]) * slope(r, neg);
      const float xh = (ys[j] - pmu[j]) * prs[j];
      o[j] = psc[j] * (dr - pk1[j] - xh * pk2[j]);
      m = fmaxf(m, fabsf(o[j]));
    }
    st_s(dy + base + 4 * (int64_t)i, make_float4(o[0], o[1], o[2], o[3]));
  }
  if (amax) block_amax(m, amax);
}

__global__ __launch_bounds__(256) void k_act_bound(const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int C,
                                                   float sq, unsigned* __restrict__ slot) {
  __shared__ float rg[256], rb[256];
  float mg = 0.f, mb = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    mg = fmaxf(mg, fabsf(gamma[c]));
    mb = fmaxf(mb, fabsf(beta[c]));
  }
  rg[threadIdx.x] = mg;
  rb[threadIdx.x] = mb;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      rg[threadIdx.x] = fmaxf(rg[threadIdx.x], rg[threadIdx.x + st]);
      rb[threadIdx.x] = fmaxf(rb[threadIdx.x], rb[threadIdx.x + st]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *slot = __float_as_uint(2.f * (rg[0] * sq + rb[0]) + 1e-30f);
}

hipError_t act_bound(const float* gamma, const float* beta, int C, double N, unsigned* slot,
                     hipStream_t s) {
  const float sq = (float)std::sqrt(std::max(N - 1.0, 1.0));
  hipLaunchKernelGGL(k_act_bound, dim3(1), dim3(256), 0, s, gamma, beta, C, sq, slot);
  return hipGetLastError();
}

hipError_t in_bwd_apply(const float* y, const float* g, float* dy, const float* mean,
                        const float* rstd, const float* al, const float* de, const float* gamma,
                        const float* A, const float* Bc, const float* k1, const float* k2, Vol vol,
                        int C, hipStream_t s, float neg, unsigned* amax, PoolAdd pa) {
  hipLaunchKernelGGL(k_in_bwd_apply, ew_grid(vol, C), dim3(ew_bs(C)), 0, s, y, g, dy, mean, rstd, al,
                     de, gamma, A, Bc, k1, k2, vol, C, neg, amax, pa);
  return hipGetLastError();
}

}  // namespace spff
