// Row-wise and elementwise kernels of the SwinUNETR variant (swin.hip): layer
// norm (Swin blocks, patch merging, proj_out), the legacy PatchMerging gather /
// scatter, the UnetResBlock residual + LeakyReLU, and the soft-Dice + CE loss of
// LitSwinUNETR_Published.  Semantics: oracle/swin_oracle.py (MONAI 1.5.2,
// parity unpinned).  All HBM-bound; reductions are fixed-order (wave shuffles,
// then per-block partials summed in order) so every result is deterministic.
#include "spff_internal.h"
#include "swin_internal.h"

#include <math.h>

namespace spff {

namespace {
inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// legacy PatchMerging slice offsets (d, h, w) of cat slot q (MONAI's x0..x7)
__device__ __forceinline__ void merge_off(int q, int& od, int& oh, int& ow) {
  // (0,0,0),(1,0,0),(0,1,0),(0,0,1),(1,0,1),(0,1,0),(0,0,1),(1,1,1)
  constexpr int tab = (0 << 0) | (4 << 3) | (2 << 6) | (1 << 9) | (5 << 12) | (2 << 15) |
                      (1 << 18) | (7 << 21);
  const int t = (tab >> (3 * q)) & 7;
  od = t >> 2; oh = (t >> 1) & 1; ow = t & 1;
}

// row geometry of a layer-norm input: MODE 0 = rows x[m*ldx + c];
// MODE 1 = the merge gather: coarse row m of [B][D/2][H/2][W/2], channel
// c = q*Cf + cf read from the fine grid x[B][D][H][W][Cf]
struct LnSrc {
  const float* x; int ldx, Cf, D, H, W;
};
// split into a per-row base and a per-channel offset so the (64-bit) row
// decomposition runs once per row, not once per element
template <int MODE>
__device__ __forceinline__ int64_t ln_base(const LnSrc& s, int64_t m) {
  if (MODE == 0) return m * s.ldx;
  const int Wl = s.W >> 1, Hl = s.H >> 1, Dl = s.D >> 1;
  int64_t t = m;
  const int w = (int)(t % Wl); t /= Wl;
  const int h = (int)(t % Hl); t /= Hl;
  const int d = (int)(t % Dl);
  const int64_t b = t / Dl;
  return (((b * s.D + 2 * d) * s.H + 2 * h) * (int64_t)s.W + 2 * w) * s.Cf;
}
template <int MODE>
__device__ __forceinline__ int64_t ln_off(const LnSrc& s, int c) {
  if (MODE == 0) return c;
  const int q = c / s.Cf, cf = c - q * s.Cf;
  int od, oh, ow;
  merge_off(q, od, oh, ow);
  return ((int64_t)(od * s.H + oh) * s.W + ow) * s.Cf + cf;
}
constexpr int LN_NJ = 12;  // channels per lane: C <= 768
}  // namespace

// one wave per row: y = (x - mean) * rstd * g + b  (g, b null: no affine)
template <int MODE>
__global__ __launch_bounds__(256) void k_ln_fwd(LnSrc src, int C, const float* __restrict__ g,
                                                const float* __restrict__ bta, float* __restrict__ y,
                                                int ldy, float* __restrict__ mu,
                                                float* __restrict__ rs, int64_t M) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float v[LN_NJ];
  float s = 0.f;
  const float* xr = src.x + ln_base<MODE>(src, m);
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? xr[ln_off<MODE>(src, c)] : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) {
    const int c = lane + 64 * j;
    const float dl = c < C ? v[j] - mean : 0.f;
    q += dl * dl;
  }
  const float rstd = 1.f / sqrtf(wave_sum(q) / (float)C + 1e-5f);
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < C) {
      float o = (v[j] - mean) * rstd;
      if (g) o = o * g[c] + bta[c];
      y[m * ldy + c] = o;
    }
  }
  if (lane == 0) {
    mu[m] = mean;
    rs[m] = rstd;
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)) [+ res]; per-block
// partial sums of dy*xhat and dy (dgamma, dbeta) over the block's rows
// rows per block: a multiple of the 4 waves, shrunk (as a function of M only,
// so the partial-sum order stays fixed) until the grid has >= 4096 blocks
inline int ln_rpb(int64_t M) {
  int r = 128;
  while (r > 8 && cdiv64(M, r) < 4096) r >>= 1;
  return r;
}
template <int MODE>
__global__ __launch_bounds__(256) void k_ln_bwd(LnSrc src, int C, const float* __restrict__ g,
                                                const float* __restrict__ mu,
                                                const float* __restrict__ rs,
                                                const float* __restrict__ dy, int lddy,
                                                float* __restrict__ dx, int lddx,
                                                const float* __restrict__ res, int ldres,
                                                float* __restrict__ part, int64_t M,
                                                int rpb) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[LN_NJ], pb[LN_NJ];
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) pg[j] = pb[j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  int64_t off[LN_NJ];
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) {
    const int c = lane + 64 * j;
    off[j] = c < C ? ln_off<MODE>(src, c) : 0;
  }
  for (int rr = wave; rr < rpb; rr += 4) {
    const int64_t m = r0 + rr;
    if (m >= M) break;
    const float mean = mu[m], rstd = rs[m];
    const float* xr = src.x + ln_base<MODE>(src, m);
    float xh[LN_NJ], gd[LN_NJ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < LN_NJ; ++j) {
      const int c = lane + 64 * j;
      xh[j] = 0.f; gd[j] = 0.f;
      if (c < C) {
        const float d = dy[m * lddy + c];
        xh[j] = (xr[off[j]] - mean) * rstd;
        gd[j] = g ? d * g[c] : d;
        pg[j] += d * xh[j];
        pb[j] += d;
      }
      s1 += gd[j];
      s2 += gd[j] * xh[j];
    }
    const float c1 = wave_sum(s1) / (float)C, c2 = wave_sum(s2) / (float)C;
#pragma unroll
    for (int j = 0; j < LN_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < C) {
        float o = rstd * (gd[j] - c1 - xh[j] * c2);
        if (res) o += res[m * ldres + c];
        dx[m * lddx + c] = o;
      }
    }
  }
  if (!part) return;
  __shared__ float red[4][2][64 * LN_NJ];
#pragma unroll
  for (int j = 0; j < LN_NJ; ++j) {
    red[wave][0][lane + 64 * j] = pg[j];
    red[wave][1][lane + 64 * j] = pb[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int qq = i / C, c = i - qq * C;
    const float t = ((red[0][qq][c] + red[1][qq][c]) + red[2][qq][c]) + red[3][qq][c];
    part[((int64_t)blockIdx.x * 2 + qq) * C + c] = t;
  }
}

// Narrow rows (C = 12, 24: the first Swin stages): one THREAD per row, the row in
// registers (float4 loads), no cross-lane reductions; 64 lanes cover 64 rows.
template <int C>
__global__ __launch_bounds__(256) void k_ln_fwd_t(const float* __restrict__ x, int ldx,
                                                  const float* __restrict__ g,
                                                  const float* __restrict__ bta,
                                                  float* __restrict__ y, int ldy,
                                                  float* __restrict__ mu, float* __restrict__ rs,
                                                  int64_t M) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float v[C];
#pragma unroll
  for (int c = 0; c < C; c += 4) {
    const float4 t = *reinterpret_cast<const float4*>(x + m * ldx + c);
    v[c] = t.x; v[c + 1] = t.y; v[c + 2] = t.z; v[c + 3] = t.w;
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) s += v[c];
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) q += (v[c] - mean) * (v[c] - mean);
  const float rstd = 1.f / sqrtf(q / (float)C + 1e-5f);
#pragma unroll
  for (int c = 0; c < C; c += 4) {
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = (v[c + k] - mean) * rstd;
      if (g) o[k] = o[k] * g[c + k] + bta[c + k];
    }
    *reinterpret_cast<float4*>(y + m * ldy + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
  mu[m] = mean;
  rs[m] = rstd;
}

constexpr int LNT_R = 8;  // rows per thread (strided by 256): 2048 rows per block
template <int C>
__global__ __launch_bounds__(256) void k_ln_bwd_t(const float* __restrict__ x, int ldx,
                                                  const float* __restrict__ g,
                                                  const float* __restrict__ mu,
                                                  const float* __restrict__ rs,
                                                  const float* __restrict__ dy, int lddy,
                                                  float* __restrict__ dx, int lddx,
                                                  const float* __restrict__ res, int ldres,
                                                  float* __restrict__ part, int64_t M) {
  float pg[C], pb[C];
#pragma unroll
  for (int c = 0; c < C; ++c) pg[c] = pb[c] = 0.f;
  for (int r = 0; r < LNT_R; ++r) {
    const int64_t m = (int64_t)blockIdx.x * 256 * LNT_R + r * 256 + threadIdx.x;
    if (m >= M) break;
    const float mean = mu[m], rstd = rs[m];
    float xh[C], gd[C];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C; c += 4) {
      const float4 tx = *reinterpret_cast<const float4*>(x + m * ldx + c);
      const float4 td = *reinterpret_cast<const float4*>(dy + m * lddy + c);
      const float xv[4] = {tx.x, tx.y, tx.z, tx.w}, dv[4] = {td.x, td.y, td.z, td.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[c + k] = (xv[k] - mean) * rstd;
        gd[c + k] = g ? dv[k] * g[c + k] : dv[k];
        pg[c + k] += dv[k] * xh[c + k];
        pb[c + k] += dv[k];
        s1 += gd[c + k];
        s2 += gd[c + k] * xh[c + k];
      }
    }
    const float c1 = s1 / (float)C, c2 = s2 / (float)C;
#pragma unroll
    for (int c = 0; c < C; c += 4) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rstd * (gd[c + k] - c1 - xh[c + k] * c2);
      if (res) {
        const float4 t = *reinterpret_cast<const float4*>(res + m * ldres + c);
        o[0] += t.x; o[1] += t.y; o[2] += t.z; o[3] += t.w;
      }
      *reinterpret_cast<float4*>(dx + m * lddx + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  if (!part) return;
  __shared__ float red[2 * C][257];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    red[c][threadIdx.x] = pg[c];
    red[C + c][threadIdx.x] = pb[c];
  }
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int i = 0; i < 2 * C; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x < 2 * C) part[(int64_t)blockIdx.x * 2 * C + threadIdx.x] = red[threadIdx.x][0];
}

// out[i] (+)= sum over k < n of part[k*stride + i] (i < count): one workgroup per
// column, each thread a strided partial sum over k, then a fixed LDS tree --
// deterministic, and parallel over k (n runs to thousands of blocks / windows).
// map = 1: out index of column i = (i % R) * nh + i / R (bias-table transpose);
// map = 2: i = h*2hd + e2 -> C + h*hd + e2 (k part) or 2C + h*hd + e2 - hd (v part).
struct ColMap {
  int mode, R, nh, hd, C;
};
__global__ __launch_bounds__(256) void k_col_reduce(const float* __restrict__ part, int n,
                                                    int64_t stride, float* __restrict__ out,
                                                    int acc, ColMap mp) {
  const int i = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < n; k += 256) s += part[(int64_t)k * stride + i];
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x) return;
  int o = i;
  if (mp.mode == 1) {
    o = (i % mp.R) * mp.nh + i / mp.R;
  } else if (mp.mode == 2) {
    const int h = i / (2 * mp.hd), e2 = i % (2 * mp.hd);
    o = e2 < mp.hd ? mp.C + h * mp.hd + e2 : 2 * mp.C + h * mp.hd + (e2 - mp.hd);
  }
  out[o] = acc ? out[o] + red[0] : red[0];
}

hipError_t col_reduce_map(const float* part, int n, int64_t stride, int count, float* out,
                          int acc, int mode, int R, int nh, int hd, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_col_reduce, dim3(count), dim3(256), 0, s, part, n, stride, out, acc,
                     ColMap{mode, R, nh, hd, C});
  return hipGetLastError();
}

hipError_t col_reduce(const float* part, int n, int64_t stride, int count, float* out, int acc,
                      hipStream_t s) {
  return col_reduce_map(part, n, stride, count, out, acc, 0, 1, 1, 1, 0, s);
}

hipError_t ln_fwd(const float* x, int ldx, int C, const float* g, const float* b, float* y,
                  int ldy, float* mu, float* rs, int64_t M, hipStream_t s) {
  if (C > 64 * LN_NJ) return hipErrorInvalidValue;
  const bool vec = ldx % 4 == 0 && ldy % 4 == 0;
  if (vec && (C == 12 || C == 24)) {
    const dim3 gr((unsigned)cdiv64(M, 256));
    if (C == 12)
      hipLaunchKernelGGL(k_ln_fwd_t<12>, gr, dim3(256), 0, s, x, ldx, g, b, y, ldy, mu, rs, M);
    else
      hipLaunchKernelGGL(k_ln_fwd_t<24>, gr, dim3(256), 0, s, x, ldx, g, b, y, ldy, mu, rs, M);
    return hipGetLastError();
  }
  LnSrc src{x, ldx, C, 0, 0, 0};
  hipLaunchKernelGGL(k_ln_fwd<0>, dim3((unsigned)cdiv64(M, 4)), dim3(256), 0, s, src, C, g, b, y,
                     ldy, mu, rs, M);
  return hipGetLastError();
}

hipError_t ln_merge_fwd(const float* xf, int Cf, int B, int D, int H, int W, const float* g,
                        const float* b, float* y, float* mu, float* rs, hipStream_t s) {
  const int C = 8 * Cf;
  if (C > 64 * LN_NJ || D % 2 || H % 2 || W % 2) return hipErrorInvalidValue;
  const int64_t M = (int64_t)B * (D / 2) * (H / 2) * (W / 2);
  LnSrc src{xf, Cf, Cf, D, H, W};
  hipLaunchKernelGGL(k_ln_fwd<1>, dim3((unsigned)cdiv64(M, 4)), dim3(256), 0, s, src, C, g, b, y,
                     C, mu, rs, M);
  return hipGetLastError();
}

size_t ln_bwd_ws_bytes(int64_t M, int C) {
  return (size_t)std::max(cdiv64(M, ln_rpb(M)), cdiv64(M, 256 * LNT_R)) * 2 * C * sizeof(float);
}

// dgb (may be null): [2][C] = dgamma, dbeta (written)
hipError_t ln_bwd(const float* x, int ldx, int C, const float* g, const float* mu,
                  const float* rs, const float* dy, int lddy, float* dx, int lddx,
                  const float* res, int ldres, float* dgb, float* ws, int64_t M, hipStream_t s) {
  if (C > 64 * LN_NJ) return hipErrorInvalidValue;
  const bool vec = ldx % 4 == 0 && lddy % 4 == 0 && lddx % 4 == 0 && (!res || ldres % 4 == 0);
  if (vec && (C == 12 || C == 24)) {
    const int64_t nbt = cdiv64(M, 256 * LNT_R);
    float* pt = dgb ? ws : nullptr;
    if (C == 12)
      hipLaunchKernelGGL(k_ln_bwd_t<12>, dim3((unsigned)nbt), dim3(256), 0, s, x, ldx, g, mu, rs,
                         dy, lddy, dx, lddx, res, ldres, pt, M);
    else
      hipLaunchKernelGGL(k_ln_bwd_t<24>, dim3((unsigned)nbt), dim3(256), 0, s, x, ldx, g, mu, rs,
                         dy, lddy, dx, lddx, res, ldres, pt, M);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !dgb) return e;
    return col_reduce(ws, (int)nbt, 2 * C, 2 * C, dgb, 0, s);
  }
  LnSrc src{x, ldx, C, 0, 0, 0};
  const int rpb = ln_rpb(M);
  const int64_t nb = cdiv64(M, rpb);
  hipLaunchKernelGGL(k_ln_bwd<0>, dim3((unsigned)nb), dim3(256), 0, s, src, C, g, mu, rs, dy, lddy,
                     dx, lddx, res, ldres, dgb ? ws : nullptr, M, rpb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !dgb) return e;
  return col_reduce(ws, (int)nb, 2 * C, 2 * C, dgb, 0, s);
}

hipError_t ln_merge_bwd(const float* xf, int Cf, int B, int D, int H, int W, const float* g,
                        const float* mu, const float* rs, const float* dy, float* dcat, float* dgb,
                        float* ws, hipStream_t s) {
  const int C = 8 * Cf;
  const int64_t M = (int64_t)B * (D / 2) * (H / 2) * (W / 2);
  LnSrc src{xf, Cf, Cf, D, H, W};
  const int rpb = ln_rpb(M);
  const int64_t nb = cdiv64(M, rpb);
  hipLaunchKernelGGL(k_ln_bwd<1>, dim3((unsigned)nb), dim3(256), 0, s, src, C, g, mu, rs, dy, C,
                     dcat, C, nullptr, 0, ws, M, rpb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return col_reduce(ws, (int)nb, 2 * C, 2 * C, dgb, 0, s);
}

// gradient of the merge gather: fine token (b, d, h, w) channel cf receives every
// cat slot q whose offset equals its parity (two for (0,1,0) / (0,0,1), none for
// (1,1,0) / (0,1,1))
__global__ void k_unmerge(const float* __restrict__ dcat, int Cf, int B, int D, int H, int W,
                          float* __restrict__ dxf, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cf = (int)(i % Cf);
    int64_t t = i / Cf;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H); t /= H;
    const int d = (int)(t % D);
    const int64_t b = t / D;
    const int64_t m = ((b * (D / 2) + d / 2) * (H / 2) + h / 2) * (int64_t)(W / 2) + w / 2;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int od, oh, ow;
      merge_off(q, od, oh, ow);
      if (od == (d & 1) && oh == (h & 1) && ow == (w & 1)) s += dcat[m * (8 * Cf) + q * Cf + cf];
    }
    dxf[i] = s;
  }
}

hipError_t unmerge(const float* dcat, int Cf, int B, int D, int H, int W, float* dxf,
                   hipStream_t s) {
  const int64_t total = (int64_t)B * D * H * W * Cf;
  hipLaunchKernelGGL(k_unmerge, dim3((unsigned)std::min<int64_t>(cdiv64(total, 256), 16384)),
                     dim3(256), 0, s, dcat, Cf, B, D, H, W, dxf, total);
  return hipGetLastError();
}

// ----------------------------------------------------- UnetResBlock tail --
// z = y2*al2[b,c] + de2[b,c] + (y3 ? y3*al3 + de3 : r);  out = lrelu(z)
// bwd: dz = dout * slope(z)
template <bool BWD>
__global__ __launch_bounds__(256) void k_res_act(const float* __restrict__ y2,
                                                 const float* __restrict__ al2,
                                                 const float* __restrict__ de2,
                                                 const float* __restrict__ y3,
                                                 const float* __restrict__ al3,
                                                 const float* __restrict__ de3,
                                                 const float* __restrict__ r,
                                                 const float* __restrict__ dout,
                                                 float* __restrict__ out, int C, int64_t vps,
                                                 int64_t n4) {
  const int C4 = C >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const int64_t v = i / C4;
    const int b = (int)(v / vps);
    const float4 a = *reinterpret_cast<const float4*>(y2 + 4 * i);
    const float4 q = y3 ? *reinterpret_cast<const float4*>(y3 + 4 * i)
                        : *reinterpret_cast<const float4*>(r + 4 * i);
    const float av[4] = {a.x, a.y, a.z, a.w}, qv[4] = {q.x, q.y, q.z, q.w};
    float o[4];
    float4 gd = make_float4(0.f, 0.f, 0.f, 0.f);
    if (BWD) gd = *reinterpret_cast<const float4*>(dout + 4 * i);
    const float gv[4] = {gd.x, gd.y, gd.z, gd.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int bc = b * C + c + j;
      float z = av[j] * al2[bc] + de2[bc];
      z += y3 ? qv[j] * al3[bc] + de3[bc] : qv[j];
      o[j] = BWD ? (z > 0.f ? gv[j] : 0.01f * gv[j]) : (z > 0.f ? z : 0.01f * z);
    }
    *reinterpret_cast<float4*>(out + 4 * i) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

hipError_t res_act(const float* y2, const float* al2, const float* de2, const float* y3,
                   const float* al3, const float* de3, const float* r, const float* dout,
                   float* out, Vol v, int C, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int64_t n4 = nvox(v) * C / 4, vps = (int64_t)v.D * v.H * v.W;
  const dim3 g((unsigned)std::min<int64_t>(cdiv64(n4, 256), 16384));
  if (dout)
    hipLaunchKernelGGL(k_res_act<true>, g, dim3(256), 0, s, y2, al2, de2, y3, al3, de3, r, dout,
                       out, C, vps, n4);
  else
    hipLaunchKernelGGL(k_res_act<false>, g, dim3(256), 0, s, y2, al2, de2, y3, al3, de3, r, dout,
                       out, C, vps, n4);
  return hipGetLastError();
}

// y += x (elementwise, n floats)
__global__ void k_add(float* __restrict__ y, const float* __restrict__ x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] += x[i];
}
hipError_t add_inplace(float* y, const float* x, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_add, dim3((unsigned)std::min<int64_t>(cdiv64(n, 256), 16384)), dim3(256), 0,
                     s, y, x, n);
  return hipGetLastError();
}

// ------------------------------------------------- soft Dice + CE loss --
// LitSwinUNETR_Published._loss (models.py:910-928):
//   L = (1-w) * (1 - mean_{b, c>=sc} 2 I/(P+G+eps)) + w * CE(ignore),
//   I = sum_v m p g, P = sum_v m p, G = sum_v g,  m = [y != ignore],
//   g = onehot(y with ignored -> 0),  p = softmax(logits).
constexpr int DL_T = 256, DL_GRID = 256, DL_KMAX = 32;
// Per (block, sample) partial sums of I_k = sum p_k g_k, P_k = sum p_k, G_k =
// sum g_k (g = one-hot of the label, ignored voxels counted at class 0 with p =
// 0, as the oracle's one_hot of the zero-filled labels), the CE sum and the
// valid count.  A wave stages 64 voxels' logit rows in its LDS slice
// (coalesced), each lane turns its row into p in place, then lane l sums
// column k = l % K over the rows r = l / K (mod 64 / K) -- three scalar
// accumulators per lane instead of 3 K-arrays per thread.
__global__ __launch_bounds__(DL_T) void k_dice_stats(const float* __restrict__ x,
                                                     const int64_t* __restrict__ lab, int64_t vps,
                                                     int K, int ignore,
                                                     double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sx = dsm + wv * 64 * K;
  int* ys = reinterpret_cast<int*>(dsm + (DL_T / 64) * 64 * K) + wv * 64;
  const int nset = 64 / K, kcol = lane % K, rset = lane / K;
  const bool colane = rset < nset;
  float I = 0.f, P = 0.f, G = 0.f;
  double ce = 0.0;
  unsigned cnt = 0;
  const int64_t ngroups = (vps + 63) / 64;
  for (int64_t grp = (int64_t)blockIdx.x * (DL_T / 64) + wv; grp < ngroups;
       grp += (int64_t)gridDim.x * (DL_T / 64)) {
    const int64_t v0 = grp * 64;
    const int nv = (int)(vps - v0 < 64 ? vps - v0 : 64);
    wave_copy_rows(sx, x + ((int64_t)b * vps + v0) * K, nv * K, lane);
    wave_lds_sync();
    if (lane < nv) {
      const int64_t y = lab[(int64_t)b * vps + v0 + lane];
      const bool valid = y != ignore;
      float* xv = sx + lane * K;
      float m = -INFINITY;
      for (int k = 0; k < K; ++k) m = fmaxf(m, xv[k]);
      const int yl = valid ? (int)y : 0;
      const float xy = xv[yl];
      float ssum = 0.f;
      for (int k = 0; k < K; ++k) {  // exp once, kept in the row
        const float e = expf(xv[k] - m);
        xv[k] = e;
        ssum += e;
      }
      if (valid) {
        ce += (double)(m + logf(ssum) - xy);
        ++cnt;
      }
      const float inv = 1.f / ssum;
      for (int k = 0; k < K; ++k) xv[k] = valid ? xv[k] * inv : 0.f;
      ys[lane] = yl;
    }
    wave_lds_sync();
    if (colane) {
      for (int r = rset; r < nv; r += nset) {
        const float p = sx[r * K + kcol];
        const bool hit = ys[r] == kcol;
        I += hit ? p : 0.f;
        P += p;
        G += hit ? 1.f : 0.f;
      }
    }
    wave_lds_sync();  // the next group overwrites the slice
  }
  __shared__ float rq[3][DL_T];
  __shared__ double red[DL_T];
  rq[0][threadIdx.x] = colane ? I : 0.f;
  rq[1][threadIdx.x] = colane ? P : 0.f;
  rq[2][threadIdx.x] = colane ? G : 0.f;
  const int nq = 3 * K + 2;
  double* out = part + ((int64_t)b * gridDim.x + blockIdx.x) * nq;
  for (int q = 0; q < 2; ++q) {
    red[threadIdx.x] = q == 0 ? ce : (double)cnt;
    __syncthreads();
    for (int st = DL_T / 2; st > 0; st >>= 1) {
      if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[3 * K + q] = red[0];
    __syncthreads();
  }
  if (threadIdx.x < 3 * K) {  // (quantity, class): waves, then row sets, in order
    const int w = threadIdx.x / K, k = threadIdx.x % K;
    double t = 0.0;
    for (int ww = 0; ww < DL_T / 64; ++ww)
      for (int j = 0; j < nset; ++j) t += (double)rq[w][ww * 64 + j * K + k];
    out[threadIdx.x] = t;
  }
}

// per (b, q) column sums of the k_dice_stats partials, one workgroup each, fixed tree
__global__ __launch_bounds__(256) void k_dice_sum(const double* __restrict__ part, int nblk,
                                                  int nq, double* __restrict__ tot) {
  const int b = blockIdx.y, q = blockIdx.x;
  double s = 0.0;
  for (int j = threadIdx.x; j < nblk; j += 256) s += part[((int64_t)b * nblk + j) * nq + q];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) tot[(int64_t)b * nq + q] = red[0];
}

// coef[b][k][2] = (alpha, beta): dL/dp_k = m * (alpha g_k + beta) for k >= sc;
// out4 = [ce, loss, dice_loss, N_valid]; scal[0] = w / N_valid (the CE gradient scale)
__global__ void k_dice_final(const double* __restrict__ tot, int B, int K, int sc, double w,
                             float* __restrict__ coef, float* __restrict__ out4,
                             double* __restrict__ scal) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int nq = 3 * K + 2;
  double ce = 0.0, N = 0.0, dsum = 0.0;
  const int nc = K - sc;
  for (int b = 0; b < B; ++b) {
    const double* q = tot + (int64_t)b * nq;
    for (int k = 0; k < K; ++k) {
      const double I = q[k], P = q[K + k], G = q[2 * K + k];
      float a = 0.f, be = 0.f;
      if (k >= sc && nc > 0) {
        const double den = P + G + 1e-6;
        dsum += 2.0 * I / den;
        a = (float)(-2.0 * (1.0 - w) / ((double)B * nc * den));
        be = (float)(2.0 * (1.0 - w) * I / ((double)B * nc * den * den));
      }
      coef[((int64_t)b * K + k) * 2 + 0] = a;
      coef[((int64_t)b * K + k) * 2 + 1] = be;
    }
    ce += q[3 * K];
    N += q[3 * K + 1];
  }
  const double dice_loss = nc > 0 ? 1.0 - dsum / ((double)B * nc) : 0.0;
  const double cem = N > 0 ? ce / N : NAN;  // F.cross_entropy: 0/0 -> nan
  out4[0] = (float)cem;
  out4[1] = (float)((1.0 - w) * dice_loss + w * cem);
  out4[2] = (float)dice_loss;
  out4[3] = (float)N;
  scal[0] = N > 0 ? w / N : 0.0;
}

// dlogits = p (G - <p, G>) + (w / N)(p - g), G_k = alpha_k g_k + beta_k; rows
// staged per wave as in k_dice_stats, overwritten in place, stored coalesced
__global__ __launch_bounds__(DL_T) void k_dice_grad(const float* __restrict__ x,
                                                    const int64_t* __restrict__ lab, int64_t vps,
                                                    int64_t V, int K, int ignore,
                                                    const float* __restrict__ coef,
                                                    const double* __restrict__ scal,
                                                    float* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  const float wN = (float)scal[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sx = dsm + wv * 64 * K;
  const int64_t ngroups = (V + 63) / 64;
  for (int64_t grp = (int64_t)blockIdx.x * (DL_T / 64) + wv; grp < ngroups;
       grp += (int64_t)gridDim.x * (DL_T / 64)) {
    const int64_t v0 = grp * 64;
    const int nv = (int)(V - v0 < 64 ? V - v0 : 64);
    wave_copy_rows(sx, x + v0 * K, nv * K, lane);
    wave_lds_sync();
    if (lane < nv) {
      const int64_t v = v0 + lane;
      const int64_t y = lab[v];
      float* xv = sx + lane * K;  // logits in, dlogits out (in place)
      if (y == ignore) {
        for (int k = 0; k < K; ++k) xv[k] = 0.f;
      } else {
        const float2* cf = reinterpret_cast<const float2*>(coef) + (int64_t)(v / vps) * K;
        const int yi = (int)y;
        float m = -INFINITY;
        for (int k = 0; k < K; ++k) m = fmaxf(m, xv[k]);
        float ssum = 0.f;
        for (int k = 0; k < K; ++k) {  // exp once, kept in the row
          const float e = expf(xv[k] - m);
          xv[k] = e;
          ssum += e;
        }
        const float inv = 1.f / ssum;
        float pg = 0.f;
        for (int k = 0; k < K; ++k) {
          const float2 c = cf[k];
          pg += xv[k] * inv * (c.x * (k == yi ? 1.f : 0.f) + c.y);
        }
        for (int k = 0; k < K; ++k) {
          const float2 c = cf[k];
          const float pk = xv[k] * inv;
          const float Gk = c.x * (k == yi ? 1.f : 0.f) + c.y;
          xv[k] = pk * (Gk - pg) + wN * (pk - (k == yi ? 1.f : 0.f));
        }
      }
    }
    wave_lds_sync();
    wave_copy_rows(dx + v0 * K, sx, nv * K, lane);
    wave_lds_sync();  // the next group overwrites the slice
  }
}

size_t dice_ce_ws_bytes(int B, int K) {
  return ((size_t)B * (DL_GRID + 1) * (3 * K + 2) + 8) * sizeof(double) +
         (size_t)B * K * 2 * sizeof(float) + 64;
}

hipError_t dice_ce_loss(const float* logits, const int64_t* labels, int B, int64_t vps, int K,
                        int ignore, int include_bg, double ce_weight, float* out4, float* dlogits,
                        void* ws, hipStream_t s) {
  if (K < 1 || K > DL_KMAX) return hipErrorInvalidValue;
  double* part = static_cast<double*>(ws);
  double* tot = part + (size_t)B * DL_GRID * (3 * K + 2);
  double* scal = tot + (size_t)B * (3 * K + 2);
  float* coef = reinterpret_cast<float*>(scal + 8);
  const size_t lds = (size_t)(DL_T / 64) * 64 * (K + 1) * sizeof(float);
  hipLaunchKernelGGL(k_dice_stats, dim3(DL_GRID, B), dim3(DL_T), lds, s, logits, labels, vps, K,
                     ignore, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_dice_sum, dim3(3 * K + 2, B), dim3(256), 0, s, part, DL_GRID, 3 * K + 2,
                     tot);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_dice_final, dim3(1), dim3(64), 0, s, tot, B, K, include_bg ? 0 : 1,
                     ce_weight, coef, out4, scal);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int64_t V = (int64_t)B * vps;
  hipLaunchKernelGGL(k_dice_grad, dim3((unsigned)std::min<int64_t>(cdiv64(V, DL_T), 2048)),
                     dim3(DL_T), lds, s, logits, labels, vps, V, K, ignore, coef, scal, dlogits);
  return hipGetLastError();
}

}  // namespace spff
