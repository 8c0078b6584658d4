// Swin window attention (MONAI 1.5.2 WindowAttention, unshifted; see
// oracle/swin_oracle.py) forward and backward for the SwinUNETR variant.
//
// One workgroup per (window, head).  A window's tokens are gathered straight
// from the token-major qkv rows [T][3C] of the real tokens; tokens of the
// zero padding (pad after norm1) take q, k, v = the qkv bias.  K and V of the
// window (n <= 343 tokens x hd) plus the head's relative-bias column sit in
// LDS; each thread owns one query and streams the keys with an online
// softmax (fp32, exp / max rescaling), so the n x n score matrix never exists.
// The backward recomputes scores from the saved log-sum-exp: dq per query
// thread; dk / dv per key thread, which also accumulates the bias-table
// gradient into its wave's private LDS table (the lanes of a wave always hit
// distinct entries), the 6 wave tables then summed in order -- every reduction
// has a fixed order, so the results are deterministic; per-window partials of
// the table and the padded tokens' k / v gradients are summed over windows in
// window order by small reduce kernels.
//
// Bias index: MONAI's relative_position_index is built for the configured
// w^3 window and sliced [:n, :n]; token t's index coordinates are therefore
// (t / w^2, t / w % w, t % w) in the w^3 enumeration even when a stage's
// window shrinks (ws < w) -- restated here exactly:
//   ridx(i, j) = key(i) - key(j) + (w-1) ((2w-1)^2 + (2w-1) + 1),
//   key(t) = c_d (2w-1)^2 + c_h (2w-1) + c_w.
#include "spff_internal.h"
#include "swin_internal.h"

#include <math.h>

#ifndef SPFF_ATTN_DIAG
#define SPFF_ATTN_DIAG 0  // timing diagnostics only: skip phase 1 (dq) or 2 (dk/dv/table)
#endif
#ifndef SPFF_ATTN_UNROLL
#define SPFF_ATTN_UNROLL 2  // key / query loop unroll of the backward (ILP at 1 WG per CU)
#endif

namespace spff {

namespace {
inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
constexpr int AT_MAXN = 343, AT_THREADS = 384;

struct WinTok {
  int64_t row;  // token row, or -1 for a padded token
};
__device__ __forceinline__ int64_t tok_row(const AttnGeo& g, int64_t win, int t) {
  int64_t r = win;
  const int iw = (int)(r % g.nww); r /= g.nww;
  const int ih = (int)(r % g.nwh); r /= g.nwh;
  const int id = (int)(r % g.nwd);
  const int64_t b = r / g.nwd;
  const int tw = t % g.wsw, th = (t / g.wsw) % g.wsh, td = t / (g.wsw * g.wsh);
  const int d = id * g.wsd + td, h = ih * g.wsh + th, w = iw * g.wsw + tw;
  if (d >= g.D || h >= g.H || w >= g.W) return -1;
  return ((b * g.D + d) * g.H + h) * (int64_t)g.W + w;
}
__device__ __forceinline__ int key7(int t, int w) {
  const int cd = t / (w * w), ch = (t / w) % w, cw = t % w;
  return (cd * (2 * w - 1) + ch) * (2 * w - 1) + cw;
}
}  // namespace

AttnGeo attn_geo(int B, int D, int H, int W, int w, int C, int nh) {
  AttnGeo g;
  g.B = B; g.D = D; g.H = H; g.W = W; g.w = w;
  g.wsd = D <= w ? D : w;
  g.wsh = H <= w ? H : w;
  g.wsw = W <= w ? W : w;
  g.nwd = (D + g.wsd - 1) / g.wsd;
  g.nwh = (H + g.wsh - 1) / g.wsh;
  g.nww = (W + g.wsw - 1) / g.wsw;
  g.n = g.wsd * g.wsh * g.wsw;
  g.C = C; g.nh = nh; g.hd = C / nh;
  g.scale = (float)pow((double)g.hd, -0.5);
  return g;
}

template <int HD>
__global__ __launch_bounds__(AT_THREADS) void k_attn_fwd(const float* __restrict__ qkv,
                                                         const float* __restrict__ bqkv,
                                                         const float* __restrict__ table,
                                                         AttnGeo g, float* __restrict__ O,
                                                         float* __restrict__ lse) {
  extern __shared__ float sm[];
  const int n = g.n, R = g.R(), C = g.C, h = blockIdx.y;
  const int64_t win = blockIdx.x;
  float* Ks = sm;                 // [n][HD]
  float* Vs = Ks + n * HD;        // [n][HD]
  float* tab = Vs + n * HD;       // [R]
  int* k7 = reinterpret_cast<int*>(tab + R);  // [n]
  const int tid = threadIdx.x;
  for (int t = tid; t < n; t += blockDim.x) {
    const int64_t row = tok_row(g, win, t);
#pragma unroll
    for (int e = 0; e < HD; ++e) {
      Ks[t * HD + e] = row >= 0 ? qkv[row * 3 * C + C + h * HD + e] : bqkv[C + h * HD + e];
      Vs[t * HD + e] = row >= 0 ? qkv[row * 3 * C + 2 * C + h * HD + e] : bqkv[2 * C + h * HD + e];
    }
    k7[t] = key7(t, g.w);
  }
  for (int r = tid; r < R; r += blockDim.x) tab[r] = table[(int64_t)r * g.nh + h];
  __syncthreads();
  const int i = tid;
  if (i >= n) return;
  const int64_t row = tok_row(g, win, i);
  float q[HD], acc[HD];
#pragma unroll
  for (int e = 0; e < HD; ++e) {
    q[e] = (row >= 0 ? qkv[row * 3 * C + h * HD + e] : bqkv[h * HD + e]) * g.scale;
    acc[e] = 0.f;
  }
  const int base = k7[i] + (g.w - 1) * ((2 * g.w - 1) * (2 * g.w - 1) + (2 * g.w - 1) + 1);
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < n; ++j) {
    float sc = 0.f;
#pragma unroll
    for (int e = 0; e < HD; ++e) sc += q[e] * Ks[j * HD + e];
    sc += tab[base - k7[j]];
    if (sc > m) {
      const float corr = expf(m - sc);  // m = -inf on the first key: corr = 0
      l = l * corr + 1.f;
#pragma unroll
      for (int e = 0; e < HD; ++e) acc[e] = acc[e] * corr + Vs[j * HD + e];
      m = sc;
    } else {
      const float p = expf(sc - m);
      l += p;
#pragma unroll
      for (int e = 0; e < HD; ++e) acc[e] += p * Vs[j * HD + e];
    }
  }
  const float inv = 1.f / l;
  if (row >= 0) {
#pragma unroll
    for (int e = 0; e < HD; ++e) O[row * C + h * HD + e] = acc[e] * inv;
  }
  lse[(win * g.nh + h) * n + i] = m + logf(l);
}

template <int HD>
__global__ __launch_bounds__(AT_THREADS) void k_attn_bwd(
    const float* __restrict__ qkv, const float* __restrict__ bqkv,
    const float* __restrict__ table, const float* __restrict__ O, const float* __restrict__ dO,
    const float* __restrict__ lse, AttnGeo g, float* __restrict__ dqkv,
    float* __restrict__ tpart, float* __restrict__ ppart) {
  extern __shared__ float sm[];
  const int n = g.n, R = g.R(), C = g.C, h = blockIdx.y, w = g.w;
  const int64_t win = blockIdx.x;
  float* Qs = sm;                 // [n][HD] (scaled)
  float* Ks = Qs + n * HD;
  float* Vs = Ks + n * HD;
  float* Gs = Vs + n * HD;        // dO
  float* Ls = Gs + n * HD;        // lse [n]
  float* Dd = Ls + n;             // rowsum(dO * O) [n]
  float* tab = Dd + n;            // [R]
  float* wred = tab + R;          // [6][2 HD]
  float* wtab = wred + 6 * 2 * HD;  // [6 waves][R] private bias-table accumulators
  int* k7 = reinterpret_cast<int*>(wtab + 6 * R);  // [n]
  const int tid = threadIdx.x;
  for (int t = tid; t < n; t += blockDim.x) {
    const int64_t row = tok_row(g, win, t);
    float dd = 0.f;
#pragma unroll
    for (int e = 0; e < HD; ++e) {
      const int c = h * HD + e;
      Qs[t * HD + e] = (row >= 0 ? qkv[row * 3 * C + c] : bqkv[c]) * g.scale;
      Ks[t * HD + e] = row >= 0 ? qkv[row * 3 * C + C + c] : bqkv[C + c];
      Vs[t * HD + e] = row >= 0 ? qkv[row * 3 * C + 2 * C + c] : bqkv[2 * C + c];
      const float go = row >= 0 ? dO[row * C + c] : 0.f;
      Gs[t * HD + e] = go;
      dd += row >= 0 ? go * O[row * C + c] : 0.f;
    }
    Dd[t] = dd;
    Ls[t] = lse[(win * g.nh + h) * n + t];
    k7[t] = key7(t, w);
  }
  for (int r = tid; r < R; r += blockDim.x) tab[r] = table[(int64_t)r * g.nh + h];
  for (int r = tid; r < 6 * R; r += blockDim.x) wtab[r] = 0.f;
  __syncthreads();
  const int off0 = (w - 1) * ((2 * w - 1) * (2 * w - 1) + (2 * w - 1) + 1);
  // ---- dq: thread per query
  if (SPFF_ATTN_DIAG != 1 && tid < n) {
    const int i = tid;
    const int64_t row = tok_row(g, win, i);
    if (row >= 0) {
      float q[HD], go[HD], dq[HD];
#pragma unroll
      for (int e = 0; e < HD; ++e) {
        q[e] = Qs[i * HD + e];
        go[e] = Gs[i * HD + e];
        dq[e] = 0.f;
      }
      const float li = Ls[i], di = Dd[i];
      const int base = k7[i] + off0;
#pragma unroll SPFF_ATTN_UNROLL
      for (int j = 0; j < n; ++j) {
        float sc = 0.f, dp = 0.f;
#pragma unroll
        for (int e = 0; e < HD; ++e) {
          sc += q[e] * Ks[j * HD + e];
          dp += go[e] * Vs[j * HD + e];
        }
        const float p = expf(sc + tab[base - k7[j]] - li);
        const float ds = p * (dp - di);
#pragma unroll
        for (int e = 0; e < HD; ++e) dq[e] += ds * Ks[j * HD + e];
      }
#pragma unroll
      for (int e = 0; e < HD; ++e) dqkv[row * 3 * C + h * HD + e] = dq[e] * g.scale;
    }
  }
  // ---- dk, dv: thread per key
  if (SPFF_ATTN_DIAG != 2) {
    const int j = tid;
    float dk[HD], dv[HD];
#pragma unroll
    for (int e = 0; e < HD; ++e) dk[e] = dv[e] = 0.f;
    int64_t row = -1;
    if (j < n) {
      row = tok_row(g, win, j);
      float k[HD], v[HD];
#pragma unroll
      for (int e = 0; e < HD; ++e) {
        k[e] = Ks[j * HD + e];
        v[e] = Vs[j * HD + e];
      }
      const int kj = k7[j] - off0;
      // bias-table gradient: at each query i the wave's lanes (keys j) hit distinct
      // entries k7[i] - kj of the wave's private table -> plain read-add-write, in
      // query order; the 6 tables are summed in wave order below (deterministic)
      float* mt = wtab + (tid >> 6) * R;
#pragma unroll SPFF_ATTN_UNROLL
      for (int i = 0; i < n; ++i) {
        float sc = 0.f, dp = 0.f;
#pragma unroll
        for (int e = 0; e < HD; ++e) {
          sc += Qs[i * HD + e] * k[e];
          dp += Gs[i * HD + e] * v[e];
        }
        const int ri = k7[i] - kj;
        const float p = expf(sc + tab[ri] - Ls[i]);
        const float ds = p * (dp - Dd[i]);
        mt[ri] += ds;
#pragma unroll
        for (int e = 0; e < HD; ++e) {
          dk[e] += ds * Qs[i * HD + e];
          dv[e] += p * Gs[i * HD + e];
        }
      }
      if (row >= 0) {
#pragma unroll
        for (int e = 0; e < HD; ++e) {
          dqkv[row * 3 * C + C + h * HD + e] = dk[e];
          dqkv[row * 3 * C + 2 * C + h * HD + e] = dv[e];
        }
      }
    }
    // padded keys' gradients -> the k / v bias: wave sums, then waves in order
    const bool pad = j < n && row < 0;
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int e = 0; e < 2 * HD; ++e) {
      float t = pad ? (e < HD ? dk[e] : dv[e - HD]) : 0.f;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0) wred[wv * 2 * HD + e] = t;
    }
  }
  __syncthreads();
  if (tid < 2 * HD) {
    float t = 0.f;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) t += wred[wv * 2 * HD + tid];
    ppart[(win * g.nh + h) * 2 * HD + tid] = t;
  }
  // ---- bias table: the waves' private tables, summed in wave order
  for (int r = tid; r < R; r += blockDim.x) {
    float acc = 0.f;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) acc += wtab[wv * R + r];
    tpart[(win * g.nh + h) * R + r] = acc;
  }
}

static size_t fwd_lds(const AttnGeo& g) {
  return (size_t)(2 * g.n * g.hd + g.R()) * sizeof(float) + (size_t)g.n * sizeof(int);
}
static size_t bwd_lds(const AttnGeo& g) {
  return (size_t)(4 * g.n * g.hd + 2 * g.n + 7 * g.R() + 6 * 2 * g.hd) * sizeof(float) +
         (size_t)g.n * sizeof(int);
}

size_t swin_attn_ws_bytes(const AttnGeo& g) {
  return (size_t)g.nwin() * g.nh * (g.R() + 2 * g.hd) * sizeof(float);
}

#define SPFF_ATTN_HD(X) X(4) X(8) X(12) X(16) X(24) X(32)

hipError_t swin_attn_fwd(const float* qkv, const float* bqkv, const float* table,
                         const AttnGeo& g, float* O, float* lse, hipStream_t s) {
  if (g.n > AT_MAXN || g.C % g.nh) return hipErrorInvalidValue;
  const dim3 grid((unsigned)g.nwin(), g.nh);
  const size_t lds = fwd_lds(g);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (g.hd) {
#define SPFF_F(HD_)                                                                             \
  case HD_: {                                                                                   \
    auto kern = k_attn_fwd<HD_>;                                                                \
    hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                    \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);  \
    if (e0 != hipSuccess) return e0;                                                            \
    hipLaunchKernelGGL(kern, grid, dim3(AT_THREADS), lds, s, qkv, bqkv, table, g, O, lse);      \
  } break;
    SPFF_ATTN_HD(SPFF_F)
#undef SPFF_F
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t swin_attn_bwd(const float* qkv, const float* bqkv, const float* table,
                         const float* O, const float* dO, const float* lse, const AttnGeo& g,
                         float* dqkv, float* dtable, float* dbqkv, float* ws, hipStream_t s) {
  if (g.n > AT_MAXN || g.C % g.nh) return hipErrorInvalidValue;
  const dim3 grid((unsigned)g.nwin(), g.nh);
  const size_t lds = bwd_lds(g);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  float* tpart = ws;
  float* ppart = ws + (size_t)g.nwin() * g.nh * g.R();
  switch (g.hd) {
#define SPFF_B(HD_)                                                                              \
  case HD_: {                                                                                    \
    auto kern = k_attn_bwd<HD_>;                                                                 \
    hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                     \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);   \
    if (e0 != hipSuccess) return e0;                                                             \
    hipLaunchKernelGGL(kern, grid, dim3(AT_THREADS), lds, s, qkv, bqkv, table, O, dO, lse, g,    \
                       dqkv, tpart, ppart);                                                      \
  } break;
    SPFF_ATTN_HD(SPFF_B)
#undef SPFF_B
    default: return hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // dtable[r][h] = sum over windows of tpart[win][h][r]
  if ((e = col_reduce_map(tpart, (int)g.nwin(), (int64_t)g.nh * g.R(), g.nh * g.R(), dtable, 0, 1,
                          g.R(), g.nh, g.hd, g.C, s)) != hipSuccess)
    return e;
  return dbqkv ? swin_attn_pad_grad(g, ws, dbqkv, s) : hipSuccess;
}

hipError_t swin_attn_pad_grad(const AttnGeo& g, const float* ws, float* dbqkv, hipStream_t s) {
  // dbqkv[C + h*hd + e] += sum_win ppart[win][h][e]; dbqkv[2C + ...] += ...[hd + e]
  const float* ppart = ws + (size_t)g.nwin() * g.nh * g.R();
  return col_reduce_map(ppart, (int)g.nwin(), (int64_t)g.nh * 2 * g.hd, g.nh * 2 * g.hd, dbqkv, 1,
                        2, g.R(), g.nh, g.hd, g.C, s);
}

}  // namespace spff
