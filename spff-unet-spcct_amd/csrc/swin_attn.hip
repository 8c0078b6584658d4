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
#include <cstdlib>

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

// ====================================================== MFMA window attention ==
// The same attention on v_mfma_f32_16x16x32_bf16 with the exact 3-plane bf16 split of
// the conv kernels (x = h + m + l; the six products hh, hm, mh, hl, lh, mm accumulate in
// fp32: fp32-faithful).  Head dim hd <= 16 (the registry's 12): token rows of q / k / v /
// dO are stored as three bf16 planes [3][NP][16] (dims >= hd zero, NP = n rounded up to
// 32), one 32-byte row per token and plane.
//   * a contraction over the head dim (S = q k^T, dP = dO v^T) packs the six products
//     into k = 96 = three k = 32 MFMAs: segment s of 16 slots pairs A plane ASEL[s] with
//     B plane BSEL[s] (h.h, m.h, h.m, l.h, h.l, m.m) -- 16 useful of every 32 MFMA slots
//     instead of 12 x 6 MFMAs of 12 useful;
//   * a contraction over tokens (O = P v, dq = dS k, dk = dS^T q, dv = P^T dO) takes the
//     tokens-major planes through ds_read_b64_tr_b16 (hd on the lanes, 2 x 4 tokens per
//     lane group) against P / dS held in registers: the score tile S^T comes out of the
//     MFMA with the query (or key) on the lane and 4 + 4 tokens per lane group, which is
//     exactly the k order of the next MFMA's register operand -- no shuffle, no LDS trip.
// Forward: one 16-query block per wave step, 32 keys per step, online softmax.  Backward:
// two kernels -- A: per 16-query block, recompute S / P / dP, dq and the bias-table
// gradient (each wave's private LDS table, ds_add_f32 in program order; the 8 tables
// summed in wave order: deterministic); B: per 16-key block, dk, dv and the padded
// tokens' k / v bias gradients.  Every reduction has a fixed order.
namespace {
typedef float f32x4m __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8m __attribute__((ext_vector_type(8)));
typedef short i16x4m __attribute__((ext_vector_type(4)));
constexpr int AM_THREADS = 512, AM_WAVES = AM_THREADS / 64, PLW = 16;
// packed head-dim contraction: plane of segment s for the A / B operand
__device__ __forceinline__ int asel(int s) { return (0x102010 >> (4 * s)) & 15; }  // 0,1,0,2,0,1
__device__ __forceinline__ int bsel(int s) { return (0x120100 >> (4 * s)) & 15; }  // 0,0,1,0,2,1

__device__ __forceinline__ void split8m(const float (&v)[8], bf16x8m (&o)[3]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float r = v[e];
    const __bf16 a = (__bf16)r;
    r -= (float)a;
    const __bf16 b = (__bf16)r;
    r -= (float)b;
    o[0][e] = a;
    o[1][e] = b;
    o[2][e] = (__bf16)r;
  }
}
typedef __attribute__((address_space(3))) i16x4m lds_i16x4m;
__device__ __forceinline__ i16x4m trr(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4m*)(p));
}
__device__ __forceinline__ bf16x8m frag2(const i16x4m& lo, const i16x4m& hi) {
  typedef short i16x8m __attribute__((ext_vector_type(8)));
  i16x8m v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8m, v);
}
__device__ __forceinline__ f32x4m mf(const bf16x8m& a, const bf16x8m& b, f32x4m c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// C += A * B over three split planes: the six leading products
__device__ __forceinline__ f32x4m mf6(const bf16x8m (&a)[3], const bf16x8m (&b)[3], f32x4m c) {
  c = mf(a[1], b[1], c);
  c = mf(a[0], b[2], c);
  c = mf(a[2], b[0], c);
  c = mf(a[0], b[1], c);
  c = mf(a[1], b[0], c);
  return mf(a[0], b[0], c);
}
__device__ __forceinline__ int np32(int n) { return (n + 31) & ~31; }

// planes [3][NP][16] of a head's hd values of every window token: src + row * ld + off
// for real tokens, bias + off (if given, else 0) for padded ones, 0 beyond n; * mul
template <int HD>
__device__ void stage_planes(unsigned short* dst, const AttnGeo& g, int64_t win, const float* src,
                             int64_t ld, int off, const float* bias, float mul) {
  const int n = g.n, NP = np32(n);
  for (int it = threadIdx.x; it < NP * 4; it += blockDim.x) {
    const int t = it >> 2, c4 = (it & 3) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < n && c4 < HD) {
      const int64_t row = tok_row(g, win, t);
      const float* p = row >= 0 ? src + row * ld + off + c4 : (bias ? bias + off + c4 : nullptr);
      if (p) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x * mul; v[1] = q.y * mul; v[2] = q.z * mul; v[3] = q.w * mul;
      }
    }
    unsigned short hs[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float r = v[e];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const __bf16 b = (__bf16)r;
        hs[pl][e] = __builtin_bit_cast(unsigned short, b);
        r -= (float)b;
      }
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      uint2 u;
      u.x = (unsigned)hs[pl][0] | ((unsigned)hs[pl][1] << 16);
      u.y = (unsigned)hs[pl][2] | ((unsigned)hs[pl][3] << 16);
      *reinterpret_cast<uint2*>(dst + ((size_t)pl * NP + t) * PLW + c4) = u;
    }
  }
}
// this lane's token row as the packed B operand of a head-dim contraction: dims
// 8 (kg & 1) .. + 8 of the three planes, segment s = 2 m + (kg >> 1) per MFMA m
template <int HD>
__device__ __forceinline__ void token_bfrag(const float* p, float mul, int kg, bf16x8m (&f)[3]) {
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int d = 8 * (kg & 1) + e;
    v[e] = (p && d < HD) ? p[d] * mul : 0.f;
  }
  bf16x8m pl[3];
  split8m(v, pl);
#pragma unroll
  for (int m = 0; m < 3; ++m) f[m] = pl[bsel(2 * m + (kg >> 1))];
}
// packed A operand (rows = 16 tokens t0 + l16 of planes P), MFMA m
__device__ __forceinline__ bf16x8m rows_afrag(const unsigned short* P, int NP, int t, int kg, int m) {
  const int s = 2 * m + (kg >> 1);
  return *reinterpret_cast<const bf16x8m*>(P + ((size_t)asel(s) * NP + t) * PLW + 8 * (kg & 1));
}
// transposed A operand (rows = the 16 head dims, k = tokens t0 + 4 kg + q and
// t0 + 16 + 4 kg + q) of planes P, by ds_read_b64_tr_b16: lane 4 q + p of each 16-lane
// group addresses token row q, dims 4 p .. 4 p + 3
__device__ __forceinline__ void tok_tfrag(const unsigned short* P, int NP, int t0, int lane,
                                          bf16x8m (&f)[3]) {
  const int kg = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int t = t0 + 4 * kg + q;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const unsigned short* b = P + ((size_t)pl * NP + t) * PLW + 4 * pp;
    f[pl] = frag2(trr(b), trr(b + 16 * PLW));
  }
}
}  // namespace

template <int HD>
__global__ __launch_bounds__(AM_THREADS, 2) void k_attn_fwd_m(const float* __restrict__ qkv,
                                                              const float* __restrict__ bqkv,
                                                              const float* __restrict__ table,
                                                              AttnGeo g, float* __restrict__ O,
                                                              float* __restrict__ lse) {
  extern __shared__ uint4 sm4[];
  const int n = g.n, NP = np32(n), R = g.R(), C = g.C, h = blockIdx.y, w = g.w;
  const int64_t win = blockIdx.x;
  unsigned short* Kp = reinterpret_cast<unsigned short*>(sm4);
  unsigned short* Vp = Kp + 3 * NP * PLW;
  float* tab = reinterpret_cast<float*>(Vp + 3 * NP * PLW);
  int* k7 = reinterpret_cast<int*>(tab + R);
  stage_planes<HD>(Kp, g, win, qkv, 3 * C, C + h * HD, bqkv, 1.f);
  stage_planes<HD>(Vp, g, win, qkv, 3 * C, 2 * C + h * HD, bqkv, 1.f);
  for (int r = threadIdx.x; r < R; r += blockDim.x) tab[r] = table[(int64_t)r * g.nh + h];
  for (int t = threadIdx.x; t < NP; t += blockDim.x) k7[t] = t < n ? key7(t, w) : 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kg = lane >> 4;
  const int off0 = (w - 1) * ((2 * w - 1) * (2 * w - 1) + (2 * w - 1) + 1);
  for (int qb = wave; qb < NP / 16; qb += AM_WAVES) {
    const int i = qb * 16 + l16;  // this lane's query (the score tiles' column)
    const bool iv = i < n;
    const int64_t row = iv ? tok_row(g, win, i) : -2;
    bf16x8m qf[3];
    token_bfrag<HD>(row >= 0 ? qkv + row * 3 * C + h * HD : (row == -1 ? bqkv + h * HD : nullptr),
                    g.scale, kg, qf);
    const int base = iv ? k7[i] + off0 : 0;
    float mrow = -INFINITY, lsum = 0.f;
    f32x4m o = {0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < NP; kb += 32) {
      float sc[8];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int j0 = kb + 16 * sb;
        f32x4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 3; ++m) acc = mf(rows_afrag(Kp, NP, j0 + l16, kg, m), qf[m], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // acc[r] = S[query i][key j0 + 4 kg + r]
          const int j = j0 + 4 * kg + r;
          sc[4 * sb + r] = !iv ? 0.f : (j < n ? acc[r] + tab[base - k7[j]] : -INFINITY);
        }
      }
      float mx = sc[0];
#pragma unroll
      for (int e = 1; e < 8; ++e) mx = fmaxf(mx, sc[e]);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mnew = fmaxf(mrow, mx);
      const float corr = expf(mrow - mnew);  // mrow = -inf on the first step: 0
      float pv[8], ps = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pv[e] = expf(sc[e] - mnew);
        ps += pv[e];
      }
      lsum = lsum * corr + ps;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] *= corr;
      mrow = mnew;
      // O^T [dim][query] += V^T [dim][key] P^T [key][query]
      bf16x8m pf[3], vf[3];
      split8m(pv, pf);
      tok_tfrag(Vp, NP, kb, lane, vf);
      o = mf6(vf, pf, o);
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    const float inv = 1.f / lsum;
    if (row >= 0 && 4 * kg < HD) {  // lane (query i, kg) holds dims 4 kg + r
      *reinterpret_cast<float4*>(O + row * C + h * HD + 4 * kg) =
          make_float4(o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
    }
    if (iv && kg == 0) lse[(win * g.nh + h) * n + i] = mrow + logf(lsum);
  }
}

// backward A: dq per 16-query block; dS [NP][NP] of the (window, head) to dsw for the
// bias-table gradient (k_attn_dtable_m: per-table-entry sums in a fixed order -- LDS
// float atomics into per-wave tables measured 2.3x this kernel's time)
template <int HD>
__global__ __launch_bounds__(AM_THREADS, 2) void k_attn_bwd_q_m(
    const float* __restrict__ qkv, const float* __restrict__ bqkv,
    const float* __restrict__ table, const float* __restrict__ O, const float* __restrict__ dO,
    const float* __restrict__ lse, AttnGeo g, float* __restrict__ dqkv,
    float* __restrict__ dsw) {
  extern __shared__ uint4 sm4[];
  const int n = g.n, NP = np32(n), R = g.R(), C = g.C, h = blockIdx.y, w = g.w;
  const int64_t win = blockIdx.x;
  unsigned short* Kp = reinterpret_cast<unsigned short*>(sm4);
  unsigned short* Vp = Kp + 3 * NP * PLW;
  float* tab = reinterpret_cast<float*>(Vp + 3 * NP * PLW);
  int* k7 = reinterpret_cast<int*>(tab + R);
  stage_planes<HD>(Kp, g, win, qkv, 3 * C, C + h * HD, bqkv, 1.f);
  stage_planes<HD>(Vp, g, win, qkv, 3 * C, 2 * C + h * HD, bqkv, 1.f);
  for (int r = threadIdx.x; r < R; r += blockDim.x) tab[r] = table[(int64_t)r * g.nh + h];
  for (int t = threadIdx.x; t < NP; t += blockDim.x) k7[t] = t < n ? key7(t, w) : 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kg = lane >> 4;
  const int off0 = (w - 1) * ((2 * w - 1) * (2 * w - 1) + (2 * w - 1) + 1);
  float* dsb = dsw + (win * g.nh + h) * (int64_t)NP * NP;
  for (int qb = wave; qb < NP / 16; qb += AM_WAVES) {
    const int i = qb * 16 + l16;
    const bool iv = i < n;
    const int64_t row = iv ? tok_row(g, win, i) : -2;
    bf16x8m qf[3], gf[3];
    token_bfrag<HD>(row >= 0 ? qkv + row * 3 * C + h * HD : (row == -1 ? bqkv + h * HD : nullptr),
                    g.scale, kg, qf);
    const float* dop = row >= 0 ? dO + row * C + h * HD : nullptr;  // padded / beyond: 0
    token_bfrag<HD>(dop, 1.f, kg, gf);
    float di = 0.f;
    if (dop) {
      const float* op = O + row * C + h * HD;
#pragma unroll
      for (int e = 0; e < HD; ++e) di += dop[e] * op[e];
    }
    const float li = iv ? lse[(win * g.nh + h) * n + i] : 0.f;
    const int base = iv ? k7[i] + off0 : 0;
    f32x4m dq = {0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < NP; kb += 32) {
      float dsv[8];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int j0 = kb + 16 * sb;
        f32x4m s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          s = mf(rows_afrag(Kp, NP, j0 + l16, kg, m), qf[m], s);
          dp = mf(rows_afrag(Vp, NP, j0 + l16, kg, m), gf[m], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + 4 * kg + r;
          const bool ok = iv && j < n;
          const int ri = ok ? base - k7[j] : 0;
          const float p = ok ? expf(s[r] + tab[ri] - li) : 0.f;
          dsv[4 * sb + r] = p * (dp[r] - di);
        }
        if (iv)  // dS[i][j0 + 4 kg .. + 3] (zero beyond n)
          *reinterpret_cast<float4*>(dsb + (int64_t)i * NP + j0 + 4 * kg) =
              make_float4(dsv[4 * sb], dsv[4 * sb + 1], dsv[4 * sb + 2], dsv[4 * sb + 3]);
      }
      bf16x8m df[3], kf[3];
      split8m(dsv, df);
      tok_tfrag(Kp, NP, kb, lane, kf);
      dq = mf6(kf, df, dq);  // dq^T [dim][query] += k^T [dim][key] dS^T [key][query]
    }
    if (row >= 0 && 4 * kg < HD)
      *reinterpret_cast<float4*>(dqkv + row * 3 * C + h * HD + 4 * kg) =
          make_float4(dq[0] * g.scale, dq[1] * g.scale, dq[2] * g.scale, dq[3] * g.scale);
  }
}

// bias-table gradient of one (window, head) from its dS.  Entry r is the relative offset
// (od, oh, ow) of the configured WW^3 window (ridx = key7(i) - key7(j) + off0, tokens
// enumerated t = (cd WW + ch) WW + cw).  Tokens group into WW^2 rows A = (cd, ch) of WW
// tokens; the WW x WW block of dS between rows A and B contributes its 2 WW - 1 diagonal
// sums to the entries (od, oh) = A - B.  Pass 1: a thread per row pair (A, B) reads its
// block (7 contiguous floats per dS row) and keeps the diagonal sums in LDS; pass 2: a
// thread per entry adds its row pairs in (cd, ch) order.  Fixed order; dS is read once.
template <int WW>
__global__ __launch_bounds__(256) void k_attn_dtable_m(const float* __restrict__ dsw, AttnGeo g,
                                                       float* __restrict__ tpart) {
  constexpr int NA = WW * WW, W2 = 2 * WW - 1;
  extern __shared__ float dsh[];  // [NA][NA][W2]
  const int n = g.n, NP = np32(n), R = g.R(), h = blockIdx.y;
  const int64_t win = blockIdx.x;
  const float* dsb = dsw + (win * g.nh + h) * (int64_t)NP * NP;
  for (int t = threadIdx.x; t < NA * NA; t += blockDim.x) {
    const int A = t / NA, Bq = t % NA;
    float d[W2];
#pragma unroll
    for (int e = 0; e < W2; ++e) d[e] = 0.f;
#pragma unroll
    for (int cw = 0; cw < WW; ++cw) {
      const int i = A * WW + cw;
      float v[WW];
#pragma unroll
      for (int c2 = 0; c2 < WW; ++c2) {
        const int j = Bq * WW + c2;
        v[c2] = (i < n && j < n) ? dsb[(int64_t)i * NP + j] : 0.f;
      }
#pragma unroll
      for (int c2 = 0; c2 < WW; ++c2) d[cw - c2 + WW - 1] += v[c2];
    }
#pragma unroll
    for (int e = 0; e < W2; ++e) dsh[t * W2 + e] = d[e];
  }
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const int od = r / (W2 * W2) - (WW - 1), oh = (r / W2) % W2 - (WW - 1), e = r % W2;
    float acc = 0.f;
    for (int cd = max(0, od); cd < min(WW, WW + od); ++cd)
      for (int ch = max(0, oh); ch < min(WW, WW + oh); ++ch)
        acc += dsh[((cd * WW + ch) * NA + (cd - od) * WW + (ch - oh)) * W2 + e];
    tpart[(win * g.nh + h) * R + r] = acc;
  }
}

// backward B: dk, dv and the padded tokens' k / v gradients, per 16-key block
template <int HD>
__global__ __launch_bounds__(AM_THREADS, 1) void k_attn_bwd_kv_m(
    const float* __restrict__ qkv, const float* __restrict__ bqkv,
    const float* __restrict__ table, const float* __restrict__ O, const float* __restrict__ dO,
    const float* __restrict__ lse, AttnGeo g, float* __restrict__ dqkv,
    float* __restrict__ ppart) {
  extern __shared__ uint4 sm4[];
  const int n = g.n, NP = np32(n), R = g.R(), C = g.C, h = blockIdx.y, w = g.w;
  const int64_t win = blockIdx.x;
  unsigned short* Qp = reinterpret_cast<unsigned short*>(sm4);
  unsigned short* Gp = Qp + 3 * NP * PLW;  // dO planes
  float* Ls = reinterpret_cast<float*>(Gp + 3 * NP * PLW);  // lse [NP]
  float* Dd = Ls + NP;                                        // rowsum(dO O) [NP]
  float* tab = Dd + NP;                                       // [R]
  int* k7 = reinterpret_cast<int*>(tab + R);                  // [NP]
  float* wred = reinterpret_cast<float*>(k7 + NP);            // [AM_WAVES][2 HD]
  stage_planes<HD>(Qp, g, win, qkv, 3 * C, h * HD, bqkv, g.scale);
  stage_planes<HD>(Gp, g, win, dO, C, h * HD, nullptr, 1.f);
  for (int t = threadIdx.x; t < NP; t += blockDim.x) {
    float dd = 0.f, l = 0.f;
    if (t < n) {
      const int64_t row = tok_row(g, win, t);
      l = lse[(win * g.nh + h) * n + t];
      if (row >= 0) {
        const float* dop = dO + row * C + h * HD;
        const float* op = O + row * C + h * HD;
#pragma unroll
        for (int e = 0; e < HD; ++e) dd += dop[e] * op[e];
      }
    }
    Dd[t] = dd;
    Ls[t] = l;
    k7[t] = t < n ? key7(t, w) : 0;
  }
  for (int r = threadIdx.x; r < R; r += blockDim.x) tab[r] = table[(int64_t)r * g.nh + h];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kg = lane >> 4;
  const int off0 = (w - 1) * ((2 * w - 1) * (2 * w - 1) + (2 * w - 1) + 1);
  float padk[4] = {0.f, 0.f, 0.f, 0.f}, padv[4] = {0.f, 0.f, 0.f, 0.f};
  for (int jb = wave; jb < NP / 16; jb += AM_WAVES) {
    const int j = jb * 16 + l16;  // this lane's key (the score tiles' column)
    const bool jv = j < n;
    const int64_t row = jv ? tok_row(g, win, j) : -2;
    bf16x8m kf[3], vf[3];
    token_bfrag<HD>(row >= 0 ? qkv + row * 3 * C + C + h * HD
                             : (row == -1 ? bqkv + C + h * HD : nullptr), 1.f, kg, kf);
    token_bfrag<HD>(row >= 0 ? qkv + row * 3 * C + 2 * C + h * HD
                             : (row == -1 ? bqkv + 2 * C + h * HD : nullptr), 1.f, kg, vf);
    const int kj = jv ? k7[j] - off0 : 0;
    f32x4m dk = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
    for (int qs = 0; qs < NP; qs += 32) {
      float pv[8], dsv[8];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int i0 = qs + 16 * sb;
        f32x4m s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          s = mf(rows_afrag(Qp, NP, i0 + l16, kg, m), kf[m], s);
          dp = mf(rows_afrag(Gp, NP, i0 + l16, kg, m), vf[m], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // s[r] = S[query i0 + 4 kg + r][key j]
          const int i = i0 + 4 * kg + r;
          const bool ok = jv && i < n;
          const float p = ok ? expf(s[r] + tab[ok ? k7[i] - kj : 0] - Ls[i]) : 0.f;
          pv[4 * sb + r] = p;
          dsv[4 * sb + r] = p * (dp[r] - Dd[i]);
        }
      }
      bf16x8m pf[3], df[3], gt[3], qt[3];
      split8m(pv, pf);
      split8m(dsv, df);
      tok_tfrag(Gp, NP, qs, lane, gt);
      dv = mf6(gt, pf, dv);  // dv^T [dim][key] += dO^T [dim][query] P [query][key]
      tok_tfrag(Qp, NP, qs, lane, qt);
      dk = mf6(qt, df, dk);  // dk^T [dim][key] += q^T [dim][query] dS [query][key]
    }
    if (row >= 0) {
      if (4 * kg < HD) {
        *reinterpret_cast<float4*>(dqkv + row * 3 * C + C + h * HD + 4 * kg) =
            make_float4(dk[0], dk[1], dk[2], dk[3]);
        *reinterpret_cast<float4*>(dqkv + row * 3 * C + 2 * C + h * HD + 4 * kg) =
            make_float4(dv[0], dv[1], dv[2], dv[3]);
      }
    } else if (row == -1) {  // a padded token: its k / v are the qkv bias
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        padk[r] += dk[r];
        padv[r] += dv[r];
      }
    }
  }
  // padded keys: sum over the 16 key lanes of each group (fixed xor tree), then waves in order
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      padk[r] += __shfl_xor(padk[r], o);
      padv[r] += __shfl_xor(padv[r], o);
    }
  if (l16 == 0 && 4 * kg < HD) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wred[wave * 2 * HD + 4 * kg + r] = padk[r];
      wred[wave * 2 * HD + HD + 4 * kg + r] = padv[r];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * HD) {
    float t = 0.f;
    for (int wv = 0; wv < AM_WAVES; ++wv) t += wred[wv * 2 * HD + threadIdx.x];
    ppart[(win * g.nh + h) * 2 * HD + threadIdx.x] = t;
  }
}

namespace {
size_t mfma_fwd_lds(const AttnGeo& g) {
  const size_t NP = (size_t)((g.n + 31) & ~31);
  return 2 * 3 * NP * PLW * 2 + (size_t)g.R() * 4 + NP * 4;
}
size_t mfma_bwdq_lds(const AttnGeo& g) { return mfma_fwd_lds(g); }
size_t mfma_bwdkv_lds(const AttnGeo& g) {
  const size_t NP = (size_t)((g.n + 31) & ~31);
  return 2 * 3 * NP * PLW * 2 + 3 * NP * 4 + (size_t)g.R() * 4 + (size_t)AM_WAVES * 2 * g.hd * 4;
}
// the MFMA kernels: window 7 (the registry's), head dims 4 .. 16 in multiples of 4
// (SPFF_ATTN_VALU=1: the VALU kernels)
bool use_mfma_attn(const AttnGeo& g) {
  static const bool valu = [] {
    const char* e = getenv("SPFF_ATTN_VALU");
    return e && e[0] == '1';
  }();
  return !valu && g.w == 7 && g.hd <= 16 && g.hd % 4 == 0 && mfma_bwdq_lds(g) <= 160 * 1024 &&
         mfma_bwdkv_lds(g) <= 160 * 1024;
}
template <typename K>
hipError_t set_lds(K kern, size_t lds) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
}  // namespace

static size_t fwd_lds(const AttnGeo& g) {
  return (size_t)(2 * g.n * g.hd + g.R()) * sizeof(float) + (size_t)g.n * sizeof(int);
}
static size_t bwd_lds(const AttnGeo& g) {
  return (size_t)(4 * g.n * g.hd + 2 * g.n + 7 * g.R() + 6 * 2 * g.hd) * sizeof(float) +
         (size_t)g.n * sizeof(int);
}

size_t swin_attn_ws_bytes(const AttnGeo& g) {
  // tpart [nwin][nh][R], ppart [nwin][nh][2 hd], then the MFMA backward's dS [nwin][nh][NP][NP]
  const size_t NP = (size_t)((g.n + 31) & ~31);
  return (size_t)g.nwin() * g.nh * (g.R() + 2 * g.hd + NP * NP) * sizeof(float);
}

#define SPFF_ATTN_HD(X) X(4) X(8) X(12) X(16) X(24) X(32)

hipError_t swin_attn_fwd(const float* qkv, const float* bqkv, const float* table,
                         const AttnGeo& g, float* O, float* lse, hipStream_t s) {
  if (g.n > AT_MAXN || g.C % g.nh) return hipErrorInvalidValue;
  const dim3 grid((unsigned)g.nwin(), g.nh);
  if (use_mfma_attn(g)) {
    const size_t lds = mfma_fwd_lds(g);
    switch (g.hd) {
#define SPFF_FM(HD_)                                                                           \
  case HD_: {                                                                                  \
    hipError_t e0 = set_lds(k_attn_fwd_m<HD_>, lds);                                           \
    if (e0 != hipSuccess) return e0;                                                           \
    hipLaunchKernelGGL(k_attn_fwd_m<HD_>, grid, dim3(AM_THREADS), lds, s, qkv, bqkv, table, g, \
                       O, lse);                                                                \
  } break;
      SPFF_FM(4) SPFF_FM(8) SPFF_FM(12) SPFF_FM(16)
#undef SPFF_FM
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
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
  float* dsw = ppart + (size_t)g.nwin() * g.nh * 2 * g.hd;
  if (use_mfma_attn(g)) {
    const size_t lq = mfma_bwdq_lds(g), lkv = mfma_bwdkv_lds(g);
    const size_t dtl = (size_t)49 * 49 * 13 * sizeof(float);  // k_attn_dtable_m<7> row-pair sums
    {
      hipError_t e0 = set_lds(k_attn_dtable_m<7>, dtl);
      if (e0 != hipSuccess) return e0;
    }
    switch (g.hd) {
#define SPFF_BM(HD_)                                                                             \
  case HD_: {                                                                                    \
    hipError_t e0 = set_lds(k_attn_bwd_q_m<HD_>, lq);                                            \
    if (e0 != hipSuccess) return e0;                                                             \
    if ((e0 = set_lds(k_attn_bwd_kv_m<HD_>, lkv)) != hipSuccess) return e0;                      \
    hipLaunchKernelGGL(k_attn_bwd_q_m<HD_>, grid, dim3(AM_THREADS), lq, s, qkv, bqkv, table, O,  \
                       dO, lse, g, dqkv, dsw);                                                   \
    hipLaunchKernelGGL(k_attn_dtable_m<7>, grid, dim3(256), dtl, s, dsw, g, tpart);               \
    hipLaunchKernelGGL(k_attn_bwd_kv_m<HD_>, grid, dim3(AM_THREADS), lkv, s, qkv, bqkv, table,   \
                       O, dO, lse, g, dqkv, ppart);                                              \
  } break;
      SPFF_BM(4) SPFF_BM(8) SPFF_BM(12) SPFF_BM(16)
#undef SPFF_BM
      default: return hipErrorInvalidValue;
    }
  } else switch (g.hd) {
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
