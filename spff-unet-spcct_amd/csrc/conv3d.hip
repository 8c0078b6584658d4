// 3x3x3 ("ksd x 3 x 3") convolution as implicit GEMM on gfx950 fp32 MFMA.
//
// Replaces nn.Conv3d(cin, cout, (ksd,3,3), padding=(ksd//2,1,1), bias=False)
// (reference models.py:616-618) -- forward, input-gradient and weight-gradient.
//
// Design (MI355X-first, see DESIGN.md "conv3d"):
//  * Activations are channel-last [B][D][H][W][C] fp32.
//  * Forward/dgrad: one workgroup (256 threads = 4 waves of 64) owns a
//    TD x TH x TW = 2 x 8 x 16 = 256-voxel output tile x BN output channels.
//    Per reduction chunk of CK input channels it stages the zero-padded input
//    halo (TD+KD-1) x 10 x 18 x CK and the weight slab [taps][CK][BN] in LDS,
//    then runs all KD*9 taps out of LDS: the halo is read 27x from LDS, never
//    re-fetched from L2.  MFMA is v_mfma_f32_32x32x2_f32 (exact fp32, k-ordered
//    fma chain) -- the parity-safe precision.
//  * dgrad = the same kernel on dy with the flipped / transposed weight pack.
//  * wgrad: per tap an MFMA block (rows = 32 ci, cols = 32 co, reduction over
//    voxels); a workgroup owns all taps of a 32x32 (ci, co) tile and a
//    contiguous range of 1x8x16 voxel tiles, register-prefetching the next
//    tile while computing the current one; it writes an fp32 partial slab and
//    a second kernel sums the slabs in a fixed order (deterministic, no float
//    atomics).
#include "spff_internal.h"

namespace spff {

typedef float f32x16 __attribute__((ext_vector_type(16)));

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// ------------------------------------------------------------ weight pack --
__global__ void k_conv_pack(const float* __restrict__ w, float* __restrict__ wt, int Cout,
                            int Cin, int T, int kpad, int npad, int dgrad) {
  // output element (tap, k, n) of wt[T][kpad][npad]
  int64_t total = (int64_t)T * kpad * npad;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int n = (int)(i % npad);
    int k = (int)((i / npad) % kpad);
    int tap = (int)(i / ((int64_t)npad * kpad));
    float v = 0.f;
    if (!dgrad) {
      // k = ci, n = co
      if (k < Cin && n < Cout) v = w[((int64_t)n * Cin + k) * T + tap];
    } else {
      // k = co, n = ci, flipped tap
      if (k < Cout && n < Cin) v = w[((int64_t)k * Cin + n) * T + (T - 1 - tap)];
    }
    wt[i] = v;
  }
}

hipError_t conv_pack_weights(const float* w, float* wt, int Cout, int Cin, int KD, int kpad,
                             int npad, bool dgrad, hipStream_t s) {
  int T = KD * 9;
  int64_t total = (int64_t)T * kpad * npad;
  int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_conv_pack, dim3(grid), dim3(256), 0, s, w, wt, Cout, Cin, T, kpad, npad,
                     dgrad ? 1 : 0);
  return hipGetLastError();
}

int conv3d_bn(int Cout) { return Cout >= 64 ? 64 : 32; }

// ------------------------------------------------------------ fwd / dgrad --
template <int BN, int CK, int KD>
__global__ __launch_bounds__(256) void k_conv3d_fwd(Src2 x, const float* __restrict__ wt,
                                                    Dst2 y, Vol vol, int Cin, int kpad, int Cout,
                                                    int npad, int tilesD, int tilesH,
                                                    int tilesW) {
  constexpr int TD = 2, TH = 8, TW = 16;
  constexpr int HD = TD + KD - 1, HH = TH + 2, HWD = TW + 2;
  constexpr int P = CK + 1;  // odd voxel pitch -> conflict-free 32-lane b32 reads
  constexpr int XS = HD * HH * HWD * P;
  constexpr int T = KD * 9;
  constexpr int NB = BN / 32, MB = 2;
  __shared__ float lds[XS + T * CK * BN];
  float* Xs = lds;
  float* Ws = lds + XS;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int khalf = lane >> 5, l32 = lane & 31;
  int t = blockIdx.x;
  const int twi = t % tilesW; t /= tilesW;
  const int thi = t % tilesH; t /= tilesH;
  const int tdi = t % tilesD;
  const int b = t / tilesD;
  const int d0 = tdi * TD, h0 = thi * TH, w0 = twi * TW;
  const int n0 = blockIdx.y * BN;
  const int D = vol.D, H = vol.H, W = vol.W;

  int hpos[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    int v = wave * 64 + mb * 32 + l32;
    int td = v / (TH * TW), th = (v / TW) % TH, tw = v % TW;
    hpos[mb] = (td * HH + th) * HWD + tw;
  }

  f32x16 acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.f;

  // Register-prefetch pipeline: chunk c0+CK's halo and weight slab are loaded
  // into registers while chunk c0 is computed out of LDS, and written to LDS
  // after the next barrier -- the global-load latency is never on the
  // critical path (the 3 co-resident workgroups then only cover barriers).
  constexpr int Q = CK / 4;
  constexpr int NHX = HD * HH * HWD * Q;            // halo float4 per chunk
  constexpr int NWX = T * CK * (BN / 4);             // weight float4 per chunk
  constexpr int RH = (NHX + 255) / 256, RW = (NWX + 255) / 256;
  float4 hreg[RH], wreg[RW];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      const int i = threadIdx.x + 256 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NHX) {
        const int q = i % Q, pos = i / Q;
        const int hw = pos % HWD, t2 = pos / HWD, hh = t2 % HH, hd = t2 / HH;
        const int gd = d0 + hd - KD / 2, gh = h0 + hh - 1, gw = w0 + hw - 1;
        const int c = c0 + 4 * q;
        const float* p = src_at(x, vol, b, gd, gh, gw, c);
        if (p && c < Cin) v = *reinterpret_cast<const float4*>(p);
      }
      hreg[k] = v;
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const int i = threadIdx.x + 256 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NWX) {
        const int j = i % (BN / 4), row = i / (BN / 4);
        const int tap = row / CK, ci = row % CK;
        v = *reinterpret_cast<const float4*>(wt + ((int64_t)(tap * kpad + c0 + ci)) * npad + n0 +
                                             4 * j);
      }
      wreg[k] = v;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < NHX) {
        const int q = i % Q, pos = i / Q;
        float* d = Xs + pos * P + 4 * q;
        d[0] = hreg[k].x; d[1] = hreg[k].y; d[2] = hreg[k].z; d[3] = hreg[k].w;
      }
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < NWX) {
        const int j = i % (BN / 4), row = i / (BN / 4);
        *reinterpret_cast<float4*>(Ws + row * BN + 4 * j) = wreg[k];
      }
    }
  };

  fetch(0);
  for (int c0 = 0; c0 < kpad; c0 += CK) {
    if (c0) __syncthreads();
    stash();
    __syncthreads();
    if (c0 + CK < kpad) fetch(c0 + CK);
#pragma unroll 3
    for (int tap = 0; tap < T; ++tap) {
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      const int toff = (kd * HH + kh) * HWD + kw;
#pragma unroll
      for (int s = 0; s < CK / 2; ++s) {
        const int ci = 2 * s + khalf;
        float a[MB], bb[NB];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) a[mb] = Xs[(hpos[mb] + toff) * P + ci];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) bb[nb] = Ws[(tap * CK + ci) * BN + nb * 32 + l32];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mb], bb[nb], acc[mb][nb], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: C[i][j], row i = voxel, col j = out channel ----
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * khalf;
      const int v = wave * 64 + mb * 32 + i;
      const int td = v / (TH * TW), th = (v / TW) % TH, tw = v % TW;
      const int gd = d0 + td, gh = h0 + th, gw = w0 + tw;
      if (gd >= D || gh >= H || gw >= W) continue;
      const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + nb * 32 + l32;
        if (n >= Cout) continue;
        float* p = n < y.split ? y.p0 + vox * y.ld0 + n : y.p1 + vox * y.ld1 + (n - y.split);
        *p = acc[mb][nb][r];
      }
    }
  }
}

hipError_t conv3d_fwd(const Src2& x, const float* wt, const Dst2& y, Vol vol, int KD, int Cin,
                      int kpad, int Cout, int npad, hipStream_t s) {
  const int BN = conv3d_bn(Cout);
  if (npad % BN || kpad % 8) return hipErrorInvalidValue;
  const int tilesD = cdiv(vol.D, 2), tilesH = cdiv(vol.H, 8), tilesW = cdiv(vol.W, 16);
  dim3 grid(vol.B * tilesD * tilesH * tilesW, npad / BN);
  if (BN == 64) {
    if (KD == 3)
      hipLaunchKernelGGL((k_conv3d_fwd<64, 4, 3>), grid, dim3(256), 0, s, x, wt, y, vol, Cin, kpad,
                         Cout, npad, tilesD, tilesH, tilesW);
    else
      hipLaunchKernelGGL((k_conv3d_fwd<64, 4, 1>), grid, dim3(256), 0, s, x, wt, y, vol, Cin, kpad,
                         Cout, npad, tilesD, tilesH, tilesW);
  } else {
    if (KD == 3)
      hipLaunchKernelGGL((k_conv3d_fwd<32, 8, 3>), grid, dim3(256), 0, s, x, wt, y, vol, Cin, kpad,
                         Cout, npad, tilesD, tilesH, tilesW);
    else
      hipLaunchKernelGGL((k_conv3d_fwd<32, 8, 1>), grid, dim3(256), 0, s, x, wt, y, vol, Cin, kpad,
                         Cout, npad, tilesD, tilesH, tilesW);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ wgrad --
// dW[co][ci][tap] = sum_v x[v + off(tap)][ci] * dy[v][co].
// One workgroup (4 waves, 1 per SIMD) owns ALL taps x CI ci x 32 co.  MFMA
// rows enumerate (tap, ci) pairs r = tap*CI + ci in blocks of 32 (block j of
// wave w is w + 4j); with CI = 32 a block is one tap (7/7/7/6 blocks for 27
// taps), with CI = 8 (first layer, Cin = 5) four taps.  col = co, reduction =
// voxels (2 per MFMA k-step).  It walks a contiguous range of
// 1 x 8 x 16 voxel tiles; the next tile's halo (3 x 10 x 18 x 32 ch) and dy tile
// (128 x 32) are prefetched into registers while the current tile is computed
// out of LDS, then written to LDS after the compute (loads never exposed).
// Each workgroup writes one fp32 partial slab; k_wgrad_reduce sums the slabs
// in a fixed order (deterministic).
namespace {
constexpr int WG_CO = 32, WG_TH = 8, WG_TW = 16, WG_TV = WG_TH * WG_TW;
inline int wgrad_ci(int Cin) { return Cin <= 8 ? 8 : 32; }
struct WgradPlan {
  int ci, kpad, npad, tilesD, tilesH, tilesW, ntiles, nsplit, tps;
};
WgradPlan wgrad_plan(Vol vol, int Cin, int Cout) {
  WgradPlan p;
  p.ci = wgrad_ci(Cin);
  p.kpad = cdiv(Cin, p.ci) * p.ci;
  p.npad = cdiv(Cout, WG_CO) * WG_CO;
  p.tilesD = vol.D;
  p.tilesH = cdiv(vol.H, WG_TH);
  p.tilesW = cdiv(vol.W, WG_TW);
  p.ntiles = vol.B * p.tilesD * p.tilesH * p.tilesW;
  const int nout = (p.kpad / p.ci) * (p.npad / WG_CO);
  // one workgroup per CU: aim at 2 rounds of 256 CUs, >= 4 tiles per workgroup
  int nsplit = std::max(1, cdiv(512, nout));
  nsplit = std::min(nsplit, std::max(1, p.ntiles / 4));
  p.tps = cdiv(p.ntiles, nsplit);
  p.nsplit = cdiv(p.ntiles, p.tps);
  return p;
}
}  // namespace

template <int KD, int CI>
__global__ __launch_bounds__(256, 1) void k_conv3d_wgrad(Src2 x, const float* __restrict__ dy,
                                                         int lddy, float* __restrict__ part,
                                                         Vol vol, int Cin, int kpad, int Cout,
                                                         int npad, int tilesH, int tilesW,
                                                         int ntiles, int tps) {
  constexpr int HD = KD, HH = WG_TH + 2, HWD = WG_TW + 2;
  constexpr int P = CI + 1;  // odd pitch: 32 lanes reading distinct (tap, ci) avoid conflicts
  constexpr int NPOS = HD * HH * HWD;
  constexpr int XS = NPOS * P;
  constexpr int T = KD * 9;
  constexpr int R = T * CI;                          // (tap, ci) rows
  constexpr int NBLK = (R + 31) / 32;
  constexpr int NJ = (NBLK + 3) / 4;
  constexpr int HQ = CI / 4;                         // float4 per halo voxel
  constexpr int NH = (NPOS * HQ + 255) / 256;        // halo float4 per thread
  constexpr int NY = WG_TV * (WG_CO / 4) / 256;      // dy float4 per thread (= 4)
  __shared__ float lds[XS + WG_TV * WG_CO];
  float* Xs = lds;
  float* Ys = lds + XS;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int khalf = lane >> 5, l32 = lane & 31;
  const int split = blockIdx.x, ci0 = blockIdx.y * CI, co0 = blockIdx.z * WG_CO;
  const int D = vol.D, H = vol.H, W = vol.W;

  int off[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int r = (wave + 4 * j) * 32 + l32;
    const int rr = r < R ? r : 0;  // rows past R: dummy reads of (tap 0, ci 0), never stored
    const int t = rr / CI, ci = rr % CI;
    const int kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
    off[j] = ((kd * HH + kh) * HWD + kw) * P + ci;
  }
  f32x16 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  float4 hreg[NH], yreg[NY];
  auto fetch = [&](int tile) {
    int t = tile;
    const int twi = t % tilesW; t /= tilesW;
    const int thi = t % tilesH; t /= tilesH;
    const int d0 = t % D;
    const int b = t / D;
    const int h0 = thi * WG_TH, w0 = twi * WG_TW;
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int i = threadIdx.x + 256 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NPOS * HQ) {
        const int q = i % HQ, pos = i / HQ;
        const int hw = pos % HWD, t2 = pos / HWD, hh = t2 % HH, hd = t2 / HH;
        const int gd = d0 + hd - KD / 2, gh = h0 + hh - 1, gw = w0 + hw - 1;
        const int c = ci0 + 4 * q;
        const float* p = src_at(x, vol, b, gd, gh, gw, c);
        if (p && c < Cin) v = *reinterpret_cast<const float4*>(p);
      }
      hreg[k] = v;
    }
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int q = i % (WG_CO / 4), kv = i / (WG_CO / 4);
      const int gh = h0 + kv / WG_TW, gw = w0 + kv % WG_TW;
      const int c = co0 + 4 * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gh < H && gw < W && c < Cout) {
        const int64_t vox = (((int64_t)b * D + d0) * H + gh) * W + gw;
        v = *reinterpret_cast<const float4*>(dy + vox * lddy + c);
      }
      yreg[k] = v;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < NPOS * HQ) {
        const int q = i % HQ, pos = i / HQ;
        float* d = Xs + pos * P + 4 * q;
        d[0] = hreg[k].x; d[1] = hreg[k].y; d[2] = hreg[k].z; d[3] = hreg[k].w;
      }
    }
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = threadIdx.x + 256 * k;
      *reinterpret_cast<float4*>(Ys + 4 * i) = yreg[k];
    }
  };

  const int tbeg = split * tps;
  const int tend = min(ntiles, tbeg + tps);
  if (tbeg < tend) fetch(tbeg);
  for (int tile = tbeg; tile < tend; ++tile) {
    __syncthreads();  // previous compute done reading LDS
    stash();
    __syncthreads();
    if (tile + 1 < tend) fetch(tile + 1);  // in flight during the MFMA loop
    // Operands of k-step s+1 are read from LDS while the MFMAs of step s run
    // (two named register sets, static indices).  No per-block guard: a wave
    // with fewer than NJ taps runs a dummy block (tap 0, never stored) -- it
    // would idle on its SIMD anyway, and a divergent-looking branch here
    // de-pipelines the whole MFMA chain.
    float a0[NJ], a1[NJ], b0, b1;
    auto ldk = [&](int s, float (&a)[NJ], float& b) {
      const int k = 2 * s + khalf;
      const int hp = ((k / WG_TW) * HWD + (k % WG_TW)) * P;
      b = Ys[k * WG_CO + l32];
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = Xs[hp + off[j]];
    };
    ldk(0, a0, b0);
#pragma unroll 2
    for (int s = 0; s < WG_TV / 2; s += 2) {
      // sched_barrier pins the order: without it hipcc sinks the prefetch
      // reads back in front of their own MFMAs (lgkmcnt stall per MFMA).
      ldk(s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[j], b0, acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 2 < WG_TV / 2) ldk(s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[j], b1, acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partial slab [split][tap][kpad][npad]: row = ci, col = co
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int blk = wave + 4 * j;
    if (blk >= NBLK) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
      if (row >= R) continue;
      const int tap = row / CI, ci = row % CI;
      part[(((int64_t)split * T + tap) * kpad + ci0 + ci) * npad + co0 + l32] = acc[j][r];
    }
  }
}

// Small layers (fewer than 1024 (ci, 32-co) tiles): one workgroup per 32
// consecutive outputs (co fastest -> coalesced slab reads) x 8 split groups; group g sums splits g, g+8, ... in order, then a fixed-order LDS
// combine: deterministic, and 8x more loads in flight than one thread per output.
__global__ __launch_bounds__(256) void k_wgrad_reduce_co(const float* __restrict__ part,
                                                         float* __restrict__ dw, int nsplit, int T,
                                                         int kpad, int npad, int Cin, int Cout) {
  __shared__ float red[8][33];
  const int64_t total = (int64_t)T * Cin * Cout;
  const int o = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t i = (int64_t)blockIdx.x * 32 + o;
  float s = 0.f;
  int co = 0, ci = 0, tap = 0;
  if (i < total) {
    co = (int)(i % Cout);
    ci = (int)((i / Cout) % Cin);
    tap = (int)(i / ((int64_t)Cout * Cin));
    const int64_t stride = (int64_t)T * kpad * npad;
    const float* p = part + ((int64_t)tap * kpad + ci) * npad + co;
#pragma unroll 4
    for (int k = g; k < nsplit; k += 8) s += p[k * stride];
  }
  red[g][o] = s;
  __syncthreads();
  if (g == 0 && i < total) {
    float t = red[0][o];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][o];
    dw[((int64_t)co * Cin + ci) * T + tap] = t;
  }
}

// One workgroup per (input channel ci, 32 output channels): 256 threads = 32
// co lanes (co fastest -> coalesced slab reads) x 8 split groups.  For every tap
// group g sums splits g, g+8, ... in order into LDS; the groups are then
// combined in fixed order while the tile is written transposed, tap fastest, so
// each co's T taps land contiguously in dw [Cout][Cin][T] (deterministic; 8x
// more loads in flight than one thread per output).
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part,
                                                      float* __restrict__ dw, int nsplit, int T,
                                                      int kpad, int npad, int Cin, int Cout) {
  extern __shared__ float red[];  // [8][T][33]
  const int ci = blockIdx.x, co0 = blockIdx.y * 32;
  const int o = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t stride = (int64_t)T * kpad * npad;
  for (int tap = 0; tap < T; ++tap) {
    float s = 0.f;
    if (co0 + o < Cout) {
      const float* p = part + ((int64_t)tap * kpad + ci) * npad + co0 + o;
      for (int k = g; k < nsplit; k += 8) s += p[k * stride];
    }
    red[(g * T + tap) * 33 + o] = s;
  }
  __syncthreads();
  const int nco = Cout - co0 < 32 ? Cout - co0 : 32;
  for (int w = threadIdx.x; w < nco * T; w += 256) {
    const int c = w / T, tap = w - c * T;
    float t = red[tap * 33 + c];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[(q * T + tap) * 33 + c];
    dw[((int64_t)(co0 + c) * Cin + ci) * T + tap] = t;
  }
}

size_t conv3d_wgrad_ws_bytes(Vol vol, int KD, int Cin, int Cout) {
  WgradPlan p = wgrad_plan(vol, Cin, Cout);
  return std::max((size_t)p.nsplit * KD * 9 * p.kpad * p.npad * sizeof(float),
                  conv3d_wgrad_x_ws_bytes(vol, KD, Cin, Cout));
}

hipError_t conv3d_wgrad_reduce(const float* part, float* dw, int nsplit, int T, int kpad,
                               int npad, int Cin, int Cout, hipStream_t s) {
  // same per-output summation order either way: results are bitwise identical
  if ((int64_t)Cin * ((Cout + 31) / 32) < 1024) {
    const int64_t total = (int64_t)T * Cin * Cout;
    hipLaunchKernelGGL(k_wgrad_reduce_co, dim3((unsigned)((total + 31) / 32)), dim3(256), 0, s,
                       part, dw, nsplit, T, kpad, npad, Cin, Cout);
  } else {
    const size_t lds = (size_t)8 * T * 33 * sizeof(float);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)Cin, (unsigned)((Cout + 31) / 32)),
                       dim3(256), lds, s, part, dw, nsplit, T, kpad, npad, Cin, Cout);
  }
  return hipGetLastError();
}

static hipError_t conv3d_wgrad_(const Src2& x, const float* dy, int lddy, float* dw, Vol vol,
                                int KD, int Cin, int Cout, int math, float* ws, hipStream_t s,
                                const unsigned* xmax, const unsigned* ymax);
hipError_t conv3d_wgrad(const Src2& x, const float* dy, int lddy, float* dw, Vol vol, int KD,
                        int Cin, int Cout, int math, float* ws, hipStream_t s,
                        const unsigned* xmax, const unsigned* ymax) {
  CProf pr(2, 2.0 * (double)nvox(vol) * Cin * Cout * 9 * KD, s);
  const hipError_t e = conv3d_wgrad_(x, dy, lddy, dw, vol, KD, Cin, Cout, math, ws, s, xmax, ymax);
  pr.end(s);
  return e;
}
static hipError_t conv3d_wgrad_(const Src2& x, const float* dy, int lddy, float* dw, Vol vol,
                                int KD, int Cin, int Cout, int math, float* ws, hipStream_t s,
                                const unsigned* xmax, const unsigned* ymax) {
  if (math != SPFF_MATH_F32 && debug_split_wgrad())
    return conv3d_wgrad_x(x, dy, lddy, dw, vol, KD, Cin, Cout, math, ws, s, xmax, ymax);
  if (lddy % 4) return hipErrorInvalidValue;
  WgradPlan p = wgrad_plan(vol, Cin, Cout);
  dim3 grid(p.nsplit, p.kpad / p.ci, p.npad / WG_CO);
#define SPFF_WG(KD_, CI_)                                                                  \
  hipLaunchKernelGGL((k_conv3d_wgrad<KD_, CI_>), grid, dim3(256), 0, s, x, dy, lddy, ws, vol, \
                     Cin, p.kpad, Cout, p.npad, p.tilesH, p.tilesW, p.ntiles, p.tps)
  if (KD == 3) {
    if (p.ci == 8) SPFF_WG(3, 8); else SPFF_WG(3, 32);
  } else {
    if (p.ci == 8) SPFF_WG(1, 8); else SPFF_WG(1, 32);
  }
#undef SPFF_WG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return conv3d_wgrad_reduce(ws, dw, p.nsplit, KD * 9, p.kpad, p.npad, Cin, Cout, s);
}

}  // namespace spff
