// Voxel-wise loss: F.cross_entropy(ignore_index) + 0.5 * (1 - hard macro-Dice)
// (reference helpers.py:782-803) and the argmax confusion matrix that both
// the hard-Dice term and per_class_metrics_3d (helpers.py:668-725) need.
//
// One HBM pass over logits [V][K] (channel-last) + int64 labels writes
// dlogits = (softmax - onehot) / N_valid (0 for ignored voxels), per-block CE
// partial sums (fixed grid -> fixed summation order -> deterministic) and an
// integer K x K confusion histogram (LDS, then int64 atomics: order-free).
// The ~100 .item() host syncs of the reference become zero: the finaliser
// kernel computes ce, the hard-Dice term and the loss on the device.
#include "spff_internal.h"
#include <math.h>

namespace spff {

// K up to KMAX classes.  Up to KHIST_LDS the K x (K + 1) confusion histogram lives in LDS
// (integer atomics there, flushed once per workgroup); above it the counts go straight
// to the int64 matrix in HBM, one atomic per distinct cell per wave (integer atomics:
// still order-free and exact).
#ifndef SPFF_LOSS_GRID
#define SPFF_LOSS_GRID 1024  // (2048: 124.8 us per k_loss, 1024: 116.8, 512: 174.9 at 2 x 128^3, K 13)
#endif
constexpr int LOSS_GRID = SPFF_LOSS_GRID, LOSS_T = 256, KMAX = 128, KHIST_LDS = 64;
#ifndef SPFF_LOSS_PF
#define SPFF_LOSS_PF 1
#endif
#ifndef SPFF_LOSS_HOIST
#define SPFF_LOSS_HOIST 1
#endif

// 16-B label pairs, four in flight per thread (one 8-B load per trip ran at ~1 TB/s)
__global__ void k_count_valid(const int64_t* __restrict__ lab, int64_t V, int ignore,
                              unsigned long long* __restrict__ cnt) {
  unsigned long long c = 0;
  const int64_t np = ((uintptr_t)lab & 15) == 0 ? V / 2 : 0;  // aligned pairs
  const longlong2* lp = reinterpret_cast<const longlong2*>(lab);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p0 < np; p0 += 4 * stride) {
    longlong2 r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (p0 + u * stride < np) r[u] = lp[p0 + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (p0 + u * stride < np)
        c += (r[u].x != ignore ? 1ull : 0ull) + (r[u].y != ignore ? 1ull : 0ull);
  }
  for (int64_t v = 2 * np + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V; v += stride)
    c += (lab[v] != ignore) ? 1ull : 0ull;
  __shared__ unsigned long long red[LOSS_T];
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = LOSS_T / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(cnt, red[0]);
}

// Each wave owns 64 consecutive voxels at a time: their 64 x K logits (one
// contiguous run) are staged into the wave's LDS slice with coalesced loads, a
// thread per voxel reads its row from LDS (odd K: conflict-free stride) and
// writes its dlogits row back in place, and the wave stores the run coalesced.
// No per-thread K-arrays (a runtime-K register array would live in scratch).
constexpr int LOSS_WAVES = LOSS_T / 64;
template <bool WITH_CE>
__global__ __launch_bounds__(LOSS_T) void k_loss(const float* __restrict__ x,
                                                 const int64_t* __restrict__ lab, int64_t V, int K,
                                                 int ignore, const int64_t* __restrict__ count,
                                                 float* __restrict__ dx,
                                                 unsigned long long* __restrict__ conf,
                                                 double* __restrict__ part,
                                                 unsigned long long* __restrict__ nbad,
                                                 const float* __restrict__ cw, int clamp1) {
  __shared__ double red[LOSS_T];
  // [LOSS_WAVES][64 K] row stage, then (K <= KHIST_LDS) the [K][K + 1] histogram
  extern __shared__ __attribute__((aligned(16))) float stage[];
  const int K1 = K + 1;  // column K = label outside [0,K) (not ignored)
  const bool lh = K <= KHIST_LDS;
  unsigned int* hist = reinterpret_cast<unsigned int*>(stage + LOSS_WAVES * 64 * K);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sx = stage + wv * 64 * K;
  if (lh)
    for (int i = threadIdx.x; i < K * K1; i += LOSS_T) hist[i] = 0;
  __syncthreads();
  int cell;  // this lane's confusion cell in the current group, -1 for none
  auto tally = [&](int i) { cell = i; };
  // clamp1: the 3DUNet's weighted CE divides by max(N_valid, 1) (models.py:796)
  const float invN =
      WITH_CE ? 1.f / (float)(clamp1 && *count < 1 ? (int64_t)1 : *count) : 0.f;
  double ce = 0.0;
  unsigned int bad = 0;
  const int64_t ngroups = (V + 63) / 64;
  const int64_t gstride = (int64_t)gridDim.x * LOSS_WAVES;
  // (SPFF_LOSS_PF) the rows (K <= 16: at most 4 quads per lane) and labels of the wave's
  // next TWO groups are in flight in registers while this group is worked on (two register
  // sets, used alternately: a wave spends ~2 us of HBM latency per group and only a few
  // hundred cycles of work on it, so one group in flight per wave left the pass latency-
  // bound); the LDS orderings of this path wait for LDS only, so the loads stay in flight
  const bool pf = SPFF_LOSS_PF && K <= 16 && (((uintptr_t)x & 15) == 0);
  struct PF {
    float4 q0, q1, q2, q3;
    int64_t y, g;
  };
  auto prefetch = [&](int64_t g) __attribute__((always_inline)) {
    PF f;
    f.q0 = f.q1 = f.q2 = f.q3 = make_float4(0.f, 0.f, 0.f, 0.f);
    f.y = ignore;
    f.g = -1;
    if (!pf || g >= ngroups) return f;
    const int64_t w0 = g * 64;
    const int nv2 = (int)(V - w0 < 64 ? V - w0 : 64);
    if ((nv2 * K) & 3) return f;  // (a ragged last run takes the plain copy)
    const int n4 = (nv2 * K) >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(x + w0 * K);
    // (streamed once: nontemporal loads, as the norm passes' SPFF_NT reads)
    auto ldn = [&](int i) {
      typedef float nt4 __attribute__((ext_vector_type(4)));
      const nt4 v = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(s4 + i));
      return make_float4(v.x, v.y, v.z, v.w);
    };
    f.q0 = ldn(min(lane, n4 - 1));
    f.q1 = ldn(min(lane + 64, n4 - 1));
    f.q2 = ldn(min(lane + 128, n4 - 1));
    f.q3 = ldn(min(lane + 192, n4 - 1));
    f.y = lane < nv2 ? lab[w0 + lane] : (int64_t)ignore;
    f.g = g;
    return f;
  };
  auto lds_only_sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };
  // one group: its rows into the wave's LDS slice (from the register set f when it holds
  // them), then set f refilled with group g2, the loss / dlogits / confusion of the rows,
  // and the dlogits run stored
  auto group = [&](int64_t grp, PF f, int64_t g2) __attribute__((always_inline)) {
    PF nx;
    const int64_t v0 = grp * 64;
    const int nv = (int)(V - v0 < 64 ? V - v0 : 64);
    const int nf = nv * K;
    int64_t y;
    if (pf && f.g == grp) {
      const int n4 = nf >> 2;
      float4* d4 = reinterpret_cast<float4*>(sx);
      if (lane < n4) d4[lane] = f.q0;
      if (lane + 64 < n4) d4[lane + 64] = f.q1;
      if (lane + 128 < n4) d4[lane + 128] = f.q2;
      if (lane + 192 < n4) d4[lane + 192] = f.q3;
      y = f.y;
    } else {
      // (SPFF_LOSS_HOIST) the label first: its load then overlaps the row copy's
      y = (SPFF_LOSS_HOIST && lane < nv) ? lab[v0 + lane] : (int64_t)ignore;
      wave_copy_rows(sx, x + v0 * K, nf, lane);
    }
    if (pf) {
      lds_only_sync();
      nx = prefetch(g2);
    } else {
      wave_lds_sync();
      nx = prefetch(ngroups);  // (no prefetch)
    }
    cell = -1;
    if (lane < nv) {
      if (!SPFF_LOSS_HOIST) y = lab[v0 + lane];
      float* xr = sx + lane * K;
      float m = xr[0];
      int am = 0;
      for (int k = 1; k < K; ++k) {
        const float t = xr[k];
        if (t > m || (isnan(t) && !isnan(m))) { m = t; am = k; }
      }
      const bool valid = (y != ignore);
      if (valid && (y < 0 || y >= K)) {
        ++bad;
        tally(am * K1 + K);
        if (WITH_CE) for (int k = 0; k < K; ++k) xr[k] = 0.f;
      } else {
        if (valid) tally(am * K1 + (int)y);
        if (WITH_CE) {
          if (valid) {
            const float xy = xr[(int)y];
            float ssum = 0.f;
            for (int k = 0; k < K; ++k) {  // exp once, kept in the row
              const float e = expf(xr[k] - m);
              xr[k] = e;
              ssum += e;
            }
            const float lse = m + logf(ssum);
            // class weights (F.cross_entropy(weight=w), reduction='none'): w[y] * nll
            const float wy = cw ? cw[(int)y] : 1.f;
            ce += cw ? (double)(wy * (lse - xy)) : (double)(lse - xy);
            const float inv = 1.f / ssum;
            for (int k = 0; k < K; ++k) {
              const float p = xr[k] * inv;
              xr[k] = cw ? wy * (p - (k == (int)y ? 1.f : 0.f)) * invN
                         : (p - (k == (int)y ? 1.f : 0.f)) * invN;
            }
          } else {
            for (int k = 0; k < K; ++k) xr[k] = 0.f;
          }
        }
      }
    }
    if (lh) {
      if (cell >= 0) atomicAdd(&hist[cell], 1u);
    } else {
      // K > KHIST_LDS: the counts go to HBM.  Labels are skewed (most voxels of a wave
      // land in a few cells, e.g. background/background), so the wave issues ONE atomic
      // per distinct cell with the number of its lanes in it, not one per voxel.
      unsigned long long todo = __ballot(cell >= 0);
      while (todo) {  // wave-uniform loop
        const int leader = __builtin_ctzll(todo);
        const int c = __shfl(cell, leader);
        const unsigned long long same = __ballot(cell == c) & todo;
        if (lane == leader) atomicAdd(&conf[c], (unsigned long long)__popcll(same));
        todo &= ~same;
      }
    }
    if (pf) lds_only_sync(); else wave_lds_sync();
    if (WITH_CE) wave_copy_rows(dx + v0 * K, sx, nf, lane);
    if (pf) lds_only_sync(); else wave_lds_sync();  // the next group overwrites the slice
    return nx;
  };
  const int64_t g0 = (int64_t)blockIdx.x * LOSS_WAVES + wv;
  PF fa = prefetch(g0);
  PF fb = prefetch(g0 + gstride);
  for (int64_t grp = g0; grp < ngroups; grp += 2 * gstride) {
    fa = group(grp, fa, grp + 2 * gstride);
    if (grp + gstride < ngroups) fb = group(grp + gstride, fb, grp + 3 * gstride);
  }
  if (WITH_CE) {
    red[threadIdx.x] = ce;
    __syncthreads();
    for (int s = LOSS_T / 2; s > 0; s >>= 1) {
      if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
  }
  __syncthreads();
  if (lh)
    for (int i = threadIdx.x; i < K * K1; i += LOSS_T)
      if (hist[i]) atomicAdd(&conf[i], (unsigned long long)hist[i]);
  if (bad && nbad) atomicAdd(nbad, (unsigned long long)bad);
}

// out4 = [ce, loss, dice_loss_part, n_valid]; dice per helpers.py:782-795 in fp64;
// loss = fp32(ce) + fp32(0.5*dice) as torch adds a python float to a fp32 tensor.
__global__ void k_loss_final(const double* __restrict__ part, int nparts,
                             const int64_t* __restrict__ count,
                             const unsigned long long* __restrict__ conf, int K, double smooth,
                             float* __restrict__ out4, int clamp1) {
  // the partials: per-thread strided sums, then a fixed tree (deterministic)
  __shared__ double red[LOSS_T];
  double t = 0.0;
  for (int i = threadIdx.x; i < nparts; i += LOSS_T) t += part[i];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = LOSS_T / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  // per-class hard-Dice terms, one thread per class, summed in class order
  __shared__ double term[KMAX];
  const int K1 = K + 1;
  const int c = threadIdx.x;
  if (c >= 1 && c < K) {
    double tp = (double)conf[c * K1 + c], rowp = 0.0, coll = 0.0;
    for (int j = 0; j < K1; ++j) rowp += (double)conf[c * K1 + j];
    for (int j = 0; j < K; ++j) coll += (double)conf[j * K1 + c];
    const double fp = rowp - tp, fn = coll - tp;
    term[c] = (2.0 * tp + smooth) / (2.0 * tp + fp + fn + smooth);
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double s = red[0];
  const double N = (clamp1 && *count < 1) ? 1.0 : (double)(*count);
  const float ce = (float)(s / N);
  double dsum = 0.0;
  for (int cc = 1; cc < K; ++cc) dsum += term[cc];
  const double macro = K > 1 ? dsum / (double)(K - 1) : 1.0;
  const double dice_loss = 1.0 - macro;
  out4[0] = ce;
  out4[1] = ce + (float)(0.5 * dice_loss);
  out4[2] = (float)dice_loss;
  out4[3] = (float)N;
}

static size_t loss_lds(int K) {
  return (size_t)LOSS_WAVES * 64 * K * sizeof(float) +
         (K <= KHIST_LDS ? (size_t)K * (K + 1) * sizeof(unsigned) : 0);
}
// dynamic LDS above the default 64 KiB (K > ~60) must be granted per kernel
template <bool WITH_CE>
static hipError_t loss_lds_attr(int K) {
  static int granted = 0;
  const int shm = (int)loss_lds(K);
  if (shm <= 65536 || shm <= granted) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_loss<WITH_CE>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, shm);
  if (e == hipSuccess) granted = shm;
  return e;
}

size_t loss_ws_bytes(int64_t V, int K) {
  (void)V; (void)K;
  return LOSS_GRID * sizeof(double) + 64;
}

hipError_t count_valid(const int64_t* labels, int64_t V, int ignore, int64_t* count,
                       hipStream_t s) {
  hipError_t e = spff::zero_async(count, sizeof(int64_t), s);
  if (e != hipSuccess) return e;
  // 256 workgroups: each ends in one 64-bit atomic on the same counter, and 2048 of them
  // queued on that one address took most of the kernel's ~30 us
  hipLaunchKernelGGL(k_count_valid, dim3(256), dim3(LOSS_T), 0, s, labels, V, ignore,
                     reinterpret_cast<unsigned long long*>(count));
  return hipGetLastError();
}

// ws: [LOSS_GRID doubles][int64 count]
hipError_t loss_fwd(const float* logits, const int64_t* labels, int64_t V, int K, int ignore,
                    double smooth, const int64_t* count_override, float* out4, float* dlogits,
                    int64_t* conf, float* ws, hipStream_t s, const float* class_w,
                    int clamp1) {
  if (K > KMAX || K < 1) return hipErrorInvalidValue;
  double* part = reinterpret_cast<double*>(ws);
  int64_t* cnt = reinterpret_cast<int64_t*>(part + LOSS_GRID);
  hipError_t e;
  const int64_t* cptr = count_override;
  if (!cptr) {
    if ((e = count_valid(labels, V, ignore, cnt, s)) != hipSuccess) return e;
    cptr = cnt;
  }
  // (library-wide timing, spff_conv_prof_*: class 3 = the pass as launched here -- confusion
  // zeroing, k_loss, finaliser; class 4 = k_loss alone)
  CProf whole(3, 0.0, s);
  if ((e = spff::zero_async(conf, sizeof(int64_t) * K * (K + 1), s)) != hipSuccess) return e;
  if ((e = loss_lds_attr<true>(K)) != hipSuccess) return e;
  CProf kern(4, 0.0, s);
  hipLaunchKernelGGL(k_loss<true>, dim3(LOSS_GRID), dim3(LOSS_T), loss_lds(K), s, logits, labels,
                     V, K, ignore, cptr, dlogits, reinterpret_cast<unsigned long long*>(conf),
                     part, nullptr, class_w, clamp1);  // (bad labels: conf column K)
  kern.end(s);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(LOSS_T), 0, s, part, LOSS_GRID, cptr,
                     reinterpret_cast<unsigned long long*>(conf), K, smooth, out4, clamp1);
  whole.end(s);
  return hipGetLastError();
}

hipError_t confusion_only(const float* logits, const int64_t* labels, int64_t V, int K, int ignore,
                          int64_t* conf, hipStream_t s) {
  if (K > KMAX || K < 1) return hipErrorInvalidValue;
  hipError_t e = spff::zero_async(conf, sizeof(int64_t) * K * (K + 1), s);
  if (e != hipSuccess) return e;
  if ((e = loss_lds_attr<false>(K)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_loss<false>, dim3(LOSS_GRID), dim3(LOSS_T), loss_lds(K), s, logits, labels,
                     V, K, ignore, nullptr, nullptr, reinterpret_cast<unsigned long long*>(conf),
                     nullptr, nullptr, nullptr, 0);
  return hipGetLastError();
}

}  // namespace spff
