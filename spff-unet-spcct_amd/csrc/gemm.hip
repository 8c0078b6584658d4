// GEMM-shaped ops of the SPFF path on fp32 MFMA (v_mfma_f32_32x32x2_f32):
//  * ConvTranspose3d(Cin->Cout, kernel (1,2,2), stride (1,2,2)) + bias
//    (reference up1..up3, models.py:668-672): non-overlapping, so it is one GEMM
//    [Vlow x Cin] . [Cin x 4*Cout] whose columns scatter to the 4 sub-lattices.
//  * the 1x1x1 classifier head nn.Conv3d(f, K, 1) (models.py:674).
// Forward / dgrad use k_gemm (C = A.B, A rows gathered by a functor, C rows
// scattered by a functor).  Weight grads use k_atb (C = X^T.Y reduced over
// voxels, split over voxel ranges into fp32 partial slabs summed in a fixed
// order -> deterministic) which also produces the bias column sums.
#include "spff_internal.h"
#include "bf16split.h"

#include <type_traits>

namespace spff {

typedef float f32x16 __attribute__((ext_vector_type(16)));
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
#ifndef SPFF_GEMM_OCC3_BN
// k_gemm_x column blocks up to this width are compiled for 3 workgroups per CU (<= 168
// VGPRs; the 64-wide up-conv dgrad went 176 -> 168 with 2 spilled): A/B gemm class
// 2.14 -> 2.10 ms/step.  The 128-wide blocks keep 2 (their accumulators alone are 64 VGPRs)
#define SPFF_GEMM_OCC3_BN 64
#endif
#ifndef SPFF_XTY_U1
#define SPFF_XTY_U1 16  // voxel pairs in flight per wave of the one-block k_xty (the head wgrad)
#endif
// SPFF_GEMM_SPLIT=0 (A/B diagnostics): the fp32 MFMA GEMMs for every math
#ifndef SPFF_GEMM_SPLIT
#define SPFF_GEMM_SPLIT 1
#endif
__host__ __device__ inline int64_t cdiv64d(int64_t a, int64_t b) { return (a + b - 1) / b; }
static int num_cus() {
  static int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return c > 0 ? c : 256;
  }();
  return n;
}
// SPFF_GEMM_PERSIST=0 (A/B diagnostics): one row tile per workgroup
#ifndef SPFF_GEMM_PERSIST
#define SPFF_GEMM_PERSIST 1
#endif
// SPFF_GEMM_F16=0 (A/B diagnostics): the GEMMs take the bf16x6 split under SPFF_MATH_F16X3
#ifndef SPFF_GEMM_F16
#define SPFF_GEMM_F16 1
#endif
// GEMM arithmetic of a conv math mode: 0 = fp32 MFMA (k_gemm / k_atb), 1 = the exact
// 3-plane bf16 split (bf16x6), 2 = scaled fp16 planes (f16x3, per-chunk scales, below)
enum { GM_F32 = 0, GM_BF16X6 = 1, GM_F16X3 = 2 };
static inline int gemm_split(int math) {
  if (!SPFF_GEMM_SPLIT) return GM_F32;
  if (math == SPFF_MATH_F16X3) return SPFF_GEMM_F16 ? GM_F16X3 : GM_BF16X6;
  return math == SPFF_MATH_BF16X6 ? GM_BF16X6 : GM_F32;
}
static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------- functors --
// Row-handle interface: prep(m) does the per-row index work once (-1 = row out
// of range); load4(h, k) / put(h + col(n), n, v) are then a few adds.  Index
// math is 32-bit (the launchers check M < 2^31); only byte offsets are 64-bit.
// raw4(h, k, ok): the loaders with kRaw load UNCONDITIONALLY from a clamped address and
// report whether the quad is in range; the kernels zero the out-of-range quads when they
// stage them (ld4 / the validity masks below).  A conditional load (zero or the load,
// merged in a branch) made the compiler wait for the load at the merge -- inside the
// register prefetch, which then ran synchronously before the MFMAs it was meant to overlap.
struct LoadRowsVec {  // A[m][k] = p[m*ld + k]; ld, kmax multiples of 4
  const float* p; int ld; int kmax; int64_t M;
  static constexpr bool kRaw = true;
  __device__ int64_t prep(int64_t m) const { return m < M ? m * ld : -1; }
  __device__ float4 load4(int64_t h, int k) const {
    if (h < 0 || k >= kmax) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(p + h + k);
  }
  __device__ float4 raw4(int64_t h, int k, bool& ok) const {
    ok = h >= 0 && k < kmax;
    return *reinterpret_cast<const float4*>(p + (ok ? h + k : 0));
  }
};
template <class L, class = void>
struct has_raw : std::false_type {};
template <class L>
struct has_raw<L, std::void_t<decltype(L::kRaw)>> : std::true_type {};
// a quad for staging: raw (validity in ok) where the loader has raw4, else load4 (ok = true)
template <class L>
__device__ __forceinline__ float4 ld4(const L& A, int64_t h, int k, bool& ok) {
  if constexpr (has_raw<L>::value) {
    return A.raw4(h, k, ok);
  } else {
    ok = true;
    return A.load4(h, k);
  }
}
__device__ __forceinline__ float4 zero_unless(const float4& v, bool ok) {
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}
struct LoadRowsScalar {  // generic
  const float* p; int ld; int kmax; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? m * ld : -1; }
  __device__ float4 load4(int64_t h, int k) const {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h < 0) return v;
    const float* q = p + h;
    if (k + 0 < kmax) v.x = q[k + 0];
    if (k + 1 < kmax) v.y = q[k + 1];
    if (k + 2 < kmax) v.z = q[k + 2];
    if (k + 3 < kmax) v.w = q[k + 3];
    return v;
  }
};
// log2(v) for a power of two, else -1: the gather / scatter index math then shifts and
// masks instead of dividing (every SPFF level and the 3DUNet's power-of-two extents; a
// runtime division is ~20 VALU, and these GEMMs are VALU-issue-bound, PMC round 3)
static inline int pow2_shift(int v) { return (v > 0 && !(v & (v - 1))) ? __builtin_ctz(v) : -1; }
// q = n / d, r = n % d (sh = log2 d, or -1); sh is uniform, so this is a scalar branch
__device__ __forceinline__ void udivmod_s(uint32_t n, uint32_t d, int sh, uint32_t& q, uint32_t& r) {
  if (sh >= 0) {
    q = n >> sh;
    r = n & (d - 1);
  } else {
    q = n / d;
    r = n - q * d;
  }
}
// A[m][k] = a block output applied as it loads (ActRows, spff_internal.h): the pre-IN rows
// y through lrelu(y al + de) P + Q -- k_act_apply's expression, so bitwise the stored out.
// The row's (b, d) = m / HW = b D + d selects the per-(b, c) and per-(b, d, c) parameters
// (float4 loads, L1/L2-resident); ld = C, a multiple of 4.
struct LoadRowsAct {
  const float* p; int ld; int kmax; int64_t M;
  const float* al; const float* de; const float* PT; const float* QT;
  int D, HW, dsh, hwsh; float neg;
  __device__ int64_t prep(int64_t m) const { return m < M ? m : -1; }
  __device__ float4 load4(int64_t h, int k) const;
  // (no branches: every quad of every row of a fetch can be in flight at once)
  static constexpr bool kRaw = true;
  __device__ float4 raw4(int64_t h, int k, bool& ok) const;
};
// high-res voxel of low-res voxel m's sub-lattice ij = 0: nsub = 4 for the
// (1,2,2) up-convs of SPFF (ij = kh*2 + kw, depth kept), nsub = 8 for the
// 2x2x2 ones of the 3DUNet (ij = (kd*2 + kh)*2 + kw, depth doubled)
__device__ inline int64_t up_high_base(uint32_t m, int D, int Hl, int Wl, int nsub, int wsh = -1,
                                       int hsh = -1) {
  uint32_t t, w, h;
  udivmod_s(m, (uint32_t)Wl, wsh, t, w);
  udivmod_s(t, (uint32_t)Hl, hsh, t, h);  // t = b*D + d
  int64_t tt = t;
  if (nsub == 8) tt = (int64_t)(t / (uint32_t)D) * (2 * D) + 2 * (t % (uint32_t)D);
  return (tt * (2 * Hl) + 2 * h) * (int64_t)(2 * Wl) + 2 * w;
}
// voxel offset of sub-lattice ij from its ij = 0 voxel
__device__ inline int64_t up_sub_off(int ij, int Hl, int Wl) {
  return (int64_t)(ij >> 2) * (4 * (int64_t)Hl * Wl) + ((ij >> 1) & 1) * (2 * Wl) + (ij & 1);
}
__device__ float4 LoadRowsAct::load4(int64_t h, int k) const {
  if (h < 0 || k >= kmax) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 v = *reinterpret_cast<const float4*>(p + h * ld + k);
  uint32_t bd, r, b, d;
  udivmod_s((uint32_t)h, (uint32_t)HW, hwsh, bd, r);
  udivmod_s(bd, (uint32_t)D, dsh, b, d);
  const float4 a = *reinterpret_cast<const float4*>(al + (int64_t)b * ld + k);
  const float4 e = *reinterpret_cast<const float4*>(de + (int64_t)b * ld + k);
  float4 pp = make_float4(1.f, 1.f, 1.f, 1.f), qq = make_float4(0.f, 0.f, 0.f, 0.f);
  if (PT) {
    pp = *reinterpret_cast<const float4*>(PT + (int64_t)bd * ld + k);
    qq = *reinterpret_cast<const float4*>(QT + (int64_t)bd * ld + k);
  }
  auto f = [&](float y, float a_, float e_, float p_, float q_) {
    const float t = y * a_ + e_;
    return (t > 0.f ? t : neg * t) * p_ + q_;
  };
  return make_float4(f(v.x, a.x, e.x, pp.x, qq.x), f(v.y, a.y, e.y, pp.y, qq.y),
                     f(v.z, a.z, e.z, pp.z, qq.z), f(v.w, a.w, e.w, pp.w, qq.w));
}
__device__ float4 LoadRowsAct::raw4(int64_t h, int k, bool& ok) const {
  ok = h >= 0 && k < kmax;
  const int64_t hh = ok ? h : 0;
  const int kk = ok ? k : 0;
  const float4 v = *reinterpret_cast<const float4*>(p + hh * ld + kk);
  uint32_t bd, r, b, d;
  udivmod_s((uint32_t)hh, (uint32_t)HW, hwsh, bd, r);
  udivmod_s(bd, (uint32_t)D, dsh, b, d);
  const float4 a = *reinterpret_cast<const float4*>(al + (int64_t)b * ld + kk);
  const float4 e = *reinterpret_cast<const float4*>(de + (int64_t)b * ld + kk);
  const float* pt = PT ? PT : al;  // (without PT: loaded, then replaced by 1 / 0 below)
  const float* qt = PT ? QT : de;
  const int64_t po = PT ? (int64_t)bd * ld + kk : (int64_t)b * ld + kk;
  const float4 pl = *reinterpret_cast<const float4*>(pt + po);
  const float4 ql = *reinterpret_cast<const float4*>(qt + po);
  // (blended, not branched: a branch would merge loaded and constant values and wait there)
  const float ps = PT ? 1.f : 0.f, pn = 1.f - ps;
  const float4 pp = make_float4(pl.x * ps + pn, pl.y * ps + pn, pl.z * ps + pn, pl.w * ps + pn);
  const float4 qq = make_float4(ql.x * ps, ql.y * ps, ql.z * ps, ql.w * ps);
  auto f = [&](float y, float a_, float e_, float p_, float q_) {
    const float t = y * a_ + e_;
    return (t > 0.f ? t : neg * t) * p_ + q_;
  };
  return make_float4(f(v.x, a.x, e.x, pp.x, qq.x), f(v.y, a.y, e.y, pp.y, qq.y),
                     f(v.z, a.z, e.z, pp.z, qq.z), f(v.w, a.w, e.w, pp.w, qq.w));
}
static LoadRowsAct act_loader(const ActRows& a, int C, int64_t M) {
  return LoadRowsAct{a.y, C, C, M, a.al, a.de, a.PT, a.QT, a.D, a.HW, pow2_shift(a.D),
                     pow2_shift(a.HW), a.neg};
}
static bool act_ok(const ActRows* a, int C) {
  return a && a->y && a->al && a->de && C % 4 == 0 && a->D > 0 && a->HW > 0 &&
         !((reinterpret_cast<uintptr_t>(a->y) | reinterpret_cast<uintptr_t>(a->al) |
            reinterpret_cast<uintptr_t>(a->de) | reinterpret_cast<uintptr_t>(a->PT) |
            reinterpret_cast<uintptr_t>(a->QT)) & 15);
}
struct LoadUpGather {  // A[m][k], k = ij*Cout + co -> dy[high(m,ij)*ld + co]
  const float* p; int ld; int Cout; int D, Hl, Wl; int64_t M; int nsub;
  int csh = -1, wsh = -1, hsh = -1;  // pow2_shift of Cout, Wl, Hl (set by the launchers)
  __device__ int64_t prep(int64_t m) const {
    return m < M ? up_high_base((uint32_t)m, D, Hl, Wl, nsub, wsh, hsh) : -1;
  }
  __device__ float4 load4(int64_t h, int k) const {
    if (h < 0 || k >= nsub * Cout) return make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t ij, co;
    udivmod_s((uint32_t)k, (uint32_t)Cout, csh, ij, co);
    return *reinterpret_cast<const float4*>(p + (h + up_sub_off((int)ij, Hl, Wl)) * ld + co);
  }
  static constexpr bool kRaw = true;
  __device__ float4 raw4(int64_t h, int k, bool& ok) const {
    ok = h >= 0 && k < nsub * Cout;
    uint32_t ij, co;
    udivmod_s((uint32_t)(ok ? k : 0), (uint32_t)Cout, csh, ij, co);
    return *reinterpret_cast<const float4*>(p + ((ok ? h : 0) + up_sub_off((int)ij, Hl, Wl)) * ld +
                                            co);
  }
};
struct StoreRows {  // C[m][n] -> p[m*ld + n] (+bias[n]), n < nmax
  float* p; int ld; int nmax; const float* bias; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? m * ld : -1; }
  __device__ int64_t col(int n) const { return n < nmax ? n : -1; }
  __device__ float bias_of(int n) const { return (bias && n < nmax) ? bias[n] : 0.f; }
  __device__ void put(int64_t idx, float v) const { p[idx] = v; }
  // 16-B column quads (k_gemm_x<..., V4 = true>): columns n .. n+3, n % 4 == 0
  static constexpr bool kVec = true;
  __host__ __device__ bool vec_ok() const { return (ld & 3) == 0 && (nmax & 3) == 0; }
  __device__ float4 bias4(int n) const {
    return (bias && n < nmax) ? *reinterpret_cast<const float4*>(bias + n)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ void put4(int64_t idx, float4 v) const { *reinterpret_cast<float4*>(p + idx) = v; }
};
struct StoreUp {  // C[m][n], n = ij*Cout + co -> y[high(m,ij)*Cout + co] + bias[co]
  float* p; int Cout; const float* bias; int D, Hl, Wl; int64_t M; int nsub;
  int csh = -1, wsh = -1, hsh = -1;  // pow2_shift of Cout, Wl, Hl (set by the launchers)
  // SPFF_MATH_F16X3: max |y| (float bits) of everything stored, into *amax (with *also
  // max-ed in) -- the decoder block input's operand scale, instead of a re-reading pass
  unsigned* amax = nullptr;
  const unsigned* also = nullptr;
  static constexpr bool kAmax = true;
  __device__ int64_t prep(int64_t m) const {
    return m < M ? up_high_base((uint32_t)m, D, Hl, Wl, nsub, wsh, hsh) * Cout : -1;
  }
  __device__ int64_t col(int n) const {
    if (n >= nsub * Cout) return -1;
    uint32_t ij, co;
    udivmod_s((uint32_t)n, (uint32_t)Cout, csh, ij, co);
    return up_sub_off((int)ij, Hl, Wl) * Cout + co;
  }
  __device__ float bias_of(int n) const { return n < nsub * Cout ? bias[n % Cout] : 0.f; }
  __device__ void put(int64_t idx, float v) const { p[idx] = v; }
  static constexpr bool kVec = true;
  __host__ __device__ bool vec_ok() const { return (Cout & 3) == 0; }
  __device__ float4 bias4(int n) const {
    return n < nsub * Cout ? *reinterpret_cast<const float4*>(bias + n % Cout)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ void put4(int64_t idx, float4 v) const { *reinterpret_cast<float4*>(p + idx) = v; }
};

// --- Linear-layer functors (SwinUNETR path, swin.hip) ---
struct LoadRows2 {  // A[m][k] from a two-source channel view (torch.cat([p0, p1], C))
  Src2 x; int kmax; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? m : -1; }
  __device__ float4 load4(int64_t m, int k) const {
    if (m < 0 || k >= kmax) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* q = k < x.split ? x.p0 + m * x.ld0 + k : x.p1 + m * x.ld1 + (k - x.split);
    return *reinterpret_cast<const float4*>(q);
  }
  static constexpr bool kRaw = true;
  __device__ float4 raw4(int64_t m, int k, bool& ok) const {
    ok = m >= 0 && k < kmax;
    const int64_t mm = ok ? m : 0;
    const int kk = ok ? k : 0;
    const float* q = kk < x.split ? x.p0 + mm * x.ld0 + kk : x.p1 + mm * x.ld1 + (kk - x.split);
    return *reinterpret_cast<const float4*>(q);
  }
};
// Patch-embedding gather (Conv3d(Cin, f, k = s = 2)): row m = output voxel of the
// half-resolution grid, k = (ci*2 + kd)*4 + kh*2 + kw (PyTorch's weight flattening)
// of the channel-last input x[b][D][H][W][ld]
struct LoadPatch {
  const float* x; int ld, Cin, D, H, W; int64_t M;  // D, H, W: full resolution
  __device__ int64_t prep(int64_t m) const {
    if (m >= M) return -1;
    const int Wl = W >> 1, Hl = H >> 1, Dl = D >> 1;
    int64_t t = m;
    const int w = (int)(t % Wl); t /= Wl;
    const int h = (int)(t % Hl); t /= Hl;
    const int d = (int)(t % Dl);
    const int64_t b = t / Dl;
    return ((b * D + 2 * d) * H + 2 * h) * (int64_t)W + 2 * w;  // full-res voxel of tap 0
  }
  __device__ float4 load4(int64_t v, int k) const {
    float r[4] = {0.f, 0.f, 0.f, 0.f};
    if (v >= 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j, ci = kk >> 3, t = kk & 7;
        if (ci < Cin) {
          const int64_t off = (((int64_t)(t >> 2) * H + ((t >> 1) & 1)) * W + (t & 1));
          r[j] = x[(v + off) * ld + ci];
        }
      }
    }
    return make_float4(r[0], r[1], r[2], r[3]);
  }
};
struct StoreRowsRes {  // y[m][n] = res[m][n] + v + bias[n]   (residual add)
  float* p; const float* res; int ld, ldr, nmax; const float* bias; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? (m << 16) : -1; }
  __device__ int64_t col(int n) const { return n < nmax ? n : -1; }
  __device__ float bias_of(int n) const { return (bias && n < nmax) ? bias[n] : 0.f; }
  __device__ void put(int64_t idx, float v) const {
    const int64_t m = idx >> 16;
    const int n = (int)(idx & 0xffff);
    p[m * ld + n] = (res ? res[m * ldr + n] : 0.f) + v;
  }
  static constexpr bool kVec = false;
  __host__ __device__ bool vec_ok() const { return false; }
  __device__ float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void put4(int64_t, float4) const {}
};
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  return cdf + x * 0.39894228040143268f * expf(-0.5f * x * x);
}
struct StoreGelu {  // pre[m][n] = v + bias[n]; act[m][n] = gelu(pre)  (nn.GELU, erf form)
  float* pre; float* act; int ld, nmax; const float* bias; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? m * ld : -1; }
  __device__ int64_t col(int n) const { return n < nmax ? n : -1; }
  __device__ float bias_of(int n) const { return (bias && n < nmax) ? bias[n] : 0.f; }
  __device__ void put(int64_t idx, float v) const {
    pre[idx] = v;
    act[idx] = gelu_erf(v);
  }
  static constexpr bool kVec = false;
  __host__ __device__ bool vec_ok() const { return false; }
  __device__ float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void put4(int64_t, float4) const {}
};
struct StoreGeluBwd {  // dpre[m][n] = v * gelu'(pre[m][n])
  float* p; const float* pre; int ld, nmax; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? m * ld : -1; }
  __device__ int64_t col(int n) const { return n < nmax ? n : -1; }
  __device__ float bias_of(int) const { return 0.f; }
  __device__ void put(int64_t idx, float v) const { p[idx] = v * gelu_erf_grad(pre[idx]); }
  static constexpr bool kVec = false;
  __host__ __device__ bool vec_ok() const { return false; }
  __device__ float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void put4(int64_t, float4) const {}
};
struct StoreDst2 {  // C[m][n] -> dst (two-source channel view), optionally accumulated
  Dst2 y; int nmax; int acc; int64_t M;
  __device__ int64_t prep(int64_t m) const { return m < M ? (m << 16) : -1; }
  __device__ int64_t col(int n) const { return n < nmax ? n : -1; }
  __device__ float bias_of(int) const { return 0.f; }
  __device__ void put(int64_t idx, float v) const {
    const int64_t m = idx >> 16;
    const int n = (int)(idx & 0xffff);
    float* q = n < y.split ? y.p0 + m * y.ld0 + n : y.p1 + m * y.ld1 + (n - y.split);
    *q = acc ? *q + v : v;
  }
  static constexpr bool kVec = false;
  __host__ __device__ bool vec_ok() const { return false; }
  __device__ float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void put4(int64_t, float4) const {}
};

// ---------------------------------------------------------------- C = A.B --
// Tile 128 rows x BN cols (BN <= 128: every column of a ConvT / head GEMM up to
// 128 wide in one workgroup, so A is read once), 4 waves each 32 rows x BN,
// K in chunks of 32.  A is loaded 8 rows x 128 B per wave instruction and
// staged transposed (As[k][row], odd pitch: conflict-free b32 stores and
// lane-contiguous ds_read_b32 A fragments), B row-major; the
// next chunk is register-prefetched during this chunk's MFMAs.  B is the packed
// weight [kpad][npad] (kpad a multiple of G_BK).
constexpr int G_BM = 128, G_BK = 32;
template <class AL, class CS, int BN>
__global__ __launch_bounds__(256, 2) void k_gemm(AL A, const float* __restrict__ B, CS C, int kpad,
                                                 int npad) {
  constexpr int NB = BN / 32, PA = G_BM + 1, NRB = BN / 32;  // B float4 per thread
  __shared__ float As[G_BK * PA];
  __shared__ __attribute__((aligned(16))) float Bs[G_BK * BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int khalf = lane >> 5, l32 = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * G_BM;
  const int n0 = blockIdx.y * BN;
  const int aq = tid & 7, arow = tid >> 3;  // A staging: k-quad, row (+32 j)
  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nb][r] = 0.f;
  float4 ra[4], rb[NRB];
  int64_t ah[4];  // this thread's 4 A rows, prepared once
#pragma unroll
  for (int j = 0; j < 4; ++j) ah[j] = A.prep(m0 + arow + 32 * j);
  auto fetch = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) ra[j] = A.load4(ah[j], k0 + 4 * aq);
#pragma unroll
    for (int j = 0; j < NRB; ++j) {
      const int i = tid + 256 * j, r = i / (BN / 4), c4 = i % (BN / 4);
      rb[j] = *reinterpret_cast<const float4*>(B + (int64_t)(k0 + r) * npad + n0 + 4 * c4);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float* d = As + 4 * aq * PA + arow + 32 * j;
      d[0] = ra[j].x; d[PA] = ra[j].y; d[2 * PA] = ra[j].z; d[3 * PA] = ra[j].w;
    }
#pragma unroll
    for (int j = 0; j < NRB; ++j) {
      const int i = tid + 256 * j, r = i / (BN / 4), c4 = i % (BN / 4);
      *reinterpret_cast<float4*>(Bs + r * BN + 4 * c4) = rb[j];
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < kpad; k0 += G_BK) {
    if (k0) __syncthreads();
    stash();
    __syncthreads();
    if (k0 + G_BK < kpad) fetch(k0 + G_BK);
#pragma unroll
    for (int s2 = 0; s2 < G_BK / 2; ++s2) {
      const int k = 2 * s2 + khalf;
      const float a = As[k * PA + wave * 32 + l32];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[k * BN + nb * 32 + l32], acc[nb], 0,
                                                        0, 0);
    }
  }
  int64_t cc[NB];
  float bv[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    cc[nb] = C.col(n0 + nb * 32 + l32);
    bv[nb] = C.bias_of(n0 + nb * 32 + l32);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * khalf;
    const int64_t rh = C.prep(m0 + wave * 32 + i);
    if (rh < 0) continue;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      if (cc[nb] >= 0) C.put(rh + cc[nb], acc[nb][r] + bv[nb]);
  }
}

// ------------------------------------------------- C = A.B, split bf16 --
// The same tile (128 rows x BN cols, K in chunks of 32, 4 waves x 32 rows) on
// v_mfma_f32_16x16x32_bf16 with the exact 3-plane bf16 split of both operands and
// the 6 leading cross products (conv3d_x.hip): ~2.7x fewer MFMA
// cycles than the fp32 MFMA, which bound the up-conv GEMMs (K = 64..128).
// A is split as it is staged, row-major per plane (16-B k-chunk XOR (row bit 3)<<1:
// conflict-free ds_read_b128 A fragments); B (the fp32 packed weight) likewise,
// k-major per plane with 32-B column units XOR-swizzled by k so that the
// ds_read_b64_tr_b16 B fragments (4 k-rows x 16 cols per 16 lanes) are conflict-free.
// Sign alternation: odd chunks stage -B and the accumulator is negated at every
// chunk boundary (the bf16 MFMA's rounding then cancels across chunks).
typedef float f32x4g __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
typedef short i16x4g __attribute__((ext_vector_type(4)));
typedef short i16x8g __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) i16x4g lds_i16x4g;
__device__ __forceinline__ void gsplit4(float4 v, uint2 (&o)[3]) { split4_pk<3>(v, o); }
// 32-B column-unit swizzle of B row k (BN / 16 units per row, 128 / BN rows per 256 B)
// store functors that track the max |element| they store (StoreUp::kAmax)
template <class T, class = void>
struct cs_amax : std::false_type {};
template <class T>
struct cs_amax<T, std::void_t<decltype(T::kAmax)>> : std::integral_constant<bool, T::kAmax> {};

template <int BN>
__device__ __forceinline__ int gx_bsw(int k) {
  constexpr int L = BN == 128 ? 0 : BN == 64 ? 1 : 2;
  return ((k & 3) >> L) | (((k >> 3) & 1) << (2 - L));
}
// |largest element| of a float4
__device__ __forceinline__ float amax4(const float4& v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ float4 ldexp4(const float4& v, int e) {
  return make_float4(ldexpf(v.x, e), ldexpf(v.y, e), ldexpf(v.z, e), ldexpf(v.w, e));
}
// float4 -> the NS planes of the split GEMMs (3 bf16 planes, or NS_F16: 2 fp16 planes of the
// already scaled values)
template <int NS>
__device__ __forceinline__ void gsplit(const float4& v, uint2 (&o)[nplanes(NS)]) {
  split4_pk<NS>(v, o);
}
// f16x3 GEMM chunk scales (NS_F16): the workgroup's largest |element| of the A (X) and B (Y)
// chunk it is about to stage, from every thread's registers -> the chunk's exponents ea, eb
// (f16_scale_exp: max |v| 2^e < 2^14), and the accumulator moved to the units of the new
// chunk's products, 2^(ea + eb).  The exponent may rise by at most 64 per chunk (ea lowered
// by the excess), so the rescaled accumulator cannot overflow; a chunk whose elements are
// that much smaller than everything summed before it then keeps 2^-39 of that bound as
// its fp16 floor, below the fp32 rounding of the sum it joins.  Every thread must call it
// (one workgroup barrier, which also separates the previous chunk's LDS reads from this
// chunk's stores).  The per-(tile, chunk) scales follow the conv kernels' (conv3d_x.hip);
// the weights carry their own per chunk here, so no operand needs a precomputed maximum.
template <int NW, int NACC>
__device__ __forceinline__ void gemm_chunk_scale(float ma, float mb, unsigned (&slot)[2][NW],
                                                 bool first, int& ecur, int& ea, int& eb,
                                                 f32x4g (&acc)[NACC]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ma = fmaxf(ma, __shfl_xor(ma, o));
    mb = fmaxf(mb, __shfl_xor(mb, o));
  }
  if (lane == 0) {
    slot[0][wave] = __float_as_uint(ma);
    slot[1][wave] = __float_as_uint(mb);
  }
  __syncthreads();
  unsigned ba = 0, bb = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    ba = max(ba, slot[0][w]);
    bb = max(bb, slot[1][w]);
  }
  ea = f16_scale_exp(__builtin_amdgcn_readfirstlane(ba));
  eb = f16_scale_exp(__builtin_amdgcn_readfirstlane(bb));
  int e = ea + eb;
  if (first) {
    ecur = e;
    return;
  }
  if (e > ecur + 64) {
    ea -= e - (ecur + 64);
    e = ecur + 64;
  }
  if (e != ecur) {
    const int d = e - ecur;
#pragma unroll
    for (int i = 0; i < NACC; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][r] = ldexpf(acc[i][r], d);
    ecur = e;
  }
}

template <class AL, class CS, int BN, bool V4, int NS = 3>
__global__ __launch_bounds__(256, BN <= SPFF_GEMM_OCC3_BN ? 3 : 2) void k_gemm_x(AL A, const float* __restrict__ B, CS C,
                                                   int kpad, int npad) {
  constexpr int CB = BN / 16, NRB = BN / 32;  // 16-wide col blocks; B float4 per thread
  constexpr int APL = G_BM * G_BK, BPL = G_BK * BN;  // bf16 per plane
  constexpr bool HF = NS == NS_F16;
  constexpr int NP = nplanes(NS);
  __shared__ __attribute__((aligned(16))) unsigned short As[NP * APL];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[NP * BPL];
  __shared__ unsigned gmx[2][4];  // HF: per-wave max |A|, |B| of the chunk
  int ecur = 0, ea = 0, eb = 0;   // HF: accumulator unit 2^ecur; the chunk's A / B exponents
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  // persistent over row tiles blockIdx.x, + gridDim.x, ...: the next tile's first
  // chunk is fetched during the current tile's last MFMAs and its epilogue, so HBM
  // reads stay in flight across tiles (K = 32..128 is only 1-4 chunks per tile)
  const int64_t ntl = cdiv64d(A.M, G_BM);
  int64_t tl = blockIdx.x;
  if (tl >= ntl) return;
  const int n0 = blockIdx.y * BN;
  const int nkc = kpad / G_BK;
  const int aq = tid & 7, arow = tid >> 3;
  f32x4g acc[2][CB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = f32x4g{0.f, 0.f, 0.f, 0.f};
  float4 ra[4], rb[NRB];
  unsigned am = 0;  // bit j: ra[j] is in range (else zeroed at the stash)
  int64_t ah[4];
  auto prep_rows = [&](int64_t t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) ah[j] = A.prep(t * G_BM + arow + 32 * j);
  };
  prep_rows(tl);
  auto fetch = [&](int k0) {
    am = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bool ok;
      ra[j] = ld4(A, ah[j], k0 + 4 * aq, ok);
      am |= ok ? 1u << j : 0u;
    }
#pragma unroll
    for (int j = 0; j < NRB; ++j) {
      const int i = tid + 256 * j, r = i / (BN / 4), c4 = i % (BN / 4);
      rb[j] = *reinterpret_cast<const float4*>(B + (int64_t)(k0 + r) * npad + n0 + 4 * c4);
    }
  };
  auto stash = [&](bool neg) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = arow + 32 * j;
      uint2 o[NP];
      float4 v = zero_unless(ra[j], (am >> j) & 1u);
      if constexpr (HF) v = ldexp4(v, ea);
      gsplit<NS>(v, o);
      const int off = m * G_BK + 8 * ((aq >> 1) ^ ((m & 8) >> 2)) + 4 * (aq & 1);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(As + p * APL + off) = o[p];
    }
#pragma unroll
    for (int j = 0; j < NRB; ++j) {
      const int i = tid + 256 * j, r = i / (BN / 4), c4 = i % (BN / 4);
      float4 v = rb[j];
      if (neg) v = make_float4(-v.x, -v.y, -v.z, -v.w);
      if constexpr (HF) v = ldexp4(v, eb);
      uint2 o[NP];
      gsplit<NS>(v, o);
      const int off = r * BN + 16 * ((c4 >> 2) ^ gx_bsw<BN>(r)) + 4 * (c4 & 3);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(Bs + p * BPL + off) = o[p];
    }
  };
  // A fragment: row 16 rb + l16 of this wave's 32, k-chunk g (8 bf16 = 16 B)
  int aoff[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int m = wave * 32 + rb * 16 + l16;
    aoff[rb] = m * G_BK + 8 * (g ^ ((m & 8) >> 2));
  }
  // B fragment (transposed reads): lane 4q + p of k-group g addresses k-row 8 g + q
  // (and + 4), columns 16 cb + 4 p
  const int q = l16 >> 2, pp = l16 & 3;
  const int kr0 = 8 * g + q, kr1 = kr0 + 4;
  fetch(0);
  bool first = true;
  float amx = 0.f;  // (cs_amax: the largest |value| this thread stored)
  for (;;) {
  const int64_t m0 = tl * G_BM;
  const int64_t tn = tl + gridDim.x;
  for (int kc = 0; kc < nkc; ++kc) {
    if (kc) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = -acc[rb][cb];
    }
    if constexpr (HF) {
      // this chunk's scales (its barrier also orders the previous chunk's LDS reads)
      float ma = 0.f, mb = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) ma = fmaxf(ma, (am >> j) & 1u ? amax4(ra[j]) : 0.f);
#pragma unroll
      for (int j = 0; j < NRB; ++j) mb = fmaxf(mb, amax4(rb[j]));
      gemm_chunk_scale<4, 2 * CB>(ma, mb, gmx, kc == 0, ecur, ea, eb,
                                  reinterpret_cast<f32x4g(&)[2 * CB]>(acc));
    } else {
      if (!first) __syncthreads();  // every wave is past its reads of the previous chunk
    }
    first = false;
    stash(kc & 1);
    __syncthreads();
    {  // one fetch site: the next chunk of this tile, or the first of the next tile (after
       // the last tile: a dummy re-fetch of this tile's first chunk, never staged -- the
       // fetch is unconditional, so no merge of old and new registers waits for the loads)
      const bool last = kc + 1 == nkc;
      if (last && tn < ntl) prep_rows(tn);
      fetch(last ? 0 : (kc + 1) * G_BK);
    }
    bf16x8g a[2][NP];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        a[rb][p] = *reinterpret_cast<const bf16x8g*>(As + p * APL + aoff[rb]);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      bf16x8g b[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const unsigned short* b0 = Bs + p * BPL + kr0 * BN + 16 * (cb ^ gx_bsw<BN>(kr0)) + 4 * pp;
        const unsigned short* b1 = Bs + p * BPL + kr1 * BN + 16 * (cb ^ gx_bsw<BN>(kr1)) + 4 * pp;
        const i16x4g lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4g*)b0);
        const i16x4g hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4g*)b1);
        const i16x8g v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        b[p] = __builtin_bit_cast(bf16x8g, v);
      }
      // V4: operands swapped (B^T . A^T), so the lane holds 4 consecutive output COLUMNS
      // of one row, stored as one 16-B write (the epilogue is store-issue bound otherwise);
      // else the lane holds 4 rows of one column (row-contiguous lanes for narrow pitches)
      auto mf = [](const bf16x8g& x, const bf16x8g& y, f32x4g c) {
        return V4 ? mfma16x32<HF>(y, x, c) : mfma16x32<HF>(x, y, c);
      };
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        f32x4g c = acc[rb][cb];
        if constexpr (HF) {  // hl, lh, hh (the dropped ll <= 2^-22 |ab|)
          c = mf(a[rb][0], b[1], c);
          c = mf(a[rb][1], b[0], c);
          c = mf(a[rb][0], b[0], c);
        } else {
          c = mf(a[rb][1], b[NP - 2], c);
          c = mf(a[rb][0], b[NP - 1], c);
          c = mf(a[rb][NP - 1], b[0], c);
          c = mf(a[rb][0], b[1], c);
          c = mf(a[rb][1], b[0], c);
          c = mf(a[rb][0], b[0], c);
        }
        acc[rb][cb] = c;
      }
    }
  }
  const float sg = ((nkc - 1) & 1) ? -1.f : 1.f;
  // (HF: the accumulator is in units of 2^ecur -- moved back by an exact ldexp)
  auto unscale = [&](float v) { return HF ? ldexpf(v, -ecur) : v; };
  if constexpr (V4) {
    // lane: row 16 rb + l16 of the wave's 32, columns n0 + 16 cb + 4 g + (0..3)
    int64_t rh[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) rh[rb] = C.prep(m0 + wave * 32 + rb * 16 + l16);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int n = n0 + cb * 16 + 4 * g;
      const int64_t c0 = C.col(n);  // the quad is valid or not as a whole (vec_ok)
      const float4 bq = C.bias4(n);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        if (rh[rb] >= 0 && c0 >= 0) {
          const float4 v = make_float4(sg * unscale(acc[rb][cb][0]) + bq.x,
                                       sg * unscale(acc[rb][cb][1]) + bq.y,
                                       sg * unscale(acc[rb][cb][2]) + bq.z,
                                       sg * unscale(acc[rb][cb][3]) + bq.w);
          C.put4(rh[rb] + c0, v);
          if constexpr (cs_amax<CS>::value)
            amx = fmaxf(amx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    }
  } else {
    // lane: rows 16 rb + 4 g + (0..3), column n0 + 16 cb + l16
    int64_t cc[CB];
    float bv[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      cc[cb] = C.col(n0 + cb * 16 + l16);
      bv[cb] = C.bias_of(n0 + cb * 16 + l16);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t rh = C.prep(m0 + wave * 32 + rb * 16 + 4 * g + r);
        if (rh < 0) continue;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          if (cc[cb] >= 0) {
            const float v = sg * unscale(acc[rb][cb][r]) + bv[cb];
            C.put(rh + cc[cb], v);
            if constexpr (cs_amax<CS>::value) amx = fmaxf(amx, fabsf(v));
          }
      }
  }
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = f32x4g{0.f, 0.f, 0.f, 0.f};
  if (tn >= ntl) break;
  tl = tn;
  }
  if constexpr (cs_amax<CS>::value) {
    if (C.amax) {  // (uniform: every thread of the workgroup reaches this)
      if (blockIdx.x == 0 && blockIdx.y == 0 && C.also) amx = fmaxf(amx, __uint_as_float(*C.also));
      block_amax(amx, C.amax);
    }
  }
}

// persistent row tiles: as many workgroups as fit the chip at once
template <int BN, bool V4, int NS, class AL, class CS>
static void launch_gemm_x(const AL& A, const float* B, const CS& C, dim3 grid, int kpad, int npad,
                          hipStream_t s) {
  auto kern = k_gemm_x<AL, CS, BN, V4, NS>;
  static int per_cu = 0;
  if (!per_cu &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess)
    per_cu = 2;
  per_cu = std::max(per_cu, 1);
  const int64_t cap = std::max<int64_t>(1, (int64_t)per_cu * num_cus() / std::max(1, (int)grid.y));
  const dim3 gx((unsigned)(SPFF_GEMM_PERSIST ? std::min<int64_t>(grid.x, cap) : grid.x), grid.y);
  hipLaunchKernelGGL(kern, gx, dim3(256), 0, s, A, B, C, kpad, npad);
}

template <int NS, class AL, class CS>
static void launch_gemm_xs(const AL& A, const float* B, const CS& C, dim3 grid, int BN, int kpad,
                           int npad, hipStream_t s) {
  // 16-B stores of column quads where the output functor and its pitch allow
  const bool v4 = CS::kVec && C.vec_ok();
  if (BN == 128) v4 ? launch_gemm_x<128, true, NS>(A, B, C, grid, kpad, npad, s)
                    : launch_gemm_x<128, false, NS>(A, B, C, grid, kpad, npad, s);
  else if (BN == 64) v4 ? launch_gemm_x<64, true, NS>(A, B, C, grid, kpad, npad, s)
                        : launch_gemm_x<64, false, NS>(A, B, C, grid, kpad, npad, s);
  else v4 ? launch_gemm_x<32, true, NS>(A, B, C, grid, kpad, npad, s)
          : launch_gemm_x<32, false, NS>(A, B, C, grid, kpad, npad, s);
}
// mode (gemm_split): GM_BF16X6 / GM_F16X3 = k_gemm_x with 3 bf16 / 2 scaled fp16 planes;
// GM_F32 = fp32 MFMA k_gemm
template <class AL, class CS>
static hipError_t launch_gemm(const AL& A, const float* B, const CS& C, int64_t M, int kpad,
                              int npad, hipStream_t s, int mode = GM_F32) {
  if (kpad % G_BK || npad % 32 || M >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const int BN = npad % 128 == 0 ? 128 : npad % 64 == 0 ? 64 : 32;
  dim3 grid((unsigned)cdiv64(M, G_BM), npad / BN);
  if (mode == GM_F16X3) {
    launch_gemm_xs<NS_F16>(A, B, C, grid, BN, kpad, npad, s);
    return hipGetLastError();
  }
  if (mode == GM_BF16X6) {
    launch_gemm_xs<3>(A, B, C, grid, BN, kpad, npad, s);
    return hipGetLastError();
  }
  if (BN == 128)
    hipLaunchKernelGGL((k_gemm<AL, CS, 128>), grid, dim3(256), 0, s, A, B, C, kpad, npad);
  else if (BN == 64)
    hipLaunchKernelGGL((k_gemm<AL, CS, 64>), grid, dim3(256), 0, s, A, B, C, kpad, npad);
  else
    hipLaunchKernelGGL((k_gemm<AL, CS, 32>), grid, dim3(256), 0, s, A, B, C, kpad, npad);
  return hipGetLastError();
}

// --------------------------------------------------------- C = X^T . Y -----
// part[split][k1pad][npad] = sum over the split's rows of X[m][k1] * Y[m][n];
// csum[split][npad] = sum of Y[m][n] (bias grads).  Tile 64 x 64, 4 waves 2x2.
constexpr int T_BM = 64;
template <class XL, class YL>
__global__ __launch_bounds__(256) void k_atb(XL X, YL Y, float* __restrict__ part,
                                             float* __restrict__ csum, int64_t M, int64_t rps,
                                             int k1pad, int npad) {
  constexpr int PX = 64 + 1;
  __shared__ float Xs[T_BM * PX];
  __shared__ float Ys[T_BM * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int khalf = lane >> 5, l32 = lane & 31;
  const int split = blockIdx.x, k10 = blockIdx.y * 64, n0 = blockIdx.z * 64;
  const int wr = wave >> 1, wc = wave & 1;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;  // column sum for column n0 + (tid&63), rows (tid>>6) mod 4
  const int64_t mb = (int64_t)split * rps, me = min(M, mb + rps);
  for (int64_t m0 = mb; m0 < me; m0 += T_BM) {
    __syncthreads();
    for (int i = threadIdx.x; i < T_BM * 16; i += 256) {
      const int q = i % 16, r = i / 16;
      const int64_t m = m0 + r;
      const float4 xv = (m < me) ? X.load4(X.prep(m), k10 + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
      float* d = Xs + r * PX + 4 * q;
      d[0] = xv.x; d[1] = xv.y; d[2] = xv.z; d[3] = xv.w;
      const float4 yv = (m < me) ? Y.load4(Y.prep(m), n0 + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(Ys + r * 64 + 4 * q) = yv;
    }
    __syncthreads();
#pragma unroll 8
    for (int s = 0; s < T_BM / 2; ++s) {
      const int k = 2 * s + khalf;
      const float a = Xs[k * PX + wr * 32 + l32];
      const float b = Ys[k * 64 + wc * 32 + l32];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (blockIdx.y == 0) {
      for (int r = wave; r < T_BM; r += 4) cs += Ys[r * 64 + lane];
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * khalf;
    part[((int64_t)split * k1pad + k10 + wr * 32 + i) * npad + n0 + wc * 32 + l32] = acc[r];
  }
  if (blockIdx.y == 0) {
    __shared__ float red[256];
    red[threadIdx.x] = cs;
    __syncthreads();
    if (threadIdx.x < 64) {
      const float v = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] +
                      red[threadIdx.x + 192];
      csum[(int64_t)split * npad + n0 + threadIdx.x] = v;
    }
  }
}

// ------------------------------------------------ C = X^T . Y, split bf16 --
// k_atb on v_mfma_f32_16x16x32_bf16 with the exact 3-plane split (see k_gemm_x):
// the same 64 x 64 output tile per workgroup (4 waves 2 x 2, each 32 x 32 = 2 x 2
// blocks), voxel chunks of 64 = two k-steps.  X and Y are staged voxel-major per
// plane ([m][64 cols], 32-B column units XOR-swizzled by m, gx_bsw<64>) and both
// MFMA operands are gathered with ds_read_b64_tr_b16 (m is the reduction axis of
// both).  Odd chunks stage -Y and the accumulator is negated at every chunk
// boundary.  The bias column sums are taken in fp32 from the staged registers.
// (NS_F16: 2 scaled fp16 planes and 3 products, per-chunk scales of X and Y as in k_gemm_x)
template <class XL, class YL, int NS = 3>
__global__ __launch_bounds__(256, 2) void k_atb_x(XL X, YL Y, float* __restrict__ part,
                                                  float* __restrict__ csum, int64_t M, int64_t rps,
                                                  int k1pad, int npad) {
  constexpr int PL = T_BM * 64;  // bf16 per plane
  constexpr bool HF = NS == NS_F16;
  constexpr int NP = nplanes(NS);
  __shared__ __attribute__((aligned(16))) unsigned short Xs[NP * PL];
  __shared__ __attribute__((aligned(16))) unsigned short Ys[NP * PL];
  __shared__ unsigned gmx[2][4];  // HF: per-wave max |X|, |Y| of the chunk
  int ecur = 0, ex = 0, ey = 0;   // HF: accumulator unit 2^ecur; the chunk's exponents
  __shared__ float4 cred[16][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, pp = l16 & 3;
  const int split = blockIdx.x, k10 = blockIdx.y * 64, n0 = blockIdx.z * 64;
  const int wr = wave >> 1, wc = wave & 1;
  const bool do_cs = blockIdx.y == 0;
  f32x4g acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4g{0.f, 0.f, 0.f, 0.f};
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);  // columns n0 + 4 (tid & 15) .. + 3
  const int sq = tid & 15, sr = tid >> 4;      // staging: col quad, row (+ 16 j)
  float4 xr[4], yr[4];
  unsigned xm = 0, ym = 0;  // validity bits of xr / yr (zeroed at the stash)
  const int64_t mb = (int64_t)split * rps, me = min(M, mb + rps);
  auto fetch = [&](int64_t m0) {
    xm = ym = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + sr + 16 * j;
      const bool ok = m < me;
      const int64_t mm = ok ? m : mb;  // (a row of this split: prep in range)
      bool ox, oy;
      xr[j] = ld4(X, X.prep(mm), k10 + 4 * sq, ox);
      yr[j] = ld4(Y, Y.prep(mm), n0 + 4 * sq, oy);
      xm |= (ok && ox) ? 1u << j : 0u;
      ym |= (ok && oy) ? 1u << j : 0u;
    }
  };
  auto stash = [&](bool neg) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = sr + 16 * j;
      const int off = m * 64 + 16 * ((sq >> 2) ^ gx_bsw<64>(m)) + 4 * (sq & 3);
      uint2 o[NP];
      float4 x = zero_unless(xr[j], (xm >> j) & 1u);
      if constexpr (HF) x = ldexp4(x, ex);
      gsplit<NS>(x, o);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(Xs + p * PL + off) = o[p];
      float4 y = zero_unless(yr[j], (ym >> j) & 1u);
      if (do_cs) { cs.x += y.x; cs.y += y.y; cs.z += y.z; cs.w += y.w; }
      if (neg) y = make_float4(-y.x, -y.y, -y.z, -y.w);
      if constexpr (HF) y = ldexp4(y, ey);
      gsplit<NS>(y, o);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(Ys + p * PL + off) = o[p];
    }
  };
  // operand of row block i (16 columns of X or Y at c0 + 16 i): lane 4q + p of k-group
  // g addresses voxel rows 32 ks + 8 g + q (and + 4), columns c0 + 16 i + 4 p
  auto frag = [&](const unsigned short* img, int ks, int unit) {
    const int r0 = 32 * ks + 8 * g + q, r1 = r0 + 4;
    const unsigned short* a0 = img + r0 * 64 + 16 * (unit ^ gx_bsw<64>(r0)) + 4 * pp;
    const unsigned short* a1 = img + r1 * 64 + 16 * (unit ^ gx_bsw<64>(r1)) + 4 * pp;
    const i16x4g lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4g*)a0);
    const i16x4g hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4g*)a1);
    const i16x8g v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8g, v);
  };
  if (mb < me) fetch(mb);
  int kc = 0;
  for (int64_t m0 = mb; m0 < me; m0 += T_BM, ++kc) {
    if (kc) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = -acc[i][j];
    }
    if constexpr (HF) {
      // this chunk's scales (the barrier inside also orders the previous chunk's reads)
      float mx = 0.f, my = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mx = fmaxf(mx, (xm >> j) & 1u ? amax4(xr[j]) : 0.f);
        my = fmaxf(my, (ym >> j) & 1u ? amax4(yr[j]) : 0.f);
      }
      gemm_chunk_scale<4, 4>(mx, my, gmx, kc == 0, ecur, ex, ey,
                             reinterpret_cast<f32x4g(&)[4]>(acc));
    } else {
      if (kc) __syncthreads();
    }
    stash(kc & 1);
    __syncthreads();
    fetch(m0 + T_BM);  // (unconditional: past the split's rows every quad is masked)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8g a[2][NP], b[2][NP];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          a[i][p] = frag(Xs + p * PL, ks, 2 * wr + i);
          b[i][p] = frag(Ys + p * PL, ks, 2 * wc + i);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4g c = acc[i][j];
          if constexpr (HF) {  // hl, lh, hh
            c = mfma16x32<true>(a[i][0], b[j][1], c);
            c = mfma16x32<true>(a[i][1], b[j][0], c);
            c = mfma16x32<true>(a[i][0], b[j][0], c);
          } else {
            c = mfma16x32<false>(a[i][1], b[j][1], c);
            c = mfma16x32<false>(a[i][0], b[j][NP - 1], c);
            c = mfma16x32<false>(a[i][NP - 1], b[j][0], c);
            c = mfma16x32<false>(a[i][0], b[j][1], c);
            c = mfma16x32<false>(a[i][1], b[j][0], c);
            c = mfma16x32<false>(a[i][0], b[j][0], c);
          }
          acc[i][j] = c;
        }
    }
  }
  const float sg = (kc > 0 && ((kc - 1) & 1)) ? -1.f : 1.f;
  // C[k1][n]: lane holds rows k10 + 32 wr + 16 i + 4 g + r, column n0 + 32 wc + 16 j + l16
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        part[((int64_t)split * k1pad + k10 + 32 * wr + 16 * i + 4 * g + r) * npad + n0 + 32 * wc +
             16 * j + l16] = sg * (HF ? ldexpf(acc[i][j][r], -ecur) : acc[i][j][r]);
  if (do_cs) {
    cred[sr][sq] = cs;
    __syncthreads();
    if (tid < 64) {
      const int c4 = tid >> 2, e = tid & 3;
      float v = 0.f;
      for (int r = 0; r < 16; ++r) {
        const float4 t = cred[r][c4];
        v += e == 0 ? t.x : e == 1 ? t.y : e == 2 ? t.z : t.w;
      }
      csum[(int64_t)split * npad + n0 + tid] = v;
    }
  }
}

// ------------------------------------------------ C = X^T . Y, streaming --
// Weight gradients of the up-convs and the head: part[split][k1][n] = sum over
// the split's voxels of X[v][k1] * Y[v][n] (+ csum[split][n] = sum Y[v][n]).
// K1 and N are small (32..512), the voxel count huge, so the MFMA operands are
// loaded straight from HBM into registers: v_mfma_f32_32x32x2_f32 takes one
// float per lane per operand -- lanes 0-31 read 32 consecutive X (or Y) columns
// of voxel v, lanes 32-63 those of voxel v+1 (128 B rows) -- no LDS staging.
// Each wave owns a (32 TM) x (32 TN) tile over every 4th voxel pair of the
// split; the 4 waves' tiles are summed in LDS in a fixed order.
struct UpGeo {
  int D, Hl, Wl, nsub, Cout;
};
// ACT: X is a block output applied as it loads (ActRows): each lane keeps its column's
// parameters for the (b, d) slab of its current voxel and reloads them when that changes
template <int TM, int TN, bool UP, bool ACT = false>
__global__ __launch_bounds__(256) void k_xty(const float* __restrict__ X, int ldx, int K1,
                                             const float* __restrict__ Y, int ldy, int N, UpGeo g,
                                             float* __restrict__ part, float* __restrict__ csum,
                                             int64_t M, int64_t rps, int k1pad, int npad,
                                             const float* __restrict__ X2, int ldx2, int xsplit,
                                             LoadRowsAct act = {}) {
  constexpr int NE = TM * TN * 16;
  __shared__ float red[4][NE][64];
  __shared__ float cred[4][2][TN][32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, khalf = lane >> 5, l32 = lane & 31;
  const int split = blockIdx.x, k10 = blockIdx.y * 32 * TM, n0 = blockIdx.z * 32 * TN;
  const int64_t vb = (int64_t)split * rps, ve = min(M, vb + rps);
  bool kok[TM], nok[TN];
  int64_t noff[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t) kok[t] = k10 + 32 * t + l32 < K1;
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = n0 + 32 * t + l32;
    nok[t] = n < N;
    if (UP) {
      const int ij = nok[t] ? n / g.Cout : 0;
      noff[t] = nok[t] ? up_sub_off(ij, g.Hl, g.Wl) * ldy + (n - ij * g.Cout) : 0;
    } else {
      noff[t] = nok[t] ? n : 0;
    }
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float cs[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) cs[t] = 0.f;
  const int64_t npairs = (ve - vb + 1) / 2;
  // voxel pairs per iteration, loads issued first: with one 32 x 32 output block (the head:
  // 4-byte loads, 13 of 32 Y lanes live) 16 pairs keep ~4x the bytes in flight per wave that
  // 4 did (the kernel streams x and dy once: bytes in flight, not issue, bound it)
  constexpr int U = (TM == 1 && TN == 1) ? SPFF_XTY_U1 : 8;
  uint32_t cbd = 0xffffffffu;  // ACT: the (b, d) slab the cached parameters belong to
  float ca[TM], ce[TM], cp[TM], cq[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) { ca[t] = 1.f; ce[t] = 0.f; cp[t] = 1.f; cq[t] = 0.f; }
  // !UP: a pair's rows start at a wave-uniform address (scalar registers) and every lane's
  // offset into them is loop-invariant (32 bits): one VGPR per column block instead of a
  // 64-bit address per load in flight (180 -> fewer VGPRs, more waves per CU)
  uint32_t xo[TM], yo[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int col = k10 + 32 * t + l32;
    xo[t] = col < xsplit ? (uint32_t)(khalf * ldx + col) : (uint32_t)(khalf * ldx2 + col - xsplit);
  }
#pragma unroll
  for (int t = 0; t < TN; ++t) yo[t] = (uint32_t)(khalf * ldy + noff[t]);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  for (int64_t p0 = wv; p0 < npairs; p0 += 4 * U) {
    float xa[U][TM], yb[U][TN];
    uint32_t vbd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v0 = vb + 2 * (p0 + 4 * u);  // the pair's first voxel (uniform)
      const int64_t v = v0 + khalf;
      const bool vok = (p0 + 4 * u < npairs) && v < ve;
      if constexpr (ACT) {
        uint32_t r;
        udivmod_s((uint32_t)(vok ? v : vb), (uint32_t)act.HW, act.hwsh, vbd[u], r);
      }
      if constexpr (UP) {
        int64_t yr = 0;
        if (vok) yr = up_high_base((uint32_t)v, g.D, g.Hl, g.Wl, g.nsub) * ldy;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          // X columns >= xsplit come from the second source (torch.cat([X, X2], 1) rows)
          const int col = k10 + 32 * t + l32;
          xa[u][t] = (vok && kok[t])
                         ? (col < xsplit ? X[v * ldx + col] : X2[v * ldx2 + (col - xsplit)])
                         : 0.f;
        }
#pragma unroll
        for (int t = 0; t < TN; ++t) yb[u][t] = (vok && nok[t]) ? Y[yr + noff[t]] : 0.f;
      } else {
        const float* xr = X + v0 * ldx;
        const float* x2r = X2 + v0 * ldx2;
        const float* yr = Y + v0 * ldy;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          const int col = k10 + 32 * t + l32;
          xa[u][t] = (vok && kok[t]) ? (col < xsplit ? xr[xo[t]] : x2r[xo[t]]) : 0.f;
        }
#pragma unroll
        for (int t = 0; t < TN; ++t) yb[u][t] = (vok && nok[t]) ? yr[yo[t]] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (ACT) {
        if (vbd[u] != cbd) {  // (divergent only where a voxel pair straddles two slabs)
          cbd = vbd[u];
          uint32_t b, d;
          udivmod_s(cbd, (uint32_t)act.D, act.dsh, b, d);
#pragma unroll
          for (int t = 0; t < TM; ++t) {
            const int col = k10 + 32 * t + l32;
            if (!kok[t]) continue;
            ca[t] = act.al[(int64_t)b * act.ld + col];
            ce[t] = act.de[(int64_t)b * act.ld + col];
            cp[t] = act.PT ? act.PT[(int64_t)cbd * act.ld + col] : 1.f;
            cq[t] = act.PT ? act.QT[(int64_t)cbd * act.ld + col] : 0.f;
          }
        }
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          // (a row past the split loads 0 and comes out non-zero here: its Y is 0, so its
          //  products vanish; a padding column keeps ca, ce, cp, cq = 1, 0, 1, 0 -> 0)
          const float tt = xa[u][t] * ca[t] + ce[t];
          xa[u][t] = (tt > 0.f ? tt : act.neg * tt) * cp[t] + cq[t];
        }
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) cs[t] += yb[u][t];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[u][a], yb[u][b], acc[a][b], 0, 0, 0);
    }
  }
  // fixed-order combination of the 4 waves
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[wave][(a * TN + b) * 16 + r][lane] = acc[a][b][r];
#pragma unroll
  for (int t = 0; t < TN; ++t) cred[wave][khalf][t][l32] = cs[t];
  __syncthreads();
  for (int e = wave; e < NE; e += 4) {
    const float v = ((red[0][e][lane] + red[1][e][lane]) + red[2][e][lane]) + red[3][e][lane];
    const int ab = e / 16, r = e % 16, a = ab / TN, b = ab % TN;
    const int i = (r & 3) + 8 * (r >> 2) + 4 * khalf;
    part[((int64_t)split * k1pad + k10 + 32 * a + i) * npad + n0 + 32 * b + l32] = v;
  }
  if (blockIdx.y == 0 && wave == 0) {
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      if (khalf) continue;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += cred[w][0][t][l32] + cred[w][1][t][l32];
      csum[(int64_t)split * npad + n0 + 32 * t + l32] = v;
    }
  }
}

struct XtyPlan {
  int tm, tn, k1pad, npad;
  int64_t nsplit, rps;
};
static XtyPlan xty_plan(int64_t M, int K1, int N) {
  XtyPlan p;
  p.tm = K1 > 32 ? 2 : 1;
  p.tn = N > 32 ? 2 : 1;
  p.k1pad = cdiv(K1, 32 * p.tm) * 32 * p.tm;
  p.npad = cdiv(N, 32 * p.tn) * 32 * p.tn;
  const int nout = (p.k1pad / (32 * p.tm)) * (p.npad / (32 * p.tn));
  // ~1024 workgroups (4 per CU) of >= 2048 voxels: enough in flight to stream
  // HBM, few enough partial slabs for k_atb_reduce
  int64_t nsplit = std::max<int64_t>(1, cdiv64(1024, nout));
  nsplit = std::min<int64_t>(nsplit, std::max<int64_t>(1, cdiv64(M, 2048)));
  p.rps = cdiv64(cdiv64(M, nsplit), 2) * 2;
  p.nsplit = cdiv64(M, p.rps);
  return p;
}
static size_t xty_ws_bytes(int64_t M, int K1, int N) {
  const XtyPlan p = xty_plan(M, K1, N);
  return (size_t)p.nsplit * (p.k1pad + 1) * p.npad * sizeof(float);
}
// X rows [M][ldx] (K1 used), Y rows [M][ldy] (N used) or the up-conv gather
static hipError_t launch_xty(const float* X, int ldx, int K1, const float* Y, int ldy, int N,
                             const UpGeo* up, int64_t M, int Cout, int mode, float* dw, float* db,
                             float* ws, hipStream_t s, const float* X2 = nullptr, int ldx2 = 0,
                             int xsplit = 1 << 30, const ActRows* act = nullptr);

// dW layouts: mode 0 = upconv W[Cin][Cout][1][2][2] from C[ci][ij*Cout+co]
//             mode 2 = upconv W[Cin][Cout][2][2][2] from C[ci][ij*Cout+co]
//             mode 1 = head   W[K][Cin]           from C[ci][k]
// One block = 32 outputs x 8 split groups; each group sums its splits in order,
// then the 8 group sums are combined in order (deterministic).  Blocks past
// nwb reduce the bias (column sums, also summed over ij for the upconv).
constexpr int ATB_RG = 32;  // k-groups of k_atb_reduce: 32 x 32 threads per block
__global__ __launch_bounds__(ATB_RG * 32) void k_atb_reduce(const float* __restrict__ part,
                                                    const float* __restrict__ csum,
                                                    float* __restrict__ dw, float* __restrict__ db,
                                                    int nsplit, int k1pad, int npad, int K1, int N,
                                                    int Cout, int mode, int nwb) {
  // thread group g sums slabs g, g + ATB_RG, ... of its block's 32 outputs (up to 1024 slabs:
  // 32 loads each, many in flight), then group 0 adds the ATB_RG partials in order
  __shared__ float red[ATB_RG][33];
  const int jl = threadIdx.x & 31, g = threadIdx.x >> 5;
  float s = 0.f;
  bool valid;
  int k1 = 0, n = 0, co = 0;
  if ((int)blockIdx.x < nwb) {
    const int j = blockIdx.x * 32 + jl;
    k1 = j / npad;
    n = j % npad;
    valid = k1 < K1 && n < N;
    if (valid) {
      const int64_t stride = (int64_t)k1pad * npad;
#pragma unroll 4
      for (int k = g; k < nsplit; k += ATB_RG) s += part[k * stride + j];
    }
  } else {
    co = (blockIdx.x - nwb) * 32 + jl;
    valid = co < Cout;
    if (valid) {
      const int nij = (mode == 0) ? 4 : (mode == 2) ? 8 : 1;
      for (int k = g; k < nsplit; k += ATB_RG)
        for (int ij = 0; ij < nij; ++ij) s += csum[(int64_t)k * npad + ij * Cout + co];
    }
  }
  red[g][jl] = s;
  __syncthreads();
  if (g == 0 && valid) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < ATB_RG; ++q) t += red[q][jl];
    if ((int)blockIdx.x >= nwb) {
      db[co] = t;
    } else if (mode == 0 || mode == 2) {
      const int ij = n / Cout, c = n % Cout;
      dw[((int64_t)k1 * Cout + c) * (mode == 2 ? 8 : 4) + ij] = t;
    } else {
      dw[(int64_t)n * K1 + k1] = t;
    }
  }
}

static hipError_t launch_xty(const float* X, int ldx, int K1, const float* Y, int ldy, int N,
                             const UpGeo* up, int64_t M, int Cout, int mode, float* dw, float* db,
                             float* ws, hipStream_t s, const float* X2, int ldx2, int xsplit,
                             const ActRows* act) {
  if (!X2) X2 = X;
  if (act && (up || xsplit < K1)) return hipErrorInvalidValue;
  if (M >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const XtyPlan p = xty_plan(M, K1, N);
  float* part = ws;
  float* csum = ws + p.nsplit * p.k1pad * p.npad;
  dim3 grid((unsigned)p.nsplit, p.k1pad / (32 * p.tm), p.npad / (32 * p.tn));
  const UpGeo g = up ? *up : UpGeo{1, 1, 1, 4, 1};
#define SPFF_XTY(TM_, TN_, UP_)                                                                   \
  hipLaunchKernelGGL((k_xty<TM_, TN_, UP_>), grid, dim3(256), 0, s, X, ldx, K1, Y, ldy, N, g,     \
                     part, csum, M, p.rps, p.k1pad, p.npad, X2, ldx2, xsplit)
  if (up) {
    if (p.tm == 2 && p.tn == 2) SPFF_XTY(2, 2, true);
    else if (p.tm == 2) SPFF_XTY(2, 1, true);
    else if (p.tn == 2) SPFF_XTY(1, 2, true);
    else SPFF_XTY(1, 1, true);
  } else if (act) {
    const LoadRowsAct la = act_loader(*act, ldx, M);
#define SPFF_XTYA(TM_, TN_)                                                                      \
  hipLaunchKernelGGL((k_xty<TM_, TN_, false, true>), grid, dim3(256), 0, s, X, ldx, K1, Y, ldy, N, \
                     g, part, csum, M, p.rps, p.k1pad, p.npad, X2, ldx2, xsplit, la)
    if (p.tm == 2 && p.tn == 2) SPFF_XTYA(2, 2);
    else if (p.tm == 2) SPFF_XTYA(2, 1);
    else if (p.tn == 2) SPFF_XTYA(1, 2);
    else SPFF_XTYA(1, 1);
#undef SPFF_XTYA
  } else {
    if (p.tm == 2 && p.tn == 2) SPFF_XTY(2, 2, false);
    else if (p.tm == 2) SPFF_XTY(2, 1, false);
    else if (p.tn == 2) SPFF_XTY(1, 2, false);
    else SPFF_XTY(1, 1, false);
  }
#undef SPFF_XTY
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int nwb = cdiv(p.k1pad * p.npad, 32);
  hipLaunchKernelGGL(k_atb_reduce, dim3(nwb + cdiv(Cout, 32)), dim3(ATB_RG * 32), 0, s, part, csum, dw,
                     db, (int)p.nsplit, p.k1pad, p.npad, K1, N, Cout, mode, nwb);
  return hipGetLastError();
}

template <class XL, class YL>
static hipError_t launch_atb(const XL& X, const YL& Y, int64_t M, int K1, int N, int Cout,
                             int mode, float* dw, float* db, float* ws, hipStream_t s,
                             int split = GM_F32) {
  if (M >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const int k1pad = cdiv(K1, 64) * 64, npad = cdiv(N, 64) * 64;
  const int nout = (k1pad / 64) * (npad / 64);
  int64_t nsplit = std::max<int64_t>(1, cdiv64(1024, nout));
  nsplit = std::min<int64_t>(nsplit, std::max<int64_t>(1, cdiv64(M, 4 * T_BM)));
  int64_t rps = cdiv64(cdiv64(M, nsplit), T_BM) * T_BM;
  nsplit = cdiv64(M, rps);
  float* part = ws;
  float* csum = ws + nsplit * k1pad * npad;
  dim3 grid((unsigned)nsplit, k1pad / 64, npad / 64);
  if (split == GM_F16X3)
    hipLaunchKernelGGL((k_atb_x<XL, YL, NS_F16>), grid, dim3(256), 0, s, X, Y, part, csum, M, rps,
                       k1pad, npad);
  else if (split == GM_BF16X6)
    hipLaunchKernelGGL((k_atb_x<XL, YL>), grid, dim3(256), 0, s, X, Y, part, csum, M, rps, k1pad,
                       npad);
  else
    hipLaunchKernelGGL((k_atb<XL, YL>), grid, dim3(256), 0, s, X, Y, part, csum, M, rps, k1pad,
                       npad);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int nwb = cdiv(k1pad * npad, 32);
  hipLaunchKernelGGL(k_atb_reduce, dim3(nwb + cdiv(Cout, 32)), dim3(ATB_RG * 32), 0, s, part, csum, dw,
                     db, (int)nsplit, k1pad, npad, K1, N, Cout, mode, nwb);
  return hipGetLastError();
}

static size_t atb_ws_bytes(int64_t M, int K1, int N) {
  const int k1pad = cdiv(K1, 64) * 64, npad = cdiv(N, 64) * 64;
  const int nout = (k1pad / 64) * (npad / 64);
  int64_t nsplit = std::max<int64_t>(1, cdiv64(1024, nout));
  nsplit = std::min<int64_t>(nsplit, std::max<int64_t>(1, cdiv64(M, 4 * T_BM)));
  int64_t rps = cdiv64(cdiv64(M, nsplit), T_BM) * T_BM;
  nsplit = cdiv64(M, rps);
  return (size_t)nsplit * (k1pad + 1) * npad * sizeof(float);
}

// ---------------------------------------------------------------- packing --
// wf[ci][ij*Cout+co] = W[ci][co][ij] (kpad = roundup(Cin,16), npad = roundup(ns*Cout, 64))
// wd[ij*Cout+co][ci] = W[ci][co][ij] (kpad = roundup(ns*Cout,16), npad = roundup(Cin, 64))
static inline int up_f_kpad(int Cin) { return cdiv(Cin, G_BK) * G_BK; }
static inline int up_f_npad(int Cout, int ns) { return cdiv(ns * Cout, 64) * 64; }
static inline int up_d_kpad(int Cout, int ns) { return cdiv(ns * Cout, G_BK) * G_BK; }
static inline int up_d_npad(int Cin) { return cdiv(Cin, 64) * 64; }

__global__ void k_up_pack(const float* __restrict__ w, float* __restrict__ wf,
                          float* __restrict__ wd, int Cin, int Cout, int ns, int fk, int fn,
                          int dk, int dn) {
  const int tf = fk * fn, td = dk * dn;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tf + td; i += gridDim.x * blockDim.x) {
    if (i < tf) {
      const int n = i % fn, k = i / fn;
      float v = 0.f;
      if (k < Cin && n < ns * Cout) v = w[((int64_t)k * Cout + n % Cout) * ns + n / Cout];
      wf[i] = v;
    } else {
      const int j = i - tf;
      const int n = j % dn, k = j / dn;
      float v = 0.f;
      if (k < ns * Cout && n < Cin) v = w[((int64_t)n * Cout + k % Cout) * ns + k / Cout];
      wd[j] = v;
    }
  }
}

hipError_t upconv_pack(const float* w, float* wf, float* wd, int Cin, int Cout, hipStream_t s,
                       int ns) {
  const int fk = up_f_kpad(Cin), fn = up_f_npad(Cout, ns), dk = up_d_kpad(Cout, ns),
            dn = up_d_npad(Cin);
  const int total = fk * fn + dk * dn;
  hipLaunchKernelGGL(k_up_pack, dim3(cdiv(total, 256)), dim3(256), 0, s, w, wf, wd, Cin, Cout, ns,
                     fk, fn, dk, dn);
  return hipGetLastError();
}

hipError_t upconv_fwd(const float* x, const float* wf, const float* bias, float* y, Vol low,
                      int Cin, int Cout, hipStream_t s, int ns, int math, const ActRows* act,
                      unsigned* amax, const unsigned* also) {
  const int64_t M = nvox(low);
  if (act && !act_ok(act, Cin)) return hipErrorInvalidValue;
  if (amax && !gemm_split(math)) return hipErrorInvalidValue;  // (the split GEMM tracks it)
  StoreUp C{y, Cout, bias, low.D, low.H, low.W, M, ns, pow2_shift(Cout), pow2_shift(low.W),
            pow2_shift(low.H), amax, also};
  if (act)
    return launch_gemm(act_loader(*act, Cin, M), wf, C, M, up_f_kpad(Cin), up_f_npad(Cout, ns),
                       s, gemm_split(math));
  LoadRowsVec A{x, Cin, Cin, M};
  return launch_gemm(A, wf, C, M, up_f_kpad(Cin), up_f_npad(Cout, ns), s, gemm_split(math));
}

hipError_t upconv_dgrad(const float* dy, int lddy, const float* wd, float* dx, Vol low, int Cin,
                        int Cout, hipStream_t s, int ns, int math) {
  const int64_t M = nvox(low);
  LoadUpGather A{dy, lddy, Cout, low.D, low.H, low.W, M, ns, pow2_shift(Cout),
                 pow2_shift(low.W), pow2_shift(low.H)};
  StoreRows C{dx, Cin, Cin, nullptr, M};
  return launch_gemm(A, wd, C, M, up_d_kpad(Cout, ns), up_d_npad(Cin), s, gemm_split(math));
}

size_t upconv_wgrad_ws_bytes(Vol low, int Cin, int Cout, int ns) {
  return atb_ws_bytes(nvox(low), Cin, ns * Cout);
}

hipError_t upconv_wgrad(const float* x, const float* dy, int lddy, float* dw, float* db, Vol low,
                        int Cin, int Cout, float* ws, hipStream_t s, int ns, int math,
                        const ActRows* act) {
  // (the streaming k_xty measured 15 % slower here: the up-conv gather needs a
  //  per-voxel index division, and 64 x 64 LDS tiles reuse X and Y better)
  const int64_t M = nvox(low);
  LoadUpGather Y{dy, lddy, Cout, low.D, low.H, low.W, M, ns, pow2_shift(Cout),
                 pow2_shift(low.W), pow2_shift(low.H)};
  if (act) {
    if (!act_ok(act, Cin)) return hipErrorInvalidValue;
    return launch_atb(act_loader(*act, Cin, M), Y, M, Cin, ns * Cout, Cout, ns == 8 ? 2 : 0, dw,
                      db, ws, s, gemm_split(math));
  }
  LoadRowsVec X{x, Cin, Cin, M};
  return launch_atb(X, Y, M, Cin, ns * Cout, Cout, ns == 8 ? 2 : 0, dw, db, ws, s,
                    gemm_split(math));
}

// ------------------------------------------------------------------- head --
// The head's packed weights are produced on the fly by tiny kernels into ws.
__global__ void k_head_pack(const float* __restrict__ w, float* __restrict__ wf,
                            float* __restrict__ wd, int Cin, int K, int fk, int fn, int dk,
                            int dn) {
  const int tf = fk * fn, td = dk * dn;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tf + td; i += gridDim.x * blockDim.x) {
    if (i < tf) {  // wf[ci][k]
      const int n = i % fn, k = i / fn;
      wf[i] = (k < Cin && n < K) ? w[(int64_t)n * Cin + k] : 0.f;
    } else {  // wd[k][ci]
      const int j = i - tf;
      const int n = j % dn, k = j / dn;
      wd[j] = (k < K && n < Cin) ? w[(int64_t)k * Cin + n] : 0.f;
    }
  }
}

static inline int head_fk(int Cin) { return cdiv(Cin, G_BK) * G_BK; }
static inline int head_fn(int K) { return cdiv(K, 32) * 32; }
static inline int head_dk(int K) { return cdiv(K, G_BK) * G_BK; }
static inline int head_dn(int Cin) { return cdiv(Cin, 32) * 32; }

// Streaming head (Cin = 32 or 64, K <= 32): the head is memory-bound (Cin floats in, K out
// per voxel) and the K <= 32 column MFMA GEMM ran it at ~3.3 TB/s.  A block takes 256
// consecutive rows: a coalesced float4 pass stages them in LDS (the loader applies the
// block-output activation, as LoadRowsAct does in the GEMM), each thread then forms its
// row's K dot products in fp32 (c in order, the uniform weights through the scalar cache),
// and a second coalesced pass stores the block's [256][K] outputs.  The input gradient is
// the mirror image.  W = wd [K][dn] (head_pack's dgrad image, the reference layout).
// (SPFF_HEAD_STREAM=0, diagnostics / A/B only: the GEMM path again)
static bool head_stream_ok(int Cin, int K) {
  static const bool off = [] {
    const char* e = getenv("SPFF_HEAD_STREAM");
    return e && e[0] == '0';
  }();
  return !off && (Cin == 32 || Cin == 64) && K >= 1 && K <= 32;
}
template <int C, int KM, class L>
__global__ __launch_bounds__(256) void k_head_fwd_s(L A, const float* __restrict__ wd, int dn,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ y, int64_t V, int K) {
  constexpr int CP = C + 1, Q = C / 4;
  __shared__ float tile[256 * CP];
  const int tid = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < V; r0 += (int64_t)gridDim.x * 256) {
    const int nr = (int)(V - r0 < 256 ? V - r0 : 256);
    float4 v[Q];
    bool done = false;
    if constexpr (std::is_same<L, LoadRowsAct>::value) {
      // HW % 256 == 0: the block's 256 rows share one (b, d), and thread tid always takes
      // channel quad tid % Q, so its activation coefficients load once per block
      if (A.HW % 256 == 0) {
        const int64_t bd = r0 / A.HW, b = bd / A.D;
        const int c = 4 * (tid % Q);
        const float4 a = *reinterpret_cast<const float4*>(A.al + b * A.ld + c);
        const float4 e = *reinterpret_cast<const float4*>(A.de + b * A.ld + c);
        float4 pp = make_float4(1.f, 1.f, 1.f, 1.f), qq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (A.PT) {
          pp = *reinterpret_cast<const float4*>(A.PT + bd * A.ld + c);
          qq = *reinterpret_cast<const float4*>(A.QT + bd * A.ld + c);
        }
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          const int rr = (tid + j * 256) / Q;
          v[j] = *reinterpret_cast<const float4*>(A.p + (r0 + (rr < nr ? rr : 0)) * A.ld + c);
        }
        auto f = [&](float y, float a_, float e_, float p_, float q_) {  // LoadRowsAct::load4's
          const float t = y * a_ + e_;
          return (t > 0.f ? t : A.neg * t) * p_ + q_;
        };
#pragma unroll
        for (int j = 0; j < Q; ++j)
          v[j] = make_float4(f(v[j].x, a.x, e.x, pp.x, qq.x), f(v[j].y, a.y, e.y, pp.y, qq.y),
                             f(v[j].z, a.z, e.z, pp.z, qq.z), f(v[j].w, a.w, e.w, pp.w, qq.w));
        done = true;
      }
    }
    if (!done) {
#pragma unroll
      for (int j = 0; j < Q; ++j) {  // Q quads per thread in flight
        const int i = tid + j * 256, rr = i / Q;
        v[j] = A.load4(A.prep(r0 + (rr < nr ? rr : 0)), 4 * (i % Q));
      }
    }
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int i = tid + j * 256;
      float* t = tile + (i / Q) * CP + 4 * (i % Q);
      t[0] = v[j].x; t[1] = v[j].y; t[2] = v[j].z; t[3] = v[j].w;
    }
    __syncthreads();
    float o[KM];
    {
      float a[C];
#pragma unroll
      for (int c = 0; c < C; ++c) a[c] = tile[tid * CP + c];
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        float s = 0.f;
        if (k < K) {
#pragma unroll
          for (int c = 0; c < C; ++c) s = fmaf(a[c], wd[k * dn + c], s);
          s += bias ? bias[k] : 0.f;
        }
        o[k] = s;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < K) tile[tid * K + k] = o[k];
    __syncthreads();
    const int n = nr * K;
    float* yb = y + r0 * K;  // 16-B aligned: r0 is a multiple of 256
    for (int i = tid; i < n / 4; i += 256)
      reinterpret_cast<float4*>(yb)[i] =
          make_float4(tile[4 * i], tile[4 * i + 1], tile[4 * i + 2], tile[4 * i + 3]);
    for (int i = (n / 4) * 4 + tid; i < n; i += 256) yb[i] = tile[i];
    __syncthreads();
  }
}
template <int C, int KM>
__global__ __launch_bounds__(256) void k_head_dgrad_s(const float* __restrict__ dy,
                                                      const float* __restrict__ wd, int dn,
                                                      float* __restrict__ dx, int64_t V, int K) {
  constexpr int CP = C + 1, NL = KM / 4;
  __shared__ float tile[256 * CP];  // the block's dy rows [256][K], then its dx rows [256][CP]
  const int tid = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < V; r0 += (int64_t)gridDim.x * 256) {
    const int nr = (int)(V - r0 < 256 ? V - r0 : 256);
    const int n = nr * K, n4 = n / 4;
    const float* gb = dy + r0 * K;  // 16-B aligned: r0 is a multiple of 256
    float4 gv[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {  // NL quads per thread in flight
      const int i = tid + j * 256;
      gv[j] = i < n4 ? reinterpret_cast<const float4*>(gb)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * 256;
      if (i < n4) {
        tile[4 * i] = gv[j].x; tile[4 * i + 1] = gv[j].y;
        tile[4 * i + 2] = gv[j].z; tile[4 * i + 3] = gv[j].w;
      }
    }
    for (int i = n4 * 4 + tid; i < n; i += 256) tile[i] = gb[i];
    __syncthreads();
    float g[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) g[k] = (k < K && tid < nr) ? tile[tid * K + k] : 0.f;
    __syncthreads();
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < K) {
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = fmaf(g[k], wd[k * dn + c], acc[c]);
      }
#pragma unroll
    for (int c = 0; c < C; ++c) tile[tid * CP + c] = acc[c];
    __syncthreads();
    float* xb = dx + r0 * C;
    for (int i = tid; i < nr * (C / 4); i += 256) {
      const float* t = tile + (i / (C / 4)) * CP + 4 * (i % (C / 4));
      reinterpret_cast<float4*>(xb)[i] = make_float4(t[0], t[1], t[2], t[3]);
    }
    __syncthreads();
  }
}
static unsigned head_grid(int64_t V) {
  return (unsigned)std::min<int64_t>((V + 255) / 256, 8192);
}
template <int C, int KM, class L>
static hipError_t head_fwd_s(const L& A, const float* wd, int dn, const float* b, float* y,
                             int64_t V, int K, hipStream_t s) {
  hipLaunchKernelGGL((k_head_fwd_s<C, KM, L>), dim3(head_grid(V)), dim3(256), 0, s, A, wd, dn, b,
                     y, V, K);
  return hipGetLastError();
}
template <class L>
static hipError_t head_fwd_stream(const L& A, const float* wd, int Cin, const float* b, float* y,
                                  int64_t V, int K, hipStream_t s) {
  const int dn = head_dn(Cin);
  if (Cin == 32)
    return K <= 16 ? head_fwd_s<32, 16>(A, wd, dn, b, y, V, K, s)
                   : head_fwd_s<32, 32>(A, wd, dn, b, y, V, K, s);
  return K <= 16 ? head_fwd_s<64, 16>(A, wd, dn, b, y, V, K, s)
                 : head_fwd_s<64, 32>(A, wd, dn, b, y, V, K, s);
}
static hipError_t head_dgrad_stream(const float* dy, const float* wd, float* dx, int64_t V,
                                    int Cin, int K, hipStream_t s) {
  const int dn = head_dn(Cin);
  const dim3 g(head_grid(V)), b(256);
  if (Cin == 32) {
    if (K <= 16) hipLaunchKernelGGL((k_head_dgrad_s<32, 16>), g, b, 0, s, dy, wd, dn, dx, V, K);
    else hipLaunchKernelGGL((k_head_dgrad_s<32, 32>), g, b, 0, s, dy, wd, dn, dx, V, K);
  } else {
    if (K <= 16) hipLaunchKernelGGL((k_head_dgrad_s<64, 16>), g, b, 0, s, dy, wd, dn, dx, V, K);
    else hipLaunchKernelGGL((k_head_dgrad_s<64, 32>), g, b, 0, s, dy, wd, dn, dx, V, K);
  }
  return hipGetLastError();
}

hipError_t head_fwd(const float* x, const float* wf, const float* b, float* y, int64_t V, int Cin,
                    int K, hipStream_t s, int math, const ActRows* act) {
  StoreRows C{y, K, K, b, V};
  if (act && !act_ok(act, Cin)) return hipErrorInvalidValue;
  const bool y16 = !(reinterpret_cast<uintptr_t>(y) & 15);
  if (head_stream_ok(Cin, K) && y16 && (act || !(reinterpret_cast<uintptr_t>(x) & 15))) {
    const float* wd = wf + head_pack_dgrad_offset(Cin, K);
    if (act) return head_fwd_stream(act_loader(*act, Cin, V), wd, Cin, b, y, V, K, s);
    return head_fwd_stream(LoadRowsVec{x, Cin, Cin, V}, wd, Cin, b, y, V, K, s);
  }
  if (act)
    return launch_gemm(act_loader(*act, Cin, V), wf, C, V, head_fk(Cin), head_fn(K), s,
                       gemm_split(math));
  LoadRowsVec A{x, Cin, Cin, V};
  return launch_gemm(A, wf, C, V, head_fk(Cin), head_fn(K), s, gemm_split(math));
}

hipError_t head_pack(const float* w, float* wf, float* wd, int Cin, int K, hipStream_t s) {
  const int fk = head_fk(Cin), fn = head_fn(K), dk = head_dk(K), dn = head_dn(Cin);
  const int total = fk * fn + dk * dn;
  hipLaunchKernelGGL(k_head_pack, dim3(cdiv(total, 256)), dim3(256), 0, s, w, wf, wd, Cin, K, fk,
                     fn, dk, dn);
  return hipGetLastError();
}
size_t head_pack_floats(int Cin, int K) {
  return (size_t)head_fk(Cin) * head_fn(K) + (size_t)head_dk(K) * head_dn(Cin);
}
size_t head_pack_dgrad_offset(int Cin, int K) { return (size_t)head_fk(Cin) * head_fn(K); }
size_t upconv_pack_floats(int Cin, int Cout, int ns) {
  return (size_t)up_f_kpad(Cin) * up_f_npad(Cout, ns) +
         (size_t)up_d_kpad(Cout, ns) * up_d_npad(Cin);
}
size_t upconv_pack_dgrad_offset(int Cin, int Cout, int ns) {
  return (size_t)up_f_kpad(Cin) * up_f_npad(Cout, ns);
}

hipError_t head_dgrad(const float* dy, const float* wd, float* dx, int64_t V, int Cin, int K,
                      hipStream_t s, int math) {
  if (head_stream_ok(Cin, K) &&
      !((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx)) & 15))
    return head_dgrad_stream(dy, wd, dx, V, Cin, K, s);
  LoadRowsScalar A{dy, K, K, V};
  StoreRows C{dx, Cin, Cin, nullptr, V};
  return launch_gemm(A, wd, C, V, head_dk(K), head_dn(Cin), s, gemm_split(math));
}

size_t head_wgrad_ws_bytes(int64_t V, int Cin, int K) { return xty_ws_bytes(V, Cin, K); }

hipError_t head_wgrad(const float* x, const float* dy, float* dw, float* db, int64_t V, int Cin,
                      int K, float* ws, hipStream_t s, const ActRows* act) {
  if (act) {
    if (!act_ok(act, Cin)) return hipErrorInvalidValue;
    return launch_xty(act->y, Cin, Cin, dy, K, K, nullptr, V, K, 1, dw, db, ws, s, nullptr, 0,
                      1 << 30, act);
  }
  return launch_xty(x, Cin, Cin, dy, K, K, nullptr, V, K, 1, dw, db, ws, s);
}

// ------------------------------------------------------- linear layers --
// nn.Linear / 1x1x1 Conv3d on channel-last rows: y = x W^T + b with W [N][K]
// (PyTorch layout), packed by head_pack(w, wf, wd, K, N) (wf = W^T, wd = W).
hipError_t linear_fwd(const float* x, int ldx, int K, const float* wf, const float* b, float* y,
                      int ldy, int N, int64_t M, const float* res, int ldres, hipStream_t s) {
  if (K > 65535 || N > 65535) return hipErrorInvalidValue;
  LoadRowsVec A{x, ldx, K, M};
  StoreRowsRes C{y, res, ldy, ldres, N, b, M};
  return launch_gemm(A, wf, C, M, head_fk(K), head_fn(N), s);
}
hipError_t linear_fwd2(const Src2& x, int K, const float* wf, const float* b, float* y, int ldy,
                       int N, int64_t M, hipStream_t s) {
  LoadRows2 A{x, K, M};
  StoreRowsRes C{y, nullptr, ldy, 0, N, b, M};
  return launch_gemm(A, wf, C, M, head_fk(K), head_fn(N), s);
}
hipError_t linear_fwd_gelu(const float* x, int ldx, int K, const float* wf, const float* b,
                           float* pre, float* act, int N, int64_t M, hipStream_t s) {
  LoadRowsVec A{x, ldx, K, M};
  StoreGelu C{pre, act, N, N, b, M};
  return launch_gemm(A, wf, C, M, head_fk(K), head_fn(N), s);
}
hipError_t patch_embed_fwd(const float* x, int ldx, int Cin, int D, int H, int W, int B,
                           const float* wf, const float* b, float* y, int N, hipStream_t s) {
  const int64_t M = (int64_t)B * (D / 2) * (H / 2) * (W / 2);
  LoadPatch A{x, ldx, Cin, D, H, W, M};
  StoreRowsRes C{y, nullptr, N, 0, N, b, M};
  return launch_gemm(A, wf, C, M, head_fk(8 * Cin), head_fn(N), s);
}
// dx = dy W  (x [M][K] gradient; dy [M][N]); gelu_pre: dx *= gelu'(pre)
hipError_t linear_dgrad(const float* dy, int lddy, int N, const float* wd, float* dx, int lddx,
                        int K, int64_t M, const float* gelu_pre, hipStream_t s) {
  if (lddy % 4 == 0 && N % 4 == 0) {
    LoadRowsVec A{dy, lddy, N, M};
    if (gelu_pre) {
      StoreGeluBwd C{dx, gelu_pre, lddx, K, M};
      return launch_gemm(A, wd, C, M, head_dk(N), head_dn(K), s);
    }
    StoreRows C{dx, lddx, K, nullptr, M};
    return launch_gemm(A, wd, C, M, head_dk(N), head_dn(K), s);
  }
  LoadRowsScalar A{dy, lddy, N, M};
  if (gelu_pre) {
    StoreGeluBwd C{dx, gelu_pre, lddx, K, M};
    return launch_gemm(A, wd, C, M, head_dk(N), head_dn(K), s);
  }
  StoreRows C{dx, lddx, K, nullptr, M};
  return launch_gemm(A, wd, C, M, head_dk(N), head_dn(K), s);
}
// the same into a two-source gradient view, overwriting (acc = 0) or adding (acc = 1)
hipError_t linear_dgrad2(const float* dy, int lddy, int N, const float* wd, const Dst2& dx, int K,
                         int64_t M, int acc, hipStream_t s) {
  LoadRowsScalar A{dy, lddy, N, M};
  StoreDst2 C{dx, K, acc, M};
  return launch_gemm(A, wd, C, M, head_dk(N), head_dn(K), s);
}
size_t linear_wgrad_ws_bytes(int64_t M, int K, int N) {
  return std::max(xty_ws_bytes(M, K, N), atb_ws_bytes(M, K, N));
}
// dW [N][K] = dy^T x, db [N] = sum dy (db may be null: a scratch column is used)
hipError_t linear_wgrad(const float* x, int ldx, int K, const float* dy, int lddy, int N,
                        float* dw, float* db, int64_t M, float* ws, hipStream_t s) {
  return launch_xty(x, ldx, K, dy, lddy, N, nullptr, M, N, 1, dw, db, ws, s);
}
hipError_t linear_wgrad2(const Src2& x, int K, const float* dy, int lddy, int N, float* dw,
                         float* db, int64_t M, float* ws, hipStream_t s) {
  // streaming X^T Y with the two-source column split (the 64 x 64 LDS tiles of
  // k_atb measured 3-4x slower at K = 24, N = 12)
  return launch_xty(x.p0, x.ld0, K, dy, lddy, N, nullptr, M, N, 1, dw, db, ws, s, x.p1, x.ld1,
                    x.split);
}
hipError_t patch_embed_wgrad(const float* x, int ldx, int Cin, int D, int H, int W, int B,
                             const float* dy, int N, float* dw, float* db, float* ws,
                             hipStream_t s) {
  const int64_t M = (int64_t)B * (D / 2) * (H / 2) * (W / 2);
  LoadPatch X{x, ldx, Cin, D, H, W, M};
  LoadRowsScalar Y{dy, N, N, M};
  return launch_atb(X, Y, M, 8 * Cin, N, N, 1, dw, db, ws, s);
}

}  // namespace spff
