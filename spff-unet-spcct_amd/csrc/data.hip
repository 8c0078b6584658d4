// Training data path on the device: the reference builds
// its volumes on the host -- per-frame TF.resize, a pure-Python ellipse-ROI
// rasterisation loop (helpers.py:125-211) -- and augments every sample in
// DataLoader worker processes (TrainGridAug, datasets.py:56-209).  Here the
// decoded volumes stay resident in HBM and the three steps are kernels:
//  * k_rasterize: label map of a frame from its ROI list, later ROIs winning,
//    with the reference's fp64 ellipse test;
//  * k_resize_aa_{w,h}: separable antialiased bilinear resize with PyTorch's
//    weights (F.interpolate(antialias=True), what TF.resize runs for tensors);
//  * the grid augmentation: flips, rot90 and the row/column stripe shuffle
//    compose into ONE source-index gather per output voxel (image and labels),
//    fused with the intensity jitter; then the optional gaussian noise (std from
//    a fixed-order fp64 reduction, counter-based normal draws) and the
//    top-left visibility stamp (max reductions).  The random decisions are
//    drawn on the host by the caller, in the reference's order (Python random),
//    and arrive as per-sample source maps and parameters.
// All HBM-bound gathers / streams; oracle: oracle/data_oracle.py.
#include "spff_internal.h"
#include "spff.h"

#include <math.h>

namespace spff {

namespace {
inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
}

// ------------------------------------------------------------ rasterise --
// rois [n][5] = (x0, y0, w0, h0, label); labels [F][H][W]
__global__ void k_rasterize(const int* __restrict__ rois, int nroi, int F, int H, int W,
                            int64_t* __restrict__ lab) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int px = (int)(i % W), py = (int)(i / W);
  int64_t l = 0;
  for (int r = 0; r < nroi; ++r) {
    const int x0 = rois[5 * r], y0 = rois[5 * r + 1], w0 = rois[5 * r + 2], h0 = rois[5 * r + 3];
    if (px < x0 || px >= x0 + w0 || py < y0 || py >= y0 + h0) continue;
    // helpers.py:125-129 in Python floats (IEEE double)
    const double cx = x0 + w0 / 2.0, cy = y0 + h0 / 2.0, a = w0 / 2.0, b = h0 / 2.0;
    const double dx = px - cx, dy = py - cy;
    if ((dx * dx) / (a * a) + (dy * dy) / (b * b) <= 1.0) l = rois[5 * r + 4];
  }
  for (int f = 0; f < F; ++f) lab[(int64_t)f * H * W + i] = l;
}

// ------------------------------------------------------- antialias resize --
// PyTorch _compute_weights_aa (bilinear, align_corners=False): scale = in/out,
// support = scale >= 1 ? scale : 1, center = scale (o + 0.5), taps
// [xmin, xmin + xsize), w = tri((j + xmin - center + 0.5) / max(scale, 1)), normalised.
__device__ __forceinline__ int aa_taps(int o, int in, float scale, float* w, int& xmin) {
  const float support = scale >= 1.f ? scale : 1.f;
  const float center = scale * (o + 0.5f);
  const float inv = scale >= 1.f ? 1.f / scale : 1.f;
  xmin = max((int)(center - support + 0.5f), 0);
  const int xsize = min((int)(center + support + 0.5f), in) - xmin;
  float tot = 0.f;
  for (int j = 0; j < xsize; ++j) {
    float x = (j + xmin - center + 0.5f) * inv;
    x = x < 0.f ? -x : x;
    w[j] = x < 1.f ? 1.f - x : 0.f;
    tot += w[j];
  }
  if (tot != 0.f)
    for (int j = 0; j < xsize; ++j) w[j] /= tot;
  return xsize;
}
constexpr int AA_MAXT = 64;  // taps: downscale factors up to ~31

// pass over W: in [n][h][win] -> out [n][h][wout]
__global__ void k_resize_aa_w(const float* __restrict__ in, int n, int h, int win, float* out,
                              int wout, float scale) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * h * wout) return;
  const int o = (int)(i % wout);
  const int64_t row = i / wout;
  float w[AA_MAXT];
  int xmin;
  const int xs = aa_taps(o, win, scale, w, xmin);
  const float* src = in + row * win + xmin;
  float s = 0.f;
  for (int j = 0; j < xs; ++j) s += src[j] * w[j];
  out[i] = s;
}
// pass over H: in [n][hin][w] -> out [n][hout][w]
__global__ void k_resize_aa_h(const float* __restrict__ in, int n, int hin, int w_, float* out,
                              int hout, float scale) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * hout * w_) return;
  const int x = (int)(i % w_);
  const int o = (int)((i / w_) % hout);
  const int64_t p = i / ((int64_t)w_ * hout);
  float w[AA_MAXT];
  int xmin;
  const int xs = aa_taps(o, hin, scale, w, xmin);
  const float* src = in + (p * hin + xmin) * w_ + x;
  float s = 0.f;
  for (int j = 0; j < xs; ++j) s += src[(int64_t)j * w_] * w[j];
  out[i] = s;
}

// ------------------------------------------------------ grid augmentation --
// prm[b][8] = {flip_w, flip_h, rot_k, jitter_on, scale, shift, noise_cap (0: off), stamp}
// maps[b][Ho + Wo] = source row (then column) in the rotated frame
constexpr int AUG_T = 256, AUG_NB = 256;  // blocks per sample for the reductions

__device__ __forceinline__ void aug_src(int ho, int wo, int H, int W, int rot, int fw, int fh,
                                        int& hi, int& wi) {
  // undo rot90(k, dims=(-2,-1)) of the H x W (flipped) frame
  int hf, wf;
  if (rot == 1) { hf = wo; wf = W - 1 - ho; }
  else if (rot == 2) { hf = H - 1 - ho; wf = W - 1 - wo; }
  else if (rot == 3) { hf = H - 1 - wo; wf = ho; }
  else { hf = ho; wf = wo; }
  if (fh) hf = H - 1 - hf;  // flip over H was applied after the flip over W
  if (fw) wf = W - 1 - wf;
  hi = hf;
  wi = wf;
}

// xo / yo gather + jitter; per-block fp64 [sum, sumsq] of xo for the noise std
__global__ __launch_bounds__(AUG_T) void k_aug_gather(const float* __restrict__ x,
                                                      const int64_t* __restrict__ y, int F, int H,
                                                      int W, const int* __restrict__ maps,
                                                      const float* __restrict__ prm,
                                                      float* __restrict__ xo,
                                                      int64_t* __restrict__ yo,
                                                      double* __restrict__ part) {
  const int b = blockIdx.y;
  const float* pp = prm + 8 * b;
  const int fw = pp[0] != 0.f, fh = pp[1] != 0.f, rot = (int)pp[2], jit = pp[3] != 0.f;
  const float sc = pp[4], sh = pp[5];
  const int Ho = rot & 1 ? W : H, Wo = rot & 1 ? H : W;
  const int* rs = maps + (int64_t)b * (H + W);
  const int* cs = rs + Ho;
  const int64_t n = (int64_t)F * H * W;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)AUG_T + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * AUG_T) {
    const int wo = (int)(i % Wo);
    const int ho = (int)((i / Wo) % Ho);
    const int f = (int)(i / ((int64_t)Wo * Ho));
    int hi, wi;
    aug_src(rs[ho], cs[wo], H, W, rot, fw, fh, hi, wi);
    const int64_t src = ((int64_t)f * H + hi) * W + wi;
    float v = x[(int64_t)b * n + src];
    if (jit) {
      // x * scale + shift with two fp32 roundings, as torch's two eager ops (no FMA)
#pragma clang fp contract(off)
      v = v * sc + sh;
    }
    xo[(int64_t)b * n + i] = v;
    if (y) yo[(int64_t)b * n + i] = y[(int64_t)b * n + src];
    s1 += v;
    s2 += (double)v * v;
  }
  __shared__ double r1[AUG_T], r2[AUG_T];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int st = AUG_T / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      r1[threadIdx.x] += r1[threadIdx.x + st];
      r2[threadIdx.x] += r2[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 0] = r1[0];
    part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = r2[0];
  }
}

// std[b] = noise std (0: no noise) = min(cap, 0.25 * x.std()) if x.std() > 0
__global__ void k_aug_std(const double* __restrict__ part, int nblk, int64_t n,
                          const float* __restrict__ prm, int B, float* __restrict__ stdv) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < nblk; ++k) {
    s1 += part[((int64_t)b * nblk + k) * 2];
    s2 += part[((int64_t)b * nblk + k) * 2 + 1];
  }
  const float cap = prm[8 * b + 6];
  float sd = 0.f;
  if (cap > 0.f && n > 1) {
    const double var = (s2 - s1 * s1 / (double)n) / (double)(n - 1);
    const double v = var > 0.0 ? sqrt(var) : 0.0;  // torch.std: unbiased
    if (v > 0.0) sd = (float)fmin((double)cap, 0.25 * v);
  }
  stdv[b] = sd;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// noise (counter-based normal draws at each output index) + per-block max|x| and
// the max of frame 0's top-left 32 x 32 (the stamp's inputs)
__global__ __launch_bounds__(AUG_T) void k_aug_noise(float* __restrict__ xo, int F, int H, int W,
                                                     const float* __restrict__ prm,
                                                     const float* __restrict__ stdv,
                                                     uint64_t seed, float* __restrict__ mpart) {
  const int b = blockIdx.y;
  const int rot = (int)prm[8 * b + 2], Ho = rot & 1 ? W : H, Wo = rot & 1 ? H : W;
  const int64_t n = (int64_t)F * Ho * Wo;
  const float sd = stdv[b];
  float am = 0.f, rm = -INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)AUG_T + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * AUG_T) {
    float v = xo[(int64_t)b * n + i];
    if (sd > 0.f) {
      const uint64_t r = mix64(seed ^ mix64(((uint64_t)b << 40) + (uint64_t)i));
      const double u1 = ((r >> 11) + 1) * (1.0 / 9007199254740993.0);  // (0, 1]
      const double u2 = (mix64(r) >> 11) * (1.0 / 9007199254740992.0);
      const float z = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
      v = v + z * sd;
      xo[(int64_t)b * n + i] = v;
    }
    am = fmaxf(am, fabsf(v));
    const int wo = (int)(i % Wo), ho = (int)((i / Wo) % Ho);
    if (i < (int64_t)Ho * Wo && ho < 32 && wo < 32) rm = fmaxf(rm, v);
  }
  __shared__ float ra[AUG_T], rr[AUG_T];
  ra[threadIdx.x] = am;
  rr[threadIdx.x] = rm;
  __syncthreads();
  for (int st = AUG_T / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      ra[threadIdx.x] = fmaxf(ra[threadIdx.x], ra[threadIdx.x + st]);
      rr[threadIdx.x] = fmaxf(rr[threadIdx.x], rr[threadIdx.x + st]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    mpart[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 0] = ra[0];
    mpart[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = rr[0];
  }
}

// x[0, 0, :32, :32] = its max + max(|x|).clamp(min=1) * 0.25 (datasets.py:200-205)
__global__ void k_aug_stamp(float* __restrict__ xo, int F, int H, int W,
                            const float* __restrict__ prm, const float* __restrict__ mpart,
                            int nblk) {
  const int b = blockIdx.x;
  if (prm[8 * b + 7] == 0.f) return;
  const int rot = (int)prm[8 * b + 2], Ho = rot & 1 ? W : H, Wo = rot & 1 ? H : W;
  __shared__ float val;
  if (threadIdx.x == 0) {
    float am = 0.f, rm = -INFINITY;
    for (int k = 0; k < nblk; ++k) {
      am = fmaxf(am, mpart[((int64_t)b * nblk + k) * 2]);
      rm = fmaxf(rm, mpart[((int64_t)b * nblk + k) * 2 + 1]);
    }
    {
#pragma clang fp contract(off)
      val = rm + fmaxf(am, 1.f) * 0.25f;
    }
  }
  __syncthreads();
  const int hh = min(Ho, 32), ww = min(Wo, 32);
  for (int i = threadIdx.x; i < hh * ww; i += blockDim.x)
    xo[(int64_t)b * F * Ho * Wo + (int64_t)(i / ww) * Wo + i % ww] = val;
}

}  // namespace spff

using namespace spff;

extern "C" {

int spff_rasterize_ellipses(const int* rois, int nroi, int frames, int height, int width,
                            int64_t* labels, void* stream) {
  if ((!rois && nroi) || !labels || frames < 1 || height < 1 || width < 1)
    return set_error(SPFF_EINVAL, "spff_rasterize_ellipses: bad argument");
  const int64_t n = (int64_t)height * width;
  hipLaunchKernelGGL(k_rasterize, dim3((unsigned)cdiv64(n, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), rois, nroi, frames, height, width, labels);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SPFF_OK : set_error(SPFF_EHIP, hipGetErrorString(e));
}

int spff_resize_bilinear_aa(const float* in, int n, int hin, int win, float* out, int hout,
                            int wout, float* tmp, void* stream) {
  if (!in || !out || !tmp || n < 1 || hin < 1 || win < 1 || hout < 1 || wout < 1)
    return set_error(SPFF_EINVAL, "spff_resize_bilinear_aa: bad argument");
  const float sw = (float)win / (float)wout, sh = (float)hin / (float)hout;
  if (2 * ceilf(fmaxf(sw, 1.f)) + 2 > AA_MAXT || 2 * ceilf(fmaxf(sh, 1.f)) + 2 > AA_MAXT)
    return set_error(SPFF_EINVAL, "spff_resize_bilinear_aa: downscale factor too large");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n1 = (int64_t)n * hin * wout, n2 = (int64_t)n * hout * wout;
  hipLaunchKernelGGL(k_resize_aa_w, dim3((unsigned)cdiv64(n1, 256)), dim3(256), 0, s, in, n, hin,
                     win, tmp, wout, sw);
  hipLaunchKernelGGL(k_resize_aa_h, dim3((unsigned)cdiv64(n2, 256)), dim3(256), 0, s, tmp, n, hin,
                     wout, out, hout, sh);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SPFF_OK : set_error(SPFF_EHIP, hipGetErrorString(e));
}

size_t spff_grid_aug_ws_bytes(int batch) {
  return (size_t)batch * AUG_NB * 2 * (sizeof(double) + sizeof(float)) + (size_t)batch * 4 + 256;
}

int spff_grid_aug(const float* x, const int64_t* y, int batch, int frames, int height, int width,
                  const int* maps, const float* prm, uint64_t seed, float* xo, int64_t* yo,
                  void* ws, void* stream) {
  if (!x || !maps || !prm || !xo || !ws || (y && !yo) || batch < 1 || frames < 1 || height < 1 ||
      width < 1)
    return set_error(SPFF_EINVAL, "spff_grid_aug: bad argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(ws);
  float* mpart = reinterpret_cast<float*>(part + (size_t)batch * AUG_NB * 2);
  float* stdv = mpart + (size_t)batch * AUG_NB * 2;
  const dim3 grid(AUG_NB, batch);
  hipLaunchKernelGGL(k_aug_gather, grid, dim3(AUG_T), 0, s, x, y, frames, height, width, maps, prm,
                     xo, yo, part);
  const int64_t n = (int64_t)frames * height * width;
  hipLaunchKernelGGL(k_aug_std, dim3((batch + 63) / 64), dim3(64), 0, s, part, AUG_NB, n, prm,
                     batch, stdv);
  // each sample's output frame is Ho x Wo (W x H after an odd rot90)
  hipLaunchKernelGGL(k_aug_noise, grid, dim3(AUG_T), 0, s, xo, frames, height, width, prm, stdv,
                     seed, mpart);
  hipLaunchKernelGGL(k_aug_stamp, dim3(batch), dim3(256), 0, s, xo, frames, height, width, prm,
                     mpart, AUG_NB);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SPFF_OK : set_error(SPFF_EHIP, hipGetErrorString(e));
}

}  // extern "C"
