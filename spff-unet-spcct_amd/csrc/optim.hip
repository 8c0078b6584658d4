// Fused Adam / AdamW parameter step over a contiguous fp32 span.
//
// Replaces the optimizer the reference builds in BaseLitModel.configure_optimizers
// (models.py:591-594, torch.optim.Adam(lr=1e-4)) and unified_optimizer.py:5-60
// (Adam / AdamW): one HBM pass over (param, grad, exp_avg, exp_avg_sq) instead of
// the ~10 foreach passes of torch's multi-tensor path.  The per-element
// arithmetic is torch's (torch/optim/adam.py, _multi_tensor_adam,
// capturable=False) in its fp32 operation order, with FMA contraction off:
//   [AdamW] p *= 1 - lr*wd        [Adam, wd != 0] g = g + wd*p
//   m = lerp(m, g, 1 - b1)        v = v*b2 + (1 - b2)*g*g
//   p = p + (-lr / bc1) * (m / (sqrt(v) / sqrt(bc2) + eps))
// with bc1 = 1 - b1^t and bc2 = 1 - b2^t evaluated in double on the host.
#include "spff_internal.h"

#include <cmath>

namespace spff {

__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, float w1, float b2, float omb2, float wd,
                       int decoupled, float decay, float step_size, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], gg = g[i];
    if (decoupled) pp = pp * decay;
    else if (wd != 0.f) gg = gg + wd * pp;
    float mm = m[i];
    mm = w1 < 0.5f ? mm + w1 * (gg - mm) : gg - (gg - mm) * (1.f - w1);
    float vv = v[i] * b2;
    vv = vv + omb2 * gg * gg;
    const float s = sqrtf(vv) / bc2_sqrt + eps;
    pp = pp + step_size * (mm / s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

hipError_t adam_step(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                     double beta1, double beta2, double eps, double wd, int decoupled,
                     int64_t step, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float step_size = (float)((lr / bc1) * -1.0);
  const float bc2_sqrt = (float)std::pow(bc2, 0.5);
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, s, p, g, m, v, n, (float)(1.0 - beta1),
                     (float)beta2, (float)(1.0 - beta2), (float)wd, decoupled,
                     (float)(1.0 - lr * wd), step_size, bc2_sqrt, (float)eps);
  return hipGetLastError();
}

}  // namespace spff
