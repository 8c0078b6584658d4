// Height sharding of the registry layout [B, 1, 5, H, W] ("in the
// registry layout (D = 5), shard H instead, in multiples of 8 rows"): rank r owns
// global rows [r H_l, (r + 1) H_l) at level 0 (H_l a multiple of 8, so the three
// (1,2,2) pools and the up-convolutions stay rank-local).
//
// The 3x3x3 convolutions read their row halo IN PLACE: every activation keeps the dense
// [B][D][H][W][C] layout of the unsharded engine, and a conv's stencil rows h = -1 and
// h = H come from the neighbours' boundary rows, which the conv kernels read through
// Src2::rlo / rhi instead of the zero padding.  Per conv only those two rows move:
//
//   hrows_pack:  rows 0 and H - 1 of the conv input (the two-source [up | skip] view in
//                channel order, raw -- an input activation applies in the conv) into
//                send_lo / send_hi of the staging slab [recv_lo | send_lo | send_hi |
//                recv_hi] (B D W ldr floats each);
//   the caller's spff_coll.halo at d_local = 2 (the callback depth sharding uses) sends
//                send_lo to rank - 1, send_hi to rank + 1 and receives into recv_lo /
//                recv_hi; the global ends keep rlo / rhi = nullptr (zero padding).
//
// Round 2 copied every conv input into a row-padded volume and every output back
// (k_hpad / k_hunpad: ~4 (Cin + Cout) bytes per voxel per conv); this moves 2 / H_l of
// the input instead.
#include "spff_internal.h"

#include <algorithm>

namespace spff {

namespace {

// one thread per (boundary row voxel, 4-channel group): row 0 -> send_lo, row H-1 -> send_hi
__global__ __launch_bounds__(256) void k_hrows_pack(Src2 x, int cin, float* __restrict__ send,
                                                    int B, int D, int H, int W, int ldr) {
  const int q4 = ldr >> 2;
  const int64_t slice = (int64_t)B * D * W * q4;  // float4 per send slice
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 2 * slice;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool top = i >= slice;
    const int64_t j = top ? i - slice : i;
    const int c = (int)(j % q4) * 4;
    const int64_t vw = j / q4;  // (b D + d) W + w
    const int w = (int)(vw % W);
    const int64_t bd = vw / W;
    const int h = top ? H - 1 : 0;
    const int64_t vi = (bd * H + h) * W + w;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < cin) {
      v = c < x.split ? *reinterpret_cast<const float4*>(x.p0 + vi * x.ld0 + c)
                      : *reinterpret_cast<const float4*>(x.p1 + vi * x.ld1 + (c - x.split));
      if (c + 4 > cin) {  // zero the pad channels of a partial group
        if (c + 1 >= cin) v.y = 0.f;
        if (c + 2 >= cin) v.z = 0.f;
        if (c + 3 >= cin) v.w = 0.f;
      }
    }
    *reinterpret_cast<float4*>(send + (top ? slice * 4 : 0) + vw * ldr + c) = v;
  }
}

}  // namespace

int hrows_ld(int cin) { return (cin + 7) / 8 * 8; }
size_t hstage_floats(Vol v, int ldr) { return (size_t)4 * v.B * v.D * v.W * ldr; }

hipError_t hrows_pack(const Src2& x, int cin, float* send, Vol v, int ldr, hipStream_t s) {
  if (ldr % 4 || cin > ldr || x.ld0 % 4 || x.ld1 % 4 || (x.split < cin && x.split % 4))
    return hipErrorInvalidValue;
  const int64_t work = 2 * (int64_t)v.B * v.D * v.W * (ldr / 4);
  hipLaunchKernelGGL(k_hrows_pack, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 4096)),
                     dim3(256), 0, s, x, cin, send, v.B, v.D, v.H, v.W, ldr);
  return hipGetLastError();
}

}  // namespace spff
