// Internal declarations shared by the SPFF HIP translation units.
// Layout convention everywhere: activations are channel-last [B][D][H][W][C]
// fp32 ("NDHWC"), voxel index v = ((b*D + d)*H + h)*W + w.
#pragma once
#include <hip/hip_runtime.h>
#include "spff.h"
#include <stdint.h>
#include <stddef.h>

namespace spff {

// records msg for spff_last_error() (calling thread) and returns code
int set_error(int code, const char* msg);

// Two-source channel view: channel c < split reads p0[v*ld0 + c], otherwise
// p1[v*ld1 + c - split].  Lets the decoder's first conv read [up | skip]
// without materialising torch.cat (reference _cat, models.py:687-691).
struct Src2 {
  const float* p0; const float* p1; int ld0, ld1, split;
  // Optional input activation of source 0, applied as the conv loads it:
  // lrelu(x * al[b*ld0 + c] + de[b*ld0 + c], 0.01).  A block's second conv reads its
  // first conv's raw output y1 through the InstanceNorm affine this way, so
  // a1 = lrelu(IN(y1)) is never written to HBM (split-bf16 conv kernels only).
  const float* al = nullptr;
  const float* de = nullptr;
  int zlo = 0, zhi = 0;  // depth-sharded: the d = -1 / d = D halo slice is zero padding
  // height-sharded: the neighbours' boundary rows h = -1 / h = H, [B][D][W][ldr] with the
  // conv's input channels in order (both sources), read by the conv kernels in place of
  // the zero padding (nullptr at a global end: zero).  Raw values: the input activation
  // (al / de) applies to them as to the local rows.
  const float* rlo = nullptr;
  const float* rhi = nullptr;
  int ldr = 0;
  __host__ __device__ bool rows() const { return rlo != nullptr || rhi != nullptr; }
};
struct Dst2 {
  float* p0; float* p1; int ld0, ld1, split;
};
inline Src2 src1(const float* p, int ld) { return Src2{p, p, ld, ld, 1 << 30}; }
inline Dst2 dst1(float* p, int ld) { return Dst2{p, p, ld, ld, 1 << 30}; }

// dh = 1: a depth-sharded plan's conv inputs carry one neighbour slice before
// and after the interior (B = 1), and the conv kernels read d = -1 and d = D
// from them instead of treating those as zero padding.
struct Vol {
  int B, D, H, W;
  int dh = 0;
};
inline int64_t nvox(const Vol& v) { return (int64_t)v.B * v.D * v.H * v.W; }

// address of channels [c, c + 4) of the conv input at (b, gd, gh, gw), or nullptr where
// the stencil reads zero padding: outside the volume, except the depth halo slices of a
// depth-sharded input (vol.dh, Src2::zlo / zhi) and the boundary rows of a height-sharded
// one (Src2::rlo / rhi).  No input activation (the split-bf16 kernels apply al / de).
__device__ __forceinline__ const float* src_at(const Src2& x, const Vol& vol, int b, int gd,
                                               int gh, int gw, int c) {
  const int D = vol.D, H = vol.H, W = vol.W;
  if ((unsigned)(gd + vol.dh) >= (unsigned)(D + 2 * vol.dh) || (unsigned)gw >= (unsigned)W ||
      (gd < 0 && x.zlo) || (gd >= D && x.zhi))
    return nullptr;
  if ((unsigned)gh >= (unsigned)H) {
    const float* r = gh < 0 ? (gh == -1 ? x.rlo : nullptr) : (gh == H ? x.rhi : nullptr);
    return r ? r + (((int64_t)b * D + gd) * W + gw) * x.ldr + c : nullptr;
  }
  const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
  return c < x.split ? x.p0 + vox * x.ld0 + c : x.p1 + vox * x.ld1 + (c - x.split);
}

// SPFF_MATH_F16X3 operand maxima: the block's largest m (>= 0) into *slot as an integer
// atomicMax of its float bits (non-negative floats order like their bits; order-independent,
// so deterministic).  Every thread of the block must call it (it synchronises the block).
__device__ __forceinline__ void block_amax(float m, unsigned* slot) {
  __shared__ float wm[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)((blockDim.x + 63) >> 6); ++w) m = fmaxf(m, wm[w]);
    if (m > 0.f) atomicMax(slot, __float_as_uint(m));
  }
}

// ---------------------------------------------------------------- conv3d --
// Weight repack: reference layout W[Cout][Cin][KD][3][3] ->
//   fwd:   Wt[tap][ci(pad cin_pad)][co(pad cout_pad)]
//   dgrad: Wt[tap][co(pad cout_pad)][ci(pad cin_pad)] with taps flipped.
hipError_t conv_pack_weights(const float* w, float* wt, int Cout, int Cin, int KD,
                             int kpad, int npad, bool dgrad, hipStream_t s);
// y = conv3d(x, W) 'same' padding (KD/2,1,1); x: Cin channels (kpad: padded
// reduction channels, multiple of 8), y: Cout channels (npad: multiple of BN).
hipError_t conv3d_fwd(const Src2& x, const float* wt, const Dst2& y, Vol vol, int KD,
                      int Cin, int kpad, int Cout, int npad, hipStream_t s);
int conv3d_bn(int Cout);        // output-channel tile the fwd kernel uses
// Layer-level conv (conv3d_x.hip): pack W[Cout_w][Cin_w][KD][3][3] for the
// forward (dgrad = false: x has Cin_w channels, y Cout_w) or the input gradient
// (dgrad = true: x = dy with Cout_w channels, y = dx with Cin_w) in the layout
// the chosen arithmetic (SPFF_MATH_*) runs on, then run it.  Volumes smaller
// than one 16 x 16 H/W tile take the fp32 kernel whatever the math.
size_t conv3d_pack_bytes(int KD, int Cin_w, int Cout_w);
// (SPFF_MATH_F16X3: wmax = a precomputed max |w| slot, else computed into the image's tail)
hipError_t conv3d_pack(const float* w, void* wpack, Vol vol, int KD, int Cin_w, int Cout_w,
                       bool dgrad, int math, hipStream_t s, const unsigned* wmax = nullptr);
// A plan's weight preparation as one launch pair at the forward start, instead of one
// max + one pack launch per conv: PrepJobs (max |w| of each weight tensor, the a1 bounds
// act_bound computes) then PackJobs (every conv image, fwd and dgrad).  The tables travel
// as kernel arguments.  conv3d_packs_batched: the math packs split images (else
// conv3d_pack per conv).
struct PrepJob {
  const float* a;     // absmax: the tensor; act_bound: gamma
  const float* b;     // act_bound: beta
  unsigned* slot;     // zeroed by the caller (absmax: atomicMax; act_bound: stored)
  int64_t n;          // absmax: elements; act_bound: channels
  float sq;           // act_bound: sqrt(max(N - 1, 1))
  int kind, blk0, nblk;  // kind 0 absmax, 1 act_bound
};
struct PrepJobs {
  int n = 0, nblk = 0;
  PrepJob j[32];
};
struct PackJob {
  const float* w;
  uint4* wp;
  const unsigned* wmx;  // SPFF_MATH_F16X3: the filled max |w| slot
  int Cout, Cin, T, T2, nkc, npad, BN, dgrad, blk0, nblk;
};
struct PackJobs {
  int n = 0, nblk = 0;
  PackJob j[40];  // 2568 B of kernel argument
};
bool conv3d_packs_batched(int math);
bool prep_absmax(PrepJobs* J, const float* p, int64_t n, unsigned* slot);
bool prep_act_bound(PrepJobs* J, const float* gamma, const float* beta, int C, double N,
                    unsigned* slot);
hipError_t prep_run(const PrepJobs& J, hipStream_t s);
bool conv3d_pack_job(PackJobs* J, const float* w, void* wpack, int KD, int Cin_w, int Cout_w,
                     bool dgrad, const unsigned* wmax);
hipError_t conv3d_pack_many(const PackJobs& J, int math, hipStream_t s);
// ws (optional, >= conv3d_splitk_bytes): scratch for split-K partial sums on
// launches that would not fill the chip; null = no split
// stats (optional, forward only, when conv3d_fuses_stats): the conv's epilogue also
// writes per-tile InstanceNorm partials (>= conv3d_stats_bytes) that
// conv3d_in_stats_fin turns into mean / rstd / al / de, replacing the two
// slab_reduce passes of the unfused path.
// dpart (depth-sharded halo overlap, when conv3d_splits_depth): 1 = only the interior
// depth tiles, whose 3x3x3 stencil reads no halo slice; 2 = only the first and last
// depth tiles; 0 = all.  1 and 2 together write exactly what 0 writes.  3 / 4: the same
// for the H tiles of a height-sharded conv (conv3d_splits_height: interior tiles read no
// boundary row; 3 and 4 together write what 0 writes).
// bst (optional, input gradient only, when conv3d_fuses_bwd_stats): the output dx is the
// gradient entering an InstanceNorm + LeakyReLU whose input was bst.y; the epilogue also
// writes per-(tile, channel) partials of sum dr and sum dr xhat (dr = dx slope(y al + de),
// xhat = (y - mean) rstd -- RED_BWD_IN's sums) that conv3d_in_bwd_stats_fin turns into the
// IN backward's k1, k2, dgamma, dbeta, replacing that slab_reduce pass
struct BStat {
  const float* y = nullptr;     // [V][ld], the layout of the conv output
  const float* al = nullptr;    // [B][ld]
  const float* de = nullptr;
  const float* mean = nullptr;
  const float* rstd = nullptr;
  float* out = nullptr;         // >= conv3d_stats_bytes(vol, KD, Cin_w, Cout_w)
  int ld = 0;
  float neg = 0.01f;
};
hipError_t conv3d_run(const Src2& x, const void* wpack, const Dst2& y, Vol vol, int KD,
                      int Cin_w, int Cout_w, bool dgrad, int math, hipStream_t s,
                      float* ws = nullptr, float* stats = nullptr, int dpart = 0,
                      const unsigned* wmax = nullptr, const BStat* bst = nullptr);
bool conv3d_fuses_bwd_stats(Vol vol, int KD, int Cin_w, int Cout_w, int math);
hipError_t conv3d_in_bwd_stats_fin(const float* part, Vol vol, int KD, int Cin_w, int Cout_w,
                                   int math, float* dgamma, float* dbeta, float* k1, float* k2,
                                   hipStream_t s);
bool conv3d_splits_depth(Vol vol, int KD, int Cin_w, int Cout_w, bool dgrad, int math);
bool conv3d_splits_height(Vol vol, int KD, int Cin_w, int Cout_w, bool dgrad, int math);
bool conv3d_fuses_stats(Vol vol, int KD, int Cin, int Cout, int math);
size_t conv3d_stats_bytes(Vol vol, int KD, int Cin, int Cout);
hipError_t conv3d_in_stats_fin(const float* stats, Vol vol, int KD, int Cin, int Cout, int math,
                               const float* gamma, const float* beta, float* mean, float* rstd,
                               float* al, float* de, hipStream_t s);
size_t conv3d_splitk_bytes(Vol vol, int KD, int Cin_w, int Cout_w);
// dW partials + reduction into reference layout dw[Cout][Cin][KD][3][3].
// math = SPFF_MATH_F32: fp32 MFMA kernel (conv3d.hip); otherwise the split-bf16
// kernel of conv3d_wgx.hip.  ws >= conv3d_wgrad_ws_bytes (covers both).
size_t conv3d_wgrad_ws_bytes(Vol vol, int KD, int Cin, int Cout);
// (SPFF_MATH_F16X3: xmax / ymax = precomputed max |x| / |dy| slots, else computed here)
hipError_t conv3d_wgrad(const Src2& x, const float* dy, int lddy, float* dw, Vol vol, int KD,
                        int Cin, int Cout, int math, float* ws, hipStream_t s,
                        const unsigned* xmax = nullptr, const unsigned* ymax = nullptr);
size_t conv3d_wgrad_x_ws_bytes(Vol vol, int KD, int Cin, int Cout);
bool debug_split_wgrad();  // SPFF_DEBUG_SPLIT (conv3d_x.hip)
// Library-wide conv timing (spff_conv_prof_*, conv3d_x.hip): when on, conv3d_run and
// conv3d_wgrad bracket their launches with HIP events on the stream they run on, whichever
// plan (SPFF, 3DUNet, SwinUNETR) or the op-level ABI calls them.  Classes: 0 fwd,
// 1 dgrad, 2 wgrad; flops = 2 V Cin Cout T (algorithmic, fp32).
struct CProf {
  int rec = -1;
  CProf(int cls, double flops, hipStream_t s);
  void end(hipStream_t s);
};
void conv_prof_enable(bool on);
hipError_t conv_prof_collect(double* out, int nclass);
// the split-bf16 fwd and wgrad kernels apply Src2::al / de to a C-channel conv input of
// a C -> C conv (conv3d_x.hip: the 32-wide tiles, so C == 32)
bool conv3d_fuses_act(int math, int C);
hipError_t conv3d_wgrad_x(const Src2& x, const float* dy, int lddy, float* dw, Vol vol, int KD,
                          int Cin, int Cout, int math, float* ws, hipStream_t s,
                          const unsigned* xmax = nullptr, const unsigned* ymax = nullptr);
// SPFF_MATH_F16X3 operand scales (conv3d_x.hip): atomicMax of the largest |element| (float
// bits) into *slot, which the caller zeroed.  absmax_src covers what a conv reads of x:
// C channels with the input activation applied, plus (halo) a depth-sharded input's halo
// slices and a height-sharded one's boundary rows; channel strides must be multiples of 4.
// (also: a slot whose value is max-ed into *slot too, after the caller's stream order)
hipError_t absmax_src(const Src2& x, Vol vol, int C, bool halo, unsigned* slot, hipStream_t s,
                      const unsigned* also = nullptr);
hipError_t absmax_f32(const float* p, int64_t n, unsigned* slot, hipStream_t s);
// fixed-order sum of the [nsplit][T][kpad][npad] partial slabs into dw[Cout][Cin][T]
hipError_t conv3d_wgrad_reduce(const float* part, float* dw, int nsplit, int T, int kpad,
                               int npad, int Cin, int Cout, hipStream_t s);

// ---------------------------------------------------------------- gemms --
// A block output applied as a GEMM reads it (the decoders' and the bottleneck's outputs
// feed only the up-convs and the head): row v = lrelu(y[v] al[b] + de[b], neg) P[b,d] + Q[b,d]
// (k_act_apply's formula, bitwise), y [V][C] channel-last, al / de [B][C], PT / QT the
// gate coefficients transposed to [B][D][C] (null: P = 1, Q = 0).  The row's (b, d) is
// v / HW = b D + d.
struct ActRows {
  const float* y = nullptr;
  const float* al = nullptr;
  const float* de = nullptr;
  const float* PT = nullptr;
  const float* QT = nullptr;
  int D = 1, HW = 1;
  float neg = 0.01f;
};
// ConvTranspose3d(Cin->Cout, k=s=(1,2,2) [ns = 4] or 2x2x2 [ns = 8]) + bias,
// low-res x [Vlow][Cin], high-res y [Vhigh][Cout] (H, W doubled; D too for
// ns = 8).  Reference weight W[Cin][Cout][1 or 2][2][2].
hipError_t upconv_pack(const float* w, float* wf, float* wd, int Cin, int Cout, hipStream_t s,
                       int ns = 4);
// (math = SPFF_MATH_BF16X6: the split-bf16 MFMA GEMM; otherwise the fp32 MFMA one)
// (act: x = the rows ActRows describes, applied as they load; the x argument is ignored)
// (amax: also the largest |y| into *amax, max-ed with *also -- an f16x3 operand scale)
hipError_t upconv_fwd(const float* x, const float* wf, const float* bias, float* y,
                      Vol low, int Cin, int Cout, hipStream_t s, int ns = 4,
                      int math = SPFF_MATH_F32, const ActRows* act = nullptr,
                      unsigned* amax = nullptr, const unsigned* also = nullptr);
hipError_t upconv_dgrad(const float* dy, int lddy, const float* wd, float* dx, Vol low,
                        int Cin, int Cout, hipStream_t s, int ns = 4, int math = SPFF_MATH_F32);
size_t upconv_wgrad_ws_bytes(Vol low, int Cin, int Cout, int ns = 4);
hipError_t upconv_wgrad(const float* x, const float* dy, int lddy, float* dw, float* db,
                        Vol low, int Cin, int Cout, float* ws, hipStream_t s, int ns = 4,
                        int math = SPFF_MATH_F32, const ActRows* act = nullptr);
size_t upconv_pack_floats(int Cin, int Cout, int ns = 4);
size_t upconv_pack_dgrad_offset(int Cin, int Cout, int ns = 4);
// 1x1x1 conv head: y[v][K] = x[v][:Cin] . W[K][Cin] + b  (wf/wd from head_pack)
hipError_t head_pack(const float* w, float* wf, float* wd, int Cin, int K, hipStream_t s);
size_t head_pack_floats(int Cin, int K);
size_t head_pack_dgrad_offset(int Cin, int K);
hipError_t head_fwd(const float* x, const float* wf, const float* b, float* y, int64_t V,
                    int Cin, int K, hipStream_t s, int math = SPFF_MATH_F32,
                    const ActRows* act = nullptr);
hipError_t head_dgrad(const float* dy, const float* wd, float* dx, int64_t V, int Cin, int K,
                      hipStream_t s, int math = SPFF_MATH_F32);
size_t head_wgrad_ws_bytes(int64_t V, int Cin, int K);
hipError_t head_wgrad(const float* x, const float* dy, float* dw, float* db, int64_t V,
                      int Cin, int K, float* ws, hipStream_t s, const ActRows* act = nullptr);

// nn.Linear / 1x1x1 Conv3d on channel-last rows (SwinUNETR path): W [N][K] packed by
// head_pack(w, wf, wd, K, N) (wf = W^T for the forward, wd = W for dgrad).
// y = res + x W^T + b (res, b optional); ld* = row pitches in floats.
hipError_t linear_fwd(const float* x, int ldx, int K, const float* wf, const float* b, float* y,
                      int ldy, int N, int64_t M, const float* res, int ldres, hipStream_t s);
hipError_t linear_fwd2(const Src2& x, int K, const float* wf, const float* b, float* y, int ldy,
                       int N, int64_t M, hipStream_t s);
// pre = x W^T + b, act = gelu(pre) (erf form, nn.GELU default)
hipError_t linear_fwd_gelu(const float* x, int ldx, int K, const float* wf, const float* b,
                           float* pre, float* act, int N, int64_t M, hipStream_t s);
// Conv3d(Cin, N, kernel = stride = 2) + bias of a channel-last [B][D][H][W][ldx] input
hipError_t patch_embed_fwd(const float* x, int ldx, int Cin, int D, int H, int W, int B,
                           const float* wf, const float* b, float* y, int N, hipStream_t s);
// dx = dy W (gelu_pre: times gelu'(pre))
hipError_t linear_dgrad(const float* dy, int lddy, int N, const float* wd, float* dx, int lddx,
                        int K, int64_t M, const float* gelu_pre, hipStream_t s);
hipError_t linear_dgrad2(const float* dy, int lddy, int N, const float* wd, const Dst2& dx, int K,
                         int64_t M, int acc, hipStream_t s);
size_t linear_wgrad_ws_bytes(int64_t M, int K, int N);
// dW [N][K] = dy^T x, db [N] = column sums of dy (db must be valid memory)
hipError_t linear_wgrad(const float* x, int ldx, int K, const float* dy, int lddy, int N,
                        float* dw, float* db, int64_t M, float* ws, hipStream_t s);
hipError_t linear_wgrad2(const Src2& x, int K, const float* dy, int lddy, int N, float* dw,
                         float* db, int64_t M, float* ws, hipStream_t s);
hipError_t patch_embed_wgrad(const float* x, int ldx, int Cin, int D, int H, int W, int B,
                             const float* dy, int N, float* dw, float* db, float* ws,
                             hipStream_t s);

// ------------------------------------------------------------- norm/gates --
// Per-(b,d,c) reductions over (h,w) with per-(b,c) affine/recompute ops.
enum RedOp {
  RED_SUM = 0,        // q0 = y
  RED_SQDEV = 1,      // q0 = (y - mean[b,c])^2            (aux0 = mean)
  RED_ACT = 2,        // q0 = lrelu(y*al + de)              (aux0 = alpha, aux1 = delta)
  RED_BWD_TAIL = 3,   // q0 = g, q1 = g*lrelu(y*al+de)      (g = dout)
  RED_BWD_IN = 4,     // r = y*al+de; dr = (g*A+Bc)*slope(r); q0 = dr, q1 = dr*xhat
  // RED_BWD_TAIL and the gated block's RED_BWD_IN in one pass: dr = (g A + Bc) s with
  // A, Bc per (b,c,d), so its sums factor as A S(g s) + Bc S(s) and A S(g s xhat) +
  // Bc S(s xhat).  out = [q0 g, q1 g*a]; out2 = [S(g s), S(s), S(g s xhat), S(s xhat)]
  // (s = slope(r)); in_sums_from_tail() turns out2 into RED_BWD_IN's [B][C][D][2]
  RED_BWD_TAIL6 = 5,
};
// An encoder block's output gradient formed where it is read: g (the skip gradient) plus
// the MaxPool3d(1,2,2) backward of the pooled gradient dp [B][D][H/2][W/2][C] routed by the
// argmax bytes idx (same layout) -- k_maxpool_bwd_add's sum, in its order, folded into its
// two consumers (the tail reduction and the IN-backward apply) instead of a pass of its own
struct PoolAdd {
  const float* dp = nullptr;
  const uint8_t* idx = nullptr;
};
struct RedArgs {
  const float* y; const float* g;     // y: [V][C] (ld = C), g: [V][C] (ld = C)
  const float* mean; const float* rstd; // [B][C]
  const float* al; const float* de;   // [B][C]
  const float* A; const float* Bc;    // [B][C][D] or null (identity)
  float neg = 0.01f;                  // activation negative slope (0: ReLU)
  PoolAdd pa;                         // g += unpool(pa) (two-operand ops only)
};
// out: [B][C][D][nq] fp32, summed over h,w in a fixed order.
size_t slab_reduce_ws_bytes(Vol vol, int C, int nq);
hipError_t slab_reduce(RedOp op, const RedArgs& a, Vol vol, int C, float* out, float* ws,
                       hipStream_t s, float* out2 = nullptr);
// out[i] = {A t4[i][0] + Bc t4[i][1], A t4[i][2] + Bc t4[i][3]} for the n = B C D slabs
hipError_t in_sums_from_tail(const float* t4, const float* A, const float* Bc, float* out,
                             int64_t n, hipStream_t s);
// stats: from per-(b,c,d) sums -> mean[b,c] ; from sqdev sums -> rstd, alpha, delta
hipError_t in_mean(const float* sums, float* mean, Vol vol, int C, hipStream_t s);
hipError_t in_rstd(const float* sqsums, const float* gamma, const float* beta,
                   const float* mean, float* rstd, float* al, float* de, Vol vol, int C,
                   hipStream_t s);
// out = lrelu(y*al[b,c]+de[b,c]) * P[b,c,d] + Q[b,c,d]   (P/Q null -> identity)
// (amax: also block_amax the largest |out| into *amax -- an f16x3 operand scale)
hipError_t act_apply(const float* y, float* out, const float* al, const float* de,
                     const float* P, const float* Q, Vol vol, int C, hipStream_t s,
                     float neg = 0.01f, unsigned* amax = nullptr);
// act_apply of an encoder block output fused with the (1,2,2) max-pool that reads it:
// out as act_apply, pooled [B][D][H/2][W/2][C] and its argmax bytes as maxpool_fwd (H, W even)
hipError_t act_apply_pool(const float* y, float* out, const float* al, const float* de,
                          const float* P, const float* Q, float* pooled, uint8_t* idx, Vol vol,
                          int C, hipStream_t s, float neg = 0.01f, unsigned* amax = nullptr);
// IN backward finalize: from per-(b,c,d) [sum dr, sum dr*xhat] -> dgamma, dbeta (over b),
// k1[b,c] = mean dr, k2[b,c] = mean dr*xhat
// depth-sharded variants: fp64 partials over the local slab, summed across the
// shard group by the caller, finalised with the global voxel count N
hipError_t in_partial(const float* sums, double* part, Vol vol, int C, int nq, hipStream_t s);
hipError_t in_mean_fin(const double* part, float* mean, int BC, double N, hipStream_t s);
hipError_t in_rstd_fin(const double* part, const float* gamma, const float* beta,
                       const float* mean, float* rstd, float* al, float* de, int B, int C,
                       double N, hipStream_t s);
hipError_t in_bwd_dgb(const double* part, float* dgamma, float* dbeta, int B, int C,
                      hipStream_t s);
hipError_t in_bwd_fin(const double* part, float* k1, float* k2, int BC, double N, hipStream_t s);
hipError_t in_bwd_stats(const float* sums, const float* gamma, float* dgamma, float* dbeta,
                        float* k1, float* k2, Vol vol, int C, hipStream_t s);
// dy = rstd*gamma*(dr - k1 - xhat*k2), dr = (g*A+Bc)*slope(y*al+de) ; may alias g
hipError_t in_bwd_apply(const float* y, const float* g, float* dy, const float* mean,
                        const float* rstd, const float* al, const float* de, const float* gamma,
                        const float* A, const float* Bc, const float* k1, const float* k2,
                        Vol vol, int C, hipStream_t s, float neg = 0.01f,
                        unsigned* amax = nullptr, PoolAdd pa = {});
// (amax: also atomicMax the largest |dy| (float bits) into *amax -- an SPFF_MATH_F16X3 operand
// scale for the convs that read dy; the caller zeroed it)
// a bound on max |lrelu(IN(y))| from the parameters alone, into *slot (float bits): per
// instance |xhat| <= sqrt(N - 1) (N = instance voxel count, population variance), so
// |lrelu(gamma xhat + beta)| <= max_c |gamma_c| sqrt(N - 1) + max_c |beta_c| (x 2 for rounding)
hipError_t act_bound(const float* gamma, const float* beta, int C, double N, unsigned* slot,
                     hipStream_t s);
// BatchNorm3d (train: batch statistics over (b,d,h,w) + running-stat update;
// eval: running statistics).  Per-channel values replicated over b into [B][C].
hipError_t bn_mean(const float* sums, float* mean, Vol vol, int C, hipStream_t s);
hipError_t bn_rstd(const float* sqsums, const float* gamma, const float* beta, const float* mean,
                   float* rstd, float* al, float* de, float* rmean, float* rvar, double mom,
                   double eps, Vol vol, int C, hipStream_t s);
hipError_t bn_eval(const float* rmean, const float* rvar, const float* gamma, const float* beta,
                   float* mean, float* rstd, float* al, float* de, double eps, int B, int C,
                   hipStream_t s);
// SyncBatchNorm (data-parallel 3DUNet, unet3d.hip): per-channel fp64 partials of the
// per-(b,c,d) slab sums, part[q][c] = sum over (b, d) of sums[b][c][d][q] (nq = 1 or 2; the
// order of bn_mean / bn_bwd_stats), all-reduced by the caller, then finalised with the
// group's voxel count N (the running statistics as bn_rstd)
hipError_t bn_partial(const float* sums, double* part, Vol vol, int C, int nq, hipStream_t s);
hipError_t bn_mean_fin(const double* part, float* mean, int B, int C, double N, hipStream_t s);
hipError_t bn_rstd_fin(const double* part, const float* gamma, const float* beta,
                       const float* mean, float* rstd, float* al, float* de, float* rmean,
                       float* rvar, double mom, double eps, int B, int C, double N, hipStream_t s);
// dgamma[c] = part[1][c], dbeta[c] = part[0][c] (this rank's share), before the all-reduce
hipError_t bn_bwd_dgb_part(const double* part, float* dgamma, float* dbeta, int C, hipStream_t s);
hipError_t bn_bwd_fin(const double* part, float* k1, float* k2, int B, int C, double N,
                      hipStream_t s);
// eval = 1: backward of the running-statistics transform (k1 = k2 = 0)
hipError_t bn_bwd_stats(const float* sums, float* dgamma, float* dbeta, float* k1, float* k2,
                        Vol vol, int C, hipStream_t s, int eval = 0);

// Depth / height sharding: the shard group's collectives, supplied by the caller through
// spff_coll (include/spff.h).  world == 1: unsharded, every call is a no-op.
struct Coll {
  int world = 1, rank = 0, d_off = 0, D_glob = 0;
  void* ctx = nullptr;
  int (*allreduce)(void*, void*, int64_t, int, void*) = nullptr;
  int (*halo)(void*, float*, int64_t, int, void*) = nullptr;
  // the first callback that failed during the current spff_forward / spff_backward
  // ("allreduce" / "halo"; nullptr: none) -- the entry points report it as SPFF_ECOLL
  mutable const char* failed = nullptr;
  bool on() const { return world > 1; }
  hipError_t sum_f64(double* buf, int64_t n, hipStream_t s) const {
    if (!on()) return hipSuccess;
    if (allreduce(ctx, buf, n, 1, s) == 0) return hipSuccess;
    if (!failed) failed = "allreduce";
    return hipErrorUnknown;
  }
  hipError_t sum_f32(float* buf, int64_t n, hipStream_t s) const {
    if (!on()) return hipSuccess;
    if (allreduce(ctx, buf, n, 0, s) == 0) return hipSuccess;
    if (!failed) failed = "allreduce";
    return hipErrorUnknown;
  }
  int do_halo(float* interior, int64_t slice_floats, int d_local, hipStream_t s) const {
    const int r = halo(ctx, interior, slice_floats, d_local, s);
    if (r != 0 && !failed) failed = "halo";
    return r;
  }
};

// EnergyFiLM hidden width / positional-code rows the scratch layouts are sized for
constexpr int EFH_MAX = 64, EFP_MAX = 32;
struct GateParams {
  const float* pe;   // sinusoidal code [efp][pe_pitch] (models.py:1495-1503), column d_off + d
  int pe_pitch, d_off;
  int efh = 32, efp = 16;  // EnergyFiLM3D hidden, pe_dims
  int fphase = 0;          // FourierGate3D(learn_phase=True): M_k + 0.01 i (models.py:1538-1539)
  // EnergyFiLM (models.py:1479-1512)
  const float* fw0; const float* fb0; const float* fw2; const float* fb2;  // null if off
  // FourierGate (models.py:1515-1544)
  const float* mask; const float* mag;                                      // null if off
  // SE (models.py:600-609)
  const float* sw0; const float* sb0; const float* sw2; const float* sb2;   // null if off
  int specse;
  bool efilm_ready = false;  // t, bt, hid already computed (efilm_fwd_all at the forward start)
};
struct GateSaved {
  float* t; float* bt; float* hid;    // EFiLM: t=tanh(gamma)[C][D], beta[C][D], hid_pre[H][D]
  float* s1; float* g1; float* sg2;   // [B][D]
  float* p; float* h; float* e;       // SE: p[B][C], h[B][Hse] (pre-ReLU), e[B][C]
  float* P; float* Q;                 // [B][C][D] apply coefficients
  float* PT = nullptr;                // optional copies [B][D][C] (GEMM loaders, ActRows)
  float* QT = nullptr;
  double* spec;                       // sharded plans: s1 spectrum [B][L][2] (global D)
};
int se_hidden(int C);
// EnergyFiLM coefficients of several blocks in one launch (they depend on the parameters
// only): t = tanh(gamma), bt = beta [C][D] and the hidden pre-activations hid [32][D]
struct EfilmJob {
  const float* fw0; const float* fb0; const float* fw2; const float* fb2;
  float* t; float* bt; float* hid; int C;
};
struct EfilmJobs {
  EfilmJob j[8];
  int n = 0;
  int H = 32, P = 16;  // hidden, pe_dims (every block alike)
};
// LDS bytes of the EFiLM coefficient kernels (H hidden, P code rows, D depths)
size_t efilm_fwd_lds(int H, int P, int D);
hipError_t efilm_fwd_all(const float* pe, int pe_pitch, const EfilmJobs& jobs, int D,
                         hipStream_t s);
// forward gate algebra from Sa[b,c,d] = sum_hw lrelu(IN(y2))
hipError_t gates_fwd(const GateParams& gp, const float* Sa, GateSaved& sv, Vol vol, int C,
                     float* scratch, hipStream_t s);
struct GateGrads {
  float* fw0; float* fb0; float* fw2; float* fb2;
  float* mask; float* mag;
  float* sw0; float* sb0; float* sw2; float* sb2;
};
// backward gate algebra: from per-(b,c,d) [sum dout, sum dout*a2] -> A,Bc with
// da2 = dout*A + Bc, plus parameter grads.
hipError_t gates_bwd(const GateParams& gp, const GateSaved& sv, const float* Sa,
                     const float* Sg, GateGrads& gg, float* A, float* Bc, Vol vol, int C,
                     float* scratch, hipStream_t s);
size_t gates_scratch_bytes(Vol vol, int C);
// the same on a depth-sharded slab: vol.D = local depth, co.D_glob the full one;
// partial spectra / channel sums are all-reduced through co between kernels
hipError_t gates_fwd_sh(const GateParams& gp, const float* Sa, GateSaved& sv, Vol vol, int C,
                        float* scratch, const Coll& co, hipStream_t s);
hipError_t gates_bwd_sh(const GateParams& gp, const GateSaved& sv, const float* Sa,
                        const float* Sg, GateGrads& gg, float* A, float* Bc, Vol vol, int C,
                        float* scratch, const Coll& co, hipStream_t s);
size_t gates_sh_scratch_bytes(Vol vol, int C, int D_glob);

// ------------------------------------------------------- height sharding --
// (hshard.hip) the boundary rows of a height-sharded plan's conv input, in place: a
// staging slab [recv_lo | send_lo | send_hi | recv_hi] of B D W ldr floats each
// (ldr = hrows_ld(cin)); hrows_pack writes rows 0 and H - 1 of x (both sources, raw)
// into the send slices, the caller exchanges them (spff_coll.halo at d_local = 2), and
// the conv reads recv_lo / recv_hi through Src2::rlo / rhi -- no padded copy of the
// volume and no copy of the conv output.
int hrows_ld(int cin);
size_t hstage_floats(Vol v, int ldr);
hipError_t hrows_pack(const Src2& x, int cin, float* send, Vol v, int ldr, hipStream_t s);

// ------------------------------------------------------------------ misc --
hipError_t ncdhw_to_ndhwc(const float* x, float* y, Vol vol, int C, int ldy, hipStream_t s);
hipError_t maxpool_fwd(const float* x, float* y, uint8_t* idx, Vol in, int C, hipStream_t s);
// dx = dskip(ld) + unpool(dp, idx)
hipError_t maxpool_bwd_add(const float* dp, const uint8_t* idx, const float* dskip, int ldskip,
                           float* dx, Vol in, int C, hipStream_t s);
hipError_t scale_by_dev(float* x, int64_t n, const float* scale, hipStream_t s);
// stream-ordered fill of 32-bit words by a kernel (graph-capturable in place of
// hipMemsetAsync); bytes and p multiples of 4
hipError_t fill32_async(void* p, size_t bytes, unsigned value, hipStream_t s);
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  return fill32_async(p, bytes, 0u, s);
}
// the decoder's _cat fallback (models.py:687-691): F.interpolate(up, skip size, trilinear,
// align_corners=False) from (D, Hi, Wi) to (D, Ho, Wo) -- the D factor is exactly 1 --
// and its backward (gather form, fixed order).  Channel-last, ld = C (multiple of 4).
hipError_t resize_hw_fwd(const float* x, float* y, Vol in, int Ho, int Wo, int C, hipStream_t s);
hipError_t resize_hw_bwd(const float* dy, float* dx, Vol in, int Ho, int Wo, int C, hipStream_t s);
// MaxPool3d(2) (full 2x2x2), first-max ties; idx = (dd*2+dh)*2+dw
hipError_t maxpool3_fwd(const float* x, float* y, uint8_t* idx, Vol in, int C, hipStream_t s);
hipError_t maxpool3_bwd_add(const float* dp, const uint8_t* idx, const float* dskip, int ldskip,
                            float* dx, Vol in, int C, hipStream_t s);
// trilinear depth resampling with H, W unchanged (align_corners=False)
hipError_t resize_d_ncdhw_to_ndhwc(const float* x, float* y, int B, int C, int Din, int Dout,
                                   int H, int W, int ldy, hipStream_t s);
hipError_t resize_d_rows(const float* x, float* y, int B, int K, int Din, int Dout, int H, int W,
                         hipStream_t s);
hipError_t resize_d_rows_bwd(const float* dy, float* dx, int B, int K, int Din, int Dout, int H,
                             int W, hipStream_t s);

// ----------------------------------------------------------------- optim --
hipError_t adam_step(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                     double beta1, double beta2, double eps, double wd, int decoupled,
                     int64_t step, hipStream_t s);

// ------------------------------------------------------------------ loss --
size_t loss_ws_bytes(int64_t V, int K);
// conf: K x (K+1) int64, conf[pred*(K+1) + label], column K = label outside [0,K)
hipError_t loss_fwd(const float* logits, const int64_t* labels, int64_t V, int K, int ignore,
                    double smooth, const int64_t* count_override, float* out4, float* dlogits,
                    int64_t* conf, float* ws, hipStream_t s, const float* class_w = nullptr,
                    int clamp1 = 0);
hipError_t count_valid(const int64_t* labels, int64_t V, int ignore, int64_t* count,
                       hipStream_t s);
hipError_t confusion_only(const float* logits, const int64_t* labels, int64_t V, int K,
                          int ignore, int64_t* conf, hipStream_t s);

// ------------------------------------------------ wave-staged voxel rows --
// The loss kernels read [V][K] channel-last rows (K = 13: 52 B per voxel).  A
// wave copies the contiguous run of its 64 voxels between HBM and its LDS slice
// with coalesced (float4 when aligned) accesses; threads then work on their own
// row in LDS.  wave_lds_sync orders one wave's LDS writes before its reads by
// other lanes (LDS executes a wave's instructions in order; the fence and
// wave_barrier keep the compiler from moving accesses across it).
// Up to 4 quads (or 4 floats) per lane are loaded before any is stored, so a run of up to
// 1024 floats (K <= 16) costs one memory latency, not one per loop trip.
#ifndef SPFF_COPY_BATCH
#define SPFF_COPY_BATCH 1
#endif
__device__ __forceinline__ void wave_copy_rows(float* __restrict__ dst,
                                               const float* __restrict__ src, int n, int lane) {
  if (!SPFF_COPY_BATCH) {
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && (n & 3) == 0) {
      for (int i = lane; i < (n >> 2); i += 64)
        reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
    } else {
      for (int i = lane; i < n; i += 64) dst[i] = src[i];
    }
    return;
  }
  // (clamped unconditional loads, predicated stores: a conditionally loaded register array
  // went to scratch)
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && (n & 3) == 0) {
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i0 = lane; i0 < n4; i0 += 256) {
      const float4 r0 = s4[i0];
      const float4 r1 = s4[min(i0 + 64, n4 - 1)];
      const float4 r2 = s4[min(i0 + 128, n4 - 1)];
      const float4 r3 = s4[min(i0 + 192, n4 - 1)];
      d4[i0] = r0;
      if (i0 + 64 < n4) d4[i0 + 64] = r1;
      if (i0 + 128 < n4) d4[i0 + 128] = r2;
      if (i0 + 192 < n4) d4[i0 + 192] = r3;
    }
  } else {
    for (int i0 = lane; i0 < n; i0 += 256) {
      const float r0 = src[i0];
      const float r1 = src[min(i0 + 64, n - 1)];
      const float r2 = src[min(i0 + 128, n - 1)];
      const float r3 = src[min(i0 + 192, n - 1)];
      dst[i0] = r0;
      if (i0 + 64 < n) dst[i0 + 64] = r1;
      if (i0 + 128 < n) dst[i0 + 128] = r2;
      if (i0 + 192 < n) dst[i0 + 192] = r3;
    }
  }
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace spff
