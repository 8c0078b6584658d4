// Internal declarations of the SwinUNETR variant's kernels (swin_ops.hip,
// swin_attn.hip), used by swin.hip.  Layout: channel-last token rows
// [B][D][H][W][C], as the rest of the engine.
#pragma once
#include "spff_internal.h"

namespace spff {

// ---------------------------------------------------------- layer norm --
// y[m][c] = (x - mean) * rstd (* g[c] + b[c] when g != null), eps 1e-5, over C
// channels of row m; mu / rs [M] saved for the backward
hipError_t ln_fwd(const float* x, int ldx, int C, const float* g, const float* b, float* y,
                  int ldy, float* mu, float* rs, int64_t M, hipStream_t s);
// legacy PatchMerging: rows of the 8 stride-2 slices of xf [B][D][H][W][Cf] in
// MONAI's cat order, normalised over 8 Cf -> y [B*D/2*H/2*W/2][8 Cf]
hipError_t ln_merge_fwd(const float* xf, int Cf, int B, int D, int H, int W, const float* g,
                        const float* b, float* y, float* mu, float* rs, hipStream_t s);
size_t ln_bwd_ws_bytes(int64_t M, int C);
// dx = LN backward of dy (+ res); dgb (optional): [2][C] = dgamma, dbeta
hipError_t ln_bwd(const float* x, int ldx, int C, const float* g, const float* mu,
                  const float* rs, const float* dy, int lddy, float* dx, int lddx,
                  const float* res, int ldres, float* dgb, float* ws, int64_t M, hipStream_t s);
// backward of ln_merge_fwd up to the cat: dcat [M][8 Cf], dgb [2][8 Cf]
hipError_t ln_merge_bwd(const float* xf, int Cf, int B, int D, int H, int W, const float* g,
                        const float* mu, const float* rs, const float* dy, float* dcat, float* dgb,
                        float* ws, hipStream_t s);
// dxf [B][D][H][W][Cf] = gradient of the merge gather from dcat (written)
hipError_t unmerge(const float* dcat, int Cf, int B, int D, int H, int W, float* dxf,
                   hipStream_t s);

// -------------------------------------------------- UnetResBlock tail --
// fwd (dout null): out = lrelu(y2*al2 + de2 + (y3 ? y3*al3 + de3 : r))
// bwd: out = dout * lrelu'(same z)
hipError_t res_act(const float* y2, const float* al2, const float* de2, const float* y3,
                   const float* al3, const float* de3, const float* r, const float* dout,
                   float* out, Vol v, int C, hipStream_t s);
hipError_t add_inplace(float* y, const float* x, int64_t n, hipStream_t s);
// out[i] (+)= sum_k part[k*stride + i] (k < n, in order), i < count
hipError_t col_reduce(const float* part, int n, int64_t stride, int count, float* out, int acc,
                      hipStream_t s);
// the same with an output index map (see swin_ops.hip): mode 1 = bias-table transpose,
// mode 2 = padded-token k / v bias columns
hipError_t col_reduce_map(const float* part, int n, int64_t stride, int count, float* out,
                          int acc, int mode, int R, int nh, int hd, int C, hipStream_t s);

// ------------------------------------------------------------- loss --
size_t dice_ce_ws_bytes(int B, int K);
// LitSwinUNETR_Published._loss: out4 = [ce, loss, dice_loss, N_valid], dlogits
// [V][K] = dloss/dlogits (channel-last rows, vps voxels per sample)
hipError_t dice_ce_loss(const float* logits, const int64_t* labels, int B, int64_t vps, int K,
                        int ignore, int include_bg, double ce_weight, float* out4, float* dlogits,
                        void* ws, hipStream_t s);

// ---------------------------------------------------- window attention --
// One unshifted Swin window-attention layer over a token grid [B][D][H][W]:
// windows of ws = min(w, dim) per axis (zero-padded after norm1, so padded
// tokens carry q, k, v = the qkv bias), heads of hd channels, relative bias
// table [(2w-1)^3][nh] indexed with the w^3 window's pairwise index.
struct AttnGeo {
  int B, D, H, W;
  int w;             // configured window (MONAI window_size)
  int wsd, wsh, wsw; // effective window per axis
  int nwd, nwh, nww; // windows per axis
  int n;             // tokens per window
  int C, nh, hd;
  float scale;       // hd ** -0.5
  __host__ __device__ int64_t nwin() const { return (int64_t)B * nwd * nwh * nww; }
  __host__ __device__ int R() const { return (2 * w - 1) * (2 * w - 1) * (2 * w - 1); }
};
AttnGeo attn_geo(int B, int D, int H, int W, int w, int C, int nh);
// qkv [T][3C] (rows of the real tokens), bqkv [3C]; O [T][C]; lse [nwin][nh][n]
hipError_t swin_attn_fwd(const float* qkv, const float* bqkv, const float* table,
                         const AttnGeo& g, float* O, float* lse, hipStream_t s);
size_t swin_attn_ws_bytes(const AttnGeo& g);
// dO [T][C] -> dqkv [T][3C] (written), dtable [R][nh] (written), dbqkv [3C]
// (the k / v parts INCREMENTED by the padded tokens' gradients; null: later, by
// swin_attn_pad_grad from the same ws)
hipError_t swin_attn_bwd(const float* qkv, const float* bqkv, const float* table,
                         const float* O, const float* dO, const float* lse, const AttnGeo& g,
                         float* dqkv, float* dtable, float* dbqkv, float* ws, hipStream_t s);
hipError_t swin_attn_pad_grad(const AttnGeo& g, const float* ws, float* dbqkv, hipStream_t s);

}  // namespace spff
