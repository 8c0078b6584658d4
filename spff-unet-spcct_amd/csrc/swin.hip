// SwinUNETR variant (BASELINE config 5): the reference's "SwinUNETR" registry
// entry (config.py:366-386) = LitSwinUNETR_Published (models.py:880-982) around
// SwinUNETR_Published (models.py:858-878), i.e. MONAI 1.5.2's SwinUNETR with
// feature_size 12, depths (1,1,1,1), heads (1,2,4,8), window 7 (the registry's
// window_size=(2,2,2) is dropped by build_class, config.py:159-182), mlp_ratio 2,
// InstanceNorm, res_block.  Semantics restated in oracle/swin_oracle.py
// (parity unpinned: MONAI is not available offline).
//
// Volumes: L0 = input (D, H, W), Ll = L0 / 2^l.  Swin stage s runs at L(s+1)
// with C = f 2^s channels; every tensor is channel-last rows [B][D][H][W][C].
//   x0 = PatchEmbed(x) (Conv3d k = s = 2)                  L1, f
//   t0 = x0; stage s: t(s+1) = Merge(Block(t s))          L(s+2), 2C
//   hs s = LN(t s) without affine (proj_out, normalize=True)
//   Block: x1 = t + Proj(WinAttn(LN1 t)); x2 = x1 + L2(GELU(L1(LN2 x1)))
//   Merge: LN(cat of 8 stride-2 slices, MONAI legacy order) -> Linear(8C -> 2C)
//   enc0 = RB(x), enc1 = RB(hs0), enc2 = RB(hs1), enc3 = RB(hs2), dec4 = RB(hs4)
//   dec3 = UP(dec4, hs3), dec2 = UP(dec3, enc3), dec1 = UP(dec2, enc2),
//   dec0 = UP(dec1, enc1), out = UP(dec0, enc0), logits = Conv1x1(out) + b
//   RB (UnetResBlock): lrelu(IN(conv(lrelu(IN(conv x)))) + [IN(conv1x1 x) | x])
//   UP (UnetrUpBlock): RB(cat[ConvT2(x), skip]) with the 1x1 shortcut
// Kernels: the engine's 3x3x3 convs (any SPFF_MATH_*), IN statistics / apply /
// backward of norm.hip (affine-free: gamma = 1, beta = 0), the fp32-MFMA GEMMs
// of gemm.hip for every Linear / 1x1 conv / ConvTranspose / patch embedding,
// and the window attention, layer norms and residual tails of swin_attn.hip /
// swin_ops.hip.
#include "spff_internal.h"
#include "swin_internal.h"
#include "spff.h"

#include <algorithm>
#include <string>
#include <vector>

using namespace spff;

namespace {

int sfail(int code, const std::string& m) { return set_error(code, m.c_str()); }
#define SHIPCK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return sfail(SPFF_EHIP, std::string(#expr) + " -> " + hipGetErrorString(_e));        \
  } while (0)
#define SCK(expr)                   \
  do {                              \
    int _r = (expr);                \
    if (_r != SPFF_OK) return _r;   \
  } while (0)

constexpr int NL = 6, NRB = 10, NUP = 5, NST = 4;

struct SEnt {
  std::string name;
  std::vector<int64_t> shape;
  int64_t off, numel;
};

struct Lin {  // nn.Linear / 1x1 conv W [N][K] (+ b)
  int64_t w = -1, b = -1;
  int K = 0, N = 0;
  size_t pk = 0;  // packed wf | wd
};

struct RB {
  std::string name;
  int L, Cin, C;
  bool has3;
  int64_t w1 = -1, w2 = -1;
  Lin c3;
  size_t y1, a1, y2, y3, out;
  size_t st[3][4];  // (mean, rstd, al, de) of the IN after conv1, conv2, conv3
  size_t pk[4] = {0, 0, 0, 0};  // batched conv images: w1 fwd, w2 fwd, w2 dgrad, w1 dgrad
};

struct Up {
  int Cin, Cout, Llow;
  int64_t w = -1;
  size_t pk, out;
};

struct Stage {
  int L, C, nh, hid;
  AttnGeo g;
  int64_t n1w, n1b, tab, n2w, n2b, mnw, mnb;
  Lin qkv, proj, l1, l2, red;
  size_t n1, mu1, rs1, qkvb, O, lse, x1, n2, mu2, rs2, hpre, hact, x2, mn, mmu, mrs;
};

inline int rup(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace

struct spff_swin {
  spff_swin_cfg cfg;
  Vol vol[NL];
  int f, K, ldx;
  std::vector<SEnt> params;
  int64_t nparam = 0;
  int64_t pe_w = -1, pe_b = -1;
  size_t pe_pk = 0;
  Stage stg[NST];
  RB rb[NRB];  // enc0, enc1, enc2, enc3, enc10, dec5, dec4, dec3, dec2, dec1
  Up up[NUP];  // decoder5 .. decoder1 transposed convs
  Lin head;
  size_t x_cl = 0, t[5] = {}, hs[5] = {}, hmu[5] = {}, hrs[5] = {};
  size_t ones = 0, zeros = 0, dummy = 0, red_ws = 0, red_out = 0, kk1 = 0, kk2 = 0, wg_ws = 0,
         wt = 0, cst = 0;
  bool pkb = false;  // conv images packed in one batch at the forward start (rb[i].pk)
  size_t wsl = 0;    // SPFF_MATH_F16X3 max |w| per conv, [NRB][2] (batched plans)
  // backward scratch
  size_t G_out = 0, G_dz = 0, G_dy2 = 0, G_da1 = 0, G_up = 0;
  size_t d_enc[4] = {}, d_hs[5] = {}, dT[5] = {};
  size_t S_a = 0, S_b = 0, S_c = 0, S_qkv = 0, S_h = 0;
  size_t total = 0;
  int maxC = 0;
  // per call
  char* ws = nullptr;
  const float* prm = nullptr;
  float* dprm = nullptr;
  hipStream_t st = nullptr;

  float* F(size_t off) const { return reinterpret_cast<float*>(ws + off); }
  const float* P(int64_t off) const { return off < 0 ? nullptr : prm + off; }
  float* DP(int64_t off) const { return off < 0 ? nullptr : dprm + off; }
  size_t alloc(size_t bytes) {
    size_t o = total;
    total += (bytes + 255) / 256 * 256;
    return o;
  }
  int64_t reg(const std::string& name, std::vector<int64_t> shape) {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    params.push_back(SEnt{name, shape, nparam, n});
    nparam += n;
    return nparam - n;
  }
};

namespace {

size_t fbytes(int64_t n) { return (size_t)n * sizeof(float); }

void reg_lin(spff_swin* p, Lin& l, const std::string& name, int K, int N, bool bias,
             std::vector<int64_t> wshape = {}) {
  l.K = K;
  l.N = N;
  if (wshape.empty()) wshape = {N, K};
  l.w = p->reg(name + ".weight", wshape);
  if (bias) l.b = p->reg(name + ".bias", {N});
  l.pk = p->alloc(head_pack_floats(K, N) * sizeof(float));
}

void reg_rb(spff_swin* p, RB& r, const std::string& name, int L, int Cin, int C) {
  r.name = name;
  r.L = L;
  r.Cin = Cin;
  r.C = C;
  r.has3 = Cin != C;
  r.w1 = p->reg(name + ".conv1.conv.weight", {C, Cin, 3, 3, 3});
  r.w2 = p->reg(name + ".conv2.conv.weight", {C, C, 3, 3, 3});
  if (r.has3) reg_lin(p, r.c3, name + ".conv3.conv", Cin, C, false, {C, Cin, 1, 1, 1});
}

int build(spff_swin* p) {
  const spff_swin_cfg& c = p->cfg;
  if (c.batch < 1 || c.in_ch < 1 || c.in_ch > 8 || c.num_classes < 1 || c.num_classes > 32)
    return sfail(SPFF_EINVAL, "invalid batch / in_ch (1..8) / num_classes (1..32)");
  if (c.depth % 32 || c.height % 32 || c.width % 32 || c.depth < 32 || c.height < 32 ||
      c.width < 32)
    return sfail(SPFF_ESHAPE, "SwinUNETR needs D, H, W divisible by 2**5 = 32 (MONAI "
                              "_check_input_size; LitSwinUNETR pads to a multiple of 32)");
  if ((c.depth / 32) * (c.height / 32) * (c.width / 32) < 2)
    return sfail(SPFF_ESHAPE, "the 1/32-resolution bottleneck must hold more than one voxel "
                              "(InstanceNorm3d: 'Expected more than 1 spatial element')");
  if (c.feature_size < 4 || c.feature_size % 4)
    return sfail(SPFF_EINVAL, "feature_size must be a positive multiple of 4");
  if (c.window < 1 || c.window > 7) return sfail(SPFF_EINVAL, "window must be 1..7");
  if (c.math < SPFF_MATH_F32 || c.math > SPFF_MATH_F16X3)
    return sfail(SPFF_EINVAL, "math must be one of SPFF_MATH_*");
  p->f = c.feature_size;
  p->K = c.num_classes;
  p->ldx = rup(c.in_ch, 8);
  for (int l = 0; l < NL; ++l) p->vol[l] = Vol{c.batch, c.depth >> l, c.height >> l, c.width >> l};
  const int f = p->f, B = c.batch;
  // ---- parameters, in MONAI SwinUNETR registration order (oracle.param_shapes)
  p->pe_w = p->reg("swinViT.patch_embed.proj.weight", {f, c.in_ch, 2, 2, 2});
  p->pe_b = p->reg("swinViT.patch_embed.proj.bias", {f});
  p->pe_pk = p->alloc(head_pack_floats(8 * c.in_ch, f) * sizeof(float));
  const int W3 = (2 * c.window - 1) * (2 * c.window - 1) * (2 * c.window - 1);
  for (int s = 0; s < NST; ++s) {
    Stage& S = p->stg[s];
    S.L = s + 1;
    S.C = f << s;
    S.nh = c.heads[s];
    if (S.nh < 1 || S.C % S.nh) return sfail(SPFF_EINVAL, "heads must divide the stage width");
    const int hd = S.C / S.nh;
    if (hd != 4 && hd != 8 && hd != 12 && hd != 16 && hd != 24 && hd != 32)
      return sfail(SPFF_EINVAL, "head_dim must be one of 4, 8, 12, 16, 24, 32");
    S.hid = (int)(S.C * (double)c.mlp_ratio);
    if (S.hid < 4 || S.hid % 4) return sfail(SPFF_EINVAL, "mlp hidden width must be a multiple of 4");
    const std::string b = "swinViT.layers" + std::to_string(s + 1) + ".0.blocks.0.";
    S.n1w = p->reg(b + "norm1.weight", {S.C});
    S.n1b = p->reg(b + "norm1.bias", {S.C});
    S.tab = p->reg(b + "attn.relative_position_bias_table", {W3, S.nh});
    reg_lin(p, S.qkv, b + "attn.qkv", S.C, 3 * S.C, true);
    reg_lin(p, S.proj, b + "attn.proj", S.C, S.C, true);
    S.n2w = p->reg(b + "norm2.weight", {S.C});
    S.n2b = p->reg(b + "norm2.bias", {S.C});
    reg_lin(p, S.l1, b + "mlp.linear1", S.C, S.hid, true);
    reg_lin(p, S.l2, b + "mlp.linear2", S.hid, S.C, true);
    const std::string d = "swinViT.layers" + std::to_string(s + 1) + ".0.downsample.";
    reg_lin(p, S.red, d + "reduction", 8 * S.C, 2 * S.C, false);
    S.mnw = p->reg(d + "norm.weight", {8 * S.C});
    S.mnb = p->reg(d + "norm.bias", {8 * S.C});
    const Vol& v = p->vol[S.L];
    S.g = attn_geo(B, v.D, v.H, v.W, c.window, S.C, S.nh);
  }
  RB* R = p->rb;
  reg_rb(p, R[0], "encoder1.layer", 0, c.in_ch, f);
  reg_rb(p, R[1], "encoder2.layer", 1, f, f);
  reg_rb(p, R[2], "encoder3.layer", 2, 2 * f, 2 * f);
  reg_rb(p, R[3], "encoder4.layer", 3, 4 * f, 4 * f);
  reg_rb(p, R[4], "encoder10.layer", 5, 16 * f, 16 * f);
  const char* dn[NUP] = {"decoder5", "decoder4", "decoder3", "decoder2", "decoder1"};
  const int uci[NUP] = {16 * f, 8 * f, 4 * f, 2 * f, f};
  const int uco[NUP] = {8 * f, 4 * f, 2 * f, f, f};
  for (int u = 0; u < NUP; ++u) {
    Up& U = p->up[u];
    U.Cin = uci[u];
    U.Cout = uco[u];
    U.Llow = 5 - u;
    U.w = p->reg(std::string(dn[u]) + ".transp_conv.conv.weight", {U.Cin, U.Cout, 2, 2, 2});
    reg_rb(p, R[5 + u], std::string(dn[u]) + ".conv_block", U.Llow - 1, 2 * U.Cout, U.Cout);
  }
  reg_lin(p, p->head, "out.conv.conv", f, p->K, true, {p->K, f, 1, 1, 1});

  // ---- workspace
  const Vol& v0 = p->vol[0];
  p->x_cl = p->alloc(fbytes(nvox(v0) * p->ldx));
  int maxC = 16 * f;
  size_t red_ws = 0, red_out = 0, wg = 0, wt = 0, cst = 0, gmax = 0;
  for (int l = 1; l <= 5; ++l) {
    const int C = f << (l - 1);
    p->t[l - 1] = p->alloc(fbytes(nvox(p->vol[l]) * C));
    p->hs[l - 1] = p->alloc(fbytes(nvox(p->vol[l]) * C));
    p->hmu[l - 1] = p->alloc(fbytes(nvox(p->vol[l])));
    p->hrs[l - 1] = p->alloc(fbytes(nvox(p->vol[l])));
    p->dT[l - 1] = p->alloc(fbytes(nvox(p->vol[l]) * C));
    p->d_hs[l - 1] = p->alloc(fbytes(nvox(p->vol[l]) * C));
    wg = std::max(wg, ln_bwd_ws_bytes(nvox(p->vol[l]), C));
  }
  size_t sa = 0, sq = 0, sh = 0;
  for (int s = 0; s < NST; ++s) {
    Stage& S = p->stg[s];
    const int64_t T = nvox(p->vol[S.L]), T8 = T / 8;
    const int C = S.C;
    S.n1 = p->alloc(fbytes(T * C));
    S.mu1 = p->alloc(fbytes(T));
    S.rs1 = p->alloc(fbytes(T));
    S.qkvb = p->alloc(fbytes(T * 3 * C));
    S.O = p->alloc(fbytes(T * C));
    S.lse = p->alloc(fbytes(S.g.nwin() * S.nh * S.g.n));
    S.x1 = p->alloc(fbytes(T * C));
    S.n2 = p->alloc(fbytes(T * C));
    S.mu2 = p->alloc(fbytes(T));
    S.rs2 = p->alloc(fbytes(T));
    S.hpre = p->alloc(fbytes(T * S.hid));
    S.hact = p->alloc(fbytes(T * S.hid));
    S.x2 = p->alloc(fbytes(T * C));
    S.mn = p->alloc(fbytes(T8 * 8 * C));
    S.mmu = p->alloc(fbytes(T8));
    S.mrs = p->alloc(fbytes(T8));
    sa = std::max(sa, fbytes(T * C));
    sq = std::max(sq, fbytes(T * 3 * C));
    sh = std::max(sh, fbytes(T * S.hid));
    wg = std::max(wg, swin_attn_ws_bytes(S.g));
    wg = std::max(wg, linear_wgrad_ws_bytes(T, C, 3 * C));
    wg = std::max(wg, linear_wgrad_ws_bytes(T, S.hid, C));
    wg = std::max(wg, linear_wgrad_ws_bytes(T, C, S.hid));
    wg = std::max(wg, linear_wgrad_ws_bytes(T8, 8 * C, 2 * C));
    wg = std::max(wg, ln_bwd_ws_bytes(T, C));
    wg = std::max(wg, ln_bwd_ws_bytes(T8, 8 * C));
    maxC = std::max(maxC, 8 * C);
  }
  p->S_a = p->alloc(sa);
  p->S_b = p->alloc(sa);
  p->S_c = p->alloc(sa);
  p->S_qkv = p->alloc(sq);
  p->S_h = p->alloc(sh);
  for (int i = 0; i < NRB; ++i) {
    RB& r = R[i];
    const Vol& v = p->vol[r.L];
    const int64_t V = nvox(v);
    const int C = r.C;
    r.y1 = p->alloc(fbytes(V * C));
    r.a1 = p->alloc(fbytes(V * C));
    r.y2 = p->alloc(fbytes(V * C));
    r.y3 = r.has3 ? p->alloc(fbytes(V * C)) : 0;
    r.out = p->alloc(fbytes(V * C));
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 4; ++j) r.st[k][j] = p->alloc(fbytes((int64_t)B * C));
    red_ws = std::max(red_ws, slab_reduce_ws_bytes(v, C, 2));
    red_out = std::max(red_out, fbytes((int64_t)B * C * v.D * 2));
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, 3, r.Cin, C));
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, 3, C, C));
    wg = std::max(wg, conv3d_splitk_bytes(v, 3, r.Cin, C));
    wg = std::max(wg, conv3d_splitk_bytes(v, 3, C, C));
    wg = std::max(wg, conv3d_splitk_bytes(v, 3, C, r.Cin));
    if (r.has3) wg = std::max(wg, linear_wgrad_ws_bytes(V, r.Cin, C));
    wt = std::max(wt, conv3d_pack_bytes(3, r.Cin, C));
    wt = std::max(wt, conv3d_pack_bytes(3, C, C));
    cst = std::max(cst, conv3d_stats_bytes(v, 3, r.Cin, C));
    cst = std::max(cst, conv3d_stats_bytes(v, 3, C, C));
    gmax = std::max(gmax, fbytes(V * std::max(C, r.Cin)));
    maxC = std::max(maxC, std::max(C, r.Cin));
  }
  for (int u = 0; u < NUP; ++u) {
    Up& U = p->up[u];
    U.out = p->alloc(fbytes(nvox(p->vol[U.Llow - 1]) * U.Cout));
    U.pk = p->alloc(upconv_pack_floats(U.Cin, U.Cout, 8) * sizeof(float));
    wg = std::max(wg, upconv_wgrad_ws_bytes(p->vol[U.Llow], U.Cin, U.Cout, 8));
  }
  wg = std::max(wg, linear_wgrad_ws_bytes(nvox(v0), f, p->K));
  wg = std::max(wg, linear_wgrad_ws_bytes(nvox(p->vol[1]), 8 * c.in_ch, f));
  p->maxC = maxC;
  p->ones = p->alloc(fbytes(maxC));
  p->zeros = p->alloc(fbytes(maxC));
  p->dummy = p->alloc(fbytes(2 * maxC));
  p->red_ws = p->alloc(red_ws);
  p->red_out = p->alloc(red_out);
  p->kk1 = p->alloc(fbytes((int64_t)B * maxC));
  p->kk2 = p->alloc(fbytes((int64_t)B * maxC));
  p->wg_ws = p->alloc(wg);
  p->pkb = conv3d_packs_batched(c.math);
  if (p->pkb) {
    for (int i = 0; i < NRB; ++i) {
      RB& r = R[i];
      r.pk[0] = p->alloc(conv3d_pack_bytes(3, r.Cin, r.C));
      r.pk[1] = p->alloc(conv3d_pack_bytes(3, r.C, r.C));
      r.pk[2] = p->alloc(conv3d_pack_bytes(3, r.C, r.C));
      if (i > 0) r.pk[3] = p->alloc(conv3d_pack_bytes(3, r.Cin, r.C));  // enc0's input: no dx
    }
    p->wsl = p->alloc(NRB * 2 * sizeof(unsigned));
  } else {
    p->wt = p->alloc(wt);
  }
  p->cst = p->alloc(cst);
  p->G_out = p->alloc(gmax);
  p->G_dz = p->alloc(gmax);
  p->G_dy2 = p->alloc(gmax);
  p->G_da1 = p->alloc(gmax);
  p->G_up = p->alloc(gmax);
  for (int l = 0; l < 4; ++l) p->d_enc[l] = p->alloc(fbytes(nvox(p->vol[l]) * (l ? f << (l - 1) : f)));
  return SPFF_OK;
}

// affine-free InstanceNorm3d statistics of y [V][C] -> (mean, rstd, al, de)
int in_stats(spff_swin* p, const Vol& v, int C, size_t y, const size_t* st4) {
  RedArgs a{};
  a.y = p->F(y);
  SHIPCK(slab_reduce(RED_SUM, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  SHIPCK(in_mean(p->F(p->red_out), p->F(st4[0]), v, C, p->st));
  a.mean = p->F(st4[0]);
  SHIPCK(slab_reduce(RED_SQDEV, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  SHIPCK(in_rstd(p->F(p->red_out), p->F(p->ones), p->F(p->zeros), p->F(st4[0]), p->F(st4[1]),
                 p->F(st4[2]), p->F(st4[3]), v, C, p->st));
  return SPFF_OK;
}

// batched plans: every conv's max |w| (f16x3) in one launch, then all 39 conv images
// (forward and input gradient) in one more, at the forward start -- the weights do not
// change between a step's forward and backward (the up-conv / linear images are packed up
// front the same way).  Otherwise conv3d_pack before each conv (max + pack launches).
int prep_weights(spff_swin* p) {
  if (!p->pkb) return SPFF_OK;
  const int math = p->cfg.math;
  const bool f16 = math == SPFF_MATH_F16X3;
  unsigned* sl = reinterpret_cast<unsigned*>(p->ws + p->wsl);
  PrepJobs pj;
  PackJobs kj;
  if (f16) SHIPCK(spff::zero_async(sl, NRB * 2 * sizeof(unsigned), p->st));
  for (int i = 0; i < NRB; ++i) {
    RB& r = p->rb[i];
    unsigned* w1 = f16 ? sl + 2 * i : nullptr;
    unsigned* w2 = f16 ? sl + 2 * i + 1 : nullptr;
    bool ok = true;
    if (f16) {
      ok = ok && prep_absmax(&pj, p->P(r.w1), (int64_t)r.C * r.Cin * 27, w1);
      ok = ok && prep_absmax(&pj, p->P(r.w2), (int64_t)r.C * r.C * 27, w2);
    }
    ok = ok && conv3d_pack_job(&kj, p->P(r.w1), p->F(r.pk[0]), 3, r.Cin, r.C, false, w1);
    ok = ok && conv3d_pack_job(&kj, p->P(r.w2), p->F(r.pk[1]), 3, r.C, r.C, false, w2);
    ok = ok && conv3d_pack_job(&kj, p->P(r.w2), p->F(r.pk[2]), 3, r.C, r.C, true, w2);
    if (r.pk[3]) ok = ok && conv3d_pack_job(&kj, p->P(r.w1), p->F(r.pk[3]), 3, r.Cin, r.C, true, w1);
    if (!ok) return sfail(SPFF_EINVAL, "weight preparation table overflow");
  }
  SHIPCK(prep_run(pj, p->st));
  SHIPCK(conv3d_pack_many(kj, math, p->st));
  return SPFF_OK;
}
// conv k of residual block r (0: w1 fwd, 1: w2 fwd, 2: w2 dgrad, 3: w1 dgrad): its image
// (the batched one, else packed now into the scratch image) and its max |w| slot
int conv_image(spff_swin* p, const RB& r, int k, const Vol& v, const float** img,
               const unsigned** wmax) {
  const bool c1 = k == 0 || k == 3;
  const int ri = (int)(&r - p->rb);
  if (p->pkb) {
    if (!r.pk[k]) return sfail(SPFF_EINVAL, "no batched image for this conv");
    *img = p->F(r.pk[k]);
    *wmax = p->cfg.math == SPFF_MATH_F16X3
                ? reinterpret_cast<const unsigned*>(p->ws + p->wsl) + 2 * ri + (c1 ? 0 : 1)
                : nullptr;
    return SPFF_OK;
  }
  SHIPCK(conv3d_pack(p->P(c1 ? r.w1 : r.w2), p->F(p->wt), v, 3, c1 ? r.Cin : r.C, r.C, k >= 2,
                     p->cfg.math, p->st));
  *img = p->F(p->wt);
  *wmax = nullptr;
  return SPFF_OK;
}

// 3x3x3 conv k (0 / 1) of r + (fused where the kernel allows) IN statistics
int conv_in(spff_swin* p, const Src2& in, const RB& r, int k, const Vol& v, int Cin, int C,
            size_t y, const size_t* st4) {
  const int math = p->cfg.math;
  const float* img;
  const unsigned* wmax;
  SCK(conv_image(p, r, k, v, &img, &wmax));
  const bool fuse = conv3d_fuses_stats(v, 3, Cin, C, math);
  SHIPCK(conv3d_run(in, img, dst1(p->F(y), C), v, 3, Cin, C, false, math, p->st,
                    p->F(p->wg_ws), fuse ? p->F(p->cst) : nullptr, 0, wmax));
  if (fuse) {
    SHIPCK(conv3d_in_stats_fin(p->F(p->cst), v, 3, Cin, C, math, p->F(p->ones), p->F(p->zeros),
                               p->F(st4[0]), p->F(st4[1]), p->F(st4[2]), p->F(st4[3]), p->st));
    return SPFF_OK;
  }
  return in_stats(p, v, C, y, st4);
}

int rb_fwd(spff_swin* p, RB& r, const Src2& in, const float* ident) {
  const Vol& v = p->vol[r.L];
  const int C = r.C;
  SCK(conv_in(p, in, r, 0, v, r.Cin, C, r.y1, r.st[0]));
  SHIPCK(act_apply(p->F(r.y1), p->F(r.a1), p->F(r.st[0][2]), p->F(r.st[0][3]), nullptr, nullptr, v,
                   C, p->st));
  SCK(conv_in(p, src1(p->F(r.a1), C), r, 1, v, C, C, r.y2, r.st[1]));
  if (r.has3) {
    float* pk = p->F(r.c3.pk);
    SHIPCK(head_pack(p->P(r.c3.w), pk, pk + head_pack_dgrad_offset(r.Cin, C), r.Cin, C, p->st));
    SHIPCK(linear_fwd2(in, r.Cin, pk, nullptr, p->F(r.y3), C, C, nvox(v), p->st));
    SCK(in_stats(p, v, C, r.y3, r.st[2]));
  }
  SHIPCK(res_act(p->F(r.y2), p->F(r.st[1][2]), p->F(r.st[1][3]), r.has3 ? p->F(r.y3) : nullptr,
                 p->F(r.st[2][2]), p->F(r.st[2][3]), ident, nullptr, p->F(r.out), v, C, p->st));
  return SPFF_OK;
}

// IN (+ activation slope neg) backward: dy = IN'(g * slope(r)) for r = y*al + de
int in_bwd(spff_swin* p, const Vol& v, int C, size_t y, const float* g, float* dy,
           const size_t* st4, float neg) {
  RedArgs a{};
  a.y = p->F(y); a.g = g; a.mean = p->F(st4[0]); a.rstd = p->F(st4[1]);
  a.al = p->F(st4[2]); a.de = p->F(st4[3]); a.neg = neg;
  SHIPCK(slab_reduce(RED_BWD_IN, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  float* dm = p->F(p->dummy);
  SHIPCK(in_bwd_stats(p->F(p->red_out), p->F(p->ones), dm, dm + p->maxC, p->F(p->kk1),
                      p->F(p->kk2), v, C, p->st));
  SHIPCK(in_bwd_apply(p->F(y), g, dy, p->F(st4[0]), p->F(st4[1]), p->F(st4[2]), p->F(st4[3]),
                      p->F(p->ones), nullptr, nullptr, p->F(p->kk1), p->F(p->kk2), v, C, p->st,
                      neg));
  return SPFF_OK;
}

// dsrc (may be null): written (conv1 dgrad), then the shortcut's gradient added
int rb_bwd(spff_swin* p, RB& r, const float* dout, const Src2& in, const float* ident,
           const Dst2* dsrc) {
  const Vol& v = p->vol[r.L];
  const int C = r.C, math = p->cfg.math;
  const int64_t V = nvox(v);
  float* dz = p->F(p->G_dz);
  float* dy2 = p->F(p->G_dy2);
  float* da1 = p->F(p->G_da1);
  SHIPCK(res_act(p->F(r.y2), p->F(r.st[1][2]), p->F(r.st[1][3]), r.has3 ? p->F(r.y3) : nullptr,
                 p->F(r.st[2][2]), p->F(r.st[2][3]), ident, dout, dz, v, C, p->st));
  SCK(in_bwd(p, v, C, r.y2, dz, dy2, r.st[1], 1.f));
  SHIPCK(conv3d_wgrad(src1(p->F(r.a1), C), dy2, C, p->DP(r.w2), v, 3, C, C, math, p->F(p->wg_ws),
                      p->st));
  const float* img;
  const unsigned* wmax;
  SCK(conv_image(p, r, 2, v, &img, &wmax));
  SHIPCK(conv3d_run(src1(dy2, C), img, dst1(da1, C), v, 3, C, C, true, math, p->st,
                    p->F(p->wg_ws), nullptr, 0, wmax));
  SCK(in_bwd(p, v, C, r.y1, da1, da1, r.st[0], 0.01f));
  SHIPCK(conv3d_wgrad(in, da1, C, p->DP(r.w1), v, 3, r.Cin, C, math, p->F(p->wg_ws), p->st));
  if (dsrc) {
    SCK(conv_image(p, r, 3, v, &img, &wmax));
    SHIPCK(conv3d_run(src1(da1, C), img, *dsrc, v, 3, r.Cin, C, true, math, p->st,
                      p->F(p->wg_ws), nullptr, 0, wmax));
  }
  if (r.has3) {
    SCK(in_bwd(p, v, C, r.y3, dz, dy2, r.st[2], 1.f));
    SHIPCK(linear_wgrad2(in, r.Cin, dy2, C, C, p->DP(r.c3.w), p->F(p->dummy), V, p->F(p->wg_ws),
                         p->st));
    if (dsrc) {
      const float* wd = p->F(r.c3.pk) + head_pack_dgrad_offset(r.Cin, C);
      SHIPCK(linear_dgrad2(dy2, C, C, wd, *dsrc, r.Cin, V, 1, p->st));
    }
  } else if (dsrc) {
    SHIPCK(add_inplace(dsrc->p0, dz, V * C, p->st));
  }
  return SPFF_OK;
}

int stage_fwd(spff_swin* p, Stage& S, const float* tin, float* tout) {
  const Vol& v = p->vol[S.L];
  const int64_t T = nvox(v), T8 = T / 8;
  const int C = S.C;
  hipStream_t st = p->st;
  auto pack = [&](Lin& l) -> hipError_t {
    float* pk = p->F(l.pk);
    return head_pack(p->P(l.w), pk, pk + head_pack_dgrad_offset(l.K, l.N), l.K, l.N, st);
  };
  SHIPCK(ln_fwd(tin, C, C, p->P(S.n1w), p->P(S.n1b), p->F(S.n1), C, p->F(S.mu1), p->F(S.rs1), T,
                st));
  SHIPCK(pack(S.qkv));
  SHIPCK(linear_fwd(p->F(S.n1), C, C, p->F(S.qkv.pk), p->P(S.qkv.b), p->F(S.qkvb), 3 * C, 3 * C, T,
                    nullptr, 0, st));
  SHIPCK(swin_attn_fwd(p->F(S.qkvb), p->P(S.qkv.b), p->P(S.tab), S.g, p->F(S.O), p->F(S.lse), st));
  SHIPCK(pack(S.proj));
  SHIPCK(linear_fwd(p->F(S.O), C, C, p->F(S.proj.pk), p->P(S.proj.b), p->F(S.x1), C, C, T, tin, C,
                    st));
  SHIPCK(ln_fwd(p->F(S.x1), C, C, p->P(S.n2w), p->P(S.n2b), p->F(S.n2), C, p->F(S.mu2),
                p->F(S.rs2), T, st));
  SHIPCK(pack(S.l1));
  SHIPCK(linear_fwd_gelu(p->F(S.n2), C, C, p->F(S.l1.pk), p->P(S.l1.b), p->F(S.hpre), p->F(S.hact),
                         S.hid, T, st));
  SHIPCK(pack(S.l2));
  SHIPCK(linear_fwd(p->F(S.hact), S.hid, S.hid, p->F(S.l2.pk), p->P(S.l2.b), p->F(S.x2), C, C, T,
                    p->F(S.x1), C, st));
  SHIPCK(ln_merge_fwd(p->F(S.x2), C, v.B, v.D, v.H, v.W, p->P(S.mnw), p->P(S.mnb), p->F(S.mn),
                      p->F(S.mmu), p->F(S.mrs), st));
  SHIPCK(pack(S.red));
  SHIPCK(linear_fwd(p->F(S.mn), 8 * C, 8 * C, p->F(S.red.pk), nullptr, tout, 2 * C, 2 * C, T8,
                    nullptr, 0, st));
  return SPFF_OK;
}

// dtout [T/8][2C] -> dtin [T][C] (written)
int stage_bwd(spff_swin* p, Stage& S, const float* tin, const float* dtout, float* dtin) {
  const Vol& v = p->vol[S.L];
  const int64_t T = nvox(v), T8 = T / 8;
  const int C = S.C;
  hipStream_t st = p->st;
  float* wg = p->F(p->wg_ws);
  auto wd = [&](Lin& l) { return p->F(l.pk) + head_pack_dgrad_offset(l.K, l.N); };
  float* A = p->F(p->S_a);  // [T][C]-sized scratch (d mn and dcat are T/8 x 8C = T x C)
  float* Bf = p->F(p->S_b);
  float* Cf = p->F(p->S_c);
  // merge: Linear(8C -> 2C) then LayerNorm(8C) of the gather
  SHIPCK(linear_wgrad(p->F(S.mn), 8 * C, 8 * C, dtout, 2 * C, 2 * C, p->DP(S.red.w), p->F(p->dummy),
                      T8, wg, st));
  SHIPCK(linear_dgrad(dtout, 2 * C, 2 * C, wd(S.red), A, 8 * C, 8 * C, T8, nullptr, st));
  SHIPCK(ln_merge_bwd(p->F(S.x2), C, v.B, v.D, v.H, v.W, p->P(S.mnw), p->F(S.mmu), p->F(S.mrs), A,
                      Bf, p->DP(S.mnw), wg, st));
  SHIPCK(unmerge(Bf, C, v.B, v.D, v.H, v.W, A, st));  // A = d x2
  // MLP: x2 = x1 + L2(gelu(L1(LN2(x1))))
  float* dh = p->F(p->S_h);
  SHIPCK(linear_wgrad(p->F(S.hact), S.hid, S.hid, A, C, C, p->DP(S.l2.w), p->DP(S.l2.b), T, wg, st));
  SHIPCK(linear_dgrad(A, C, C, wd(S.l2), dh, S.hid, S.hid, T, p->F(S.hpre), st));
  SHIPCK(linear_wgrad(p->F(S.n2), C, C, dh, S.hid, S.hid, p->DP(S.l1.w), p->DP(S.l1.b), T, wg, st));
  SHIPCK(linear_dgrad(dh, S.hid, S.hid, wd(S.l1), Bf, C, C, T, nullptr, st));  // Bf = d n2
  // d x1 = d x2 + LN2'(d n2)  (into Cf)
  SHIPCK(ln_bwd(p->F(S.x1), C, C, p->P(S.n2w), p->F(S.mu2), p->F(S.rs2), Bf, C, Cf, C, A, C,
                p->DP(S.n2w), wg, T, st));
  // attention: x1 = t + Proj(O)
  SHIPCK(linear_wgrad(p->F(S.O), C, C, Cf, C, C, p->DP(S.proj.w), p->DP(S.proj.b), T, wg, st));
  SHIPCK(linear_dgrad(Cf, C, C, wd(S.proj), A, C, C, T, nullptr, st));  // A = dO
  float* dq = p->F(p->S_qkv);
  SHIPCK(swin_attn_bwd(p->F(S.qkvb), p->P(S.qkv.b), p->P(S.tab), p->F(S.O), A, p->F(S.lse), S.g,
                       dq, p->DP(S.tab), nullptr, wg, st));
  // the qkv weight gradient reuses wg: take the padded tokens' bias part first
  SHIPCK(linear_dgrad(dq, 3 * C, 3 * C, wd(S.qkv), Bf, C, C, T, nullptr, st));  // Bf = d n1
  float* dpad = p->F(p->dummy);  // [3C] padded-token k / v bias grads
  SHIPCK(spff::zero_async(dpad, fbytes(3 * C), st));
  SHIPCK(swin_attn_pad_grad(S.g, wg, dpad, st));
  SHIPCK(hipMemcpyAsync(A, dpad, fbytes(3 * C), hipMemcpyDeviceToDevice, st));  // A free again
  SHIPCK(linear_wgrad(p->F(S.n1), C, C, dq, 3 * C, 3 * C, p->DP(S.qkv.w), p->DP(S.qkv.b), T, wg,
                      st));
  SHIPCK(add_inplace(p->DP(S.qkv.b), A, 3 * C, st));
  // d t = d x1 + LN1'(d n1)
  SHIPCK(ln_bwd(tin, C, C, p->P(S.n1w), p->F(S.mu1), p->F(S.rs1), Bf, C, dtin, C, Cf, C,
                p->DP(S.n1w), wg, T, st));
  return SPFF_OK;
}

int forward(spff_swin* p, const float* x, float* logits) {
  const spff_swin_cfg& c = p->cfg;
  const int f = p->f;
  const Vol& v0 = p->vol[0];
  hipStream_t st = p->st;
  SHIPCK(spff::fill32_async(p->F(p->ones), (size_t)p->maxC * 4, 0x3f800000u, st));
  SHIPCK(spff::zero_async(p->F(p->zeros), fbytes(p->maxC), st));
  SHIPCK(ncdhw_to_ndhwc(x, p->F(p->x_cl), v0, c.in_ch, p->ldx, st));
  // patch embedding -> t0 (L1, f); hs0 = LN(t0)
  float* pk = p->F(p->pe_pk);
  SHIPCK(head_pack(p->P(p->pe_w), pk, pk + head_pack_dgrad_offset(8 * c.in_ch, f), 8 * c.in_ch, f,
                   st));
  SHIPCK(patch_embed_fwd(p->F(p->x_cl), p->ldx, c.in_ch, v0.D, v0.H, v0.W, v0.B, pk, p->P(p->pe_b),
                         p->F(p->t[0]), f, st));
  for (int l = 0; l < 5; ++l) {
    if (l > 0) SCK(stage_fwd(p, p->stg[l - 1], p->F(p->t[l - 1]), p->F(p->t[l])));
    const int C = f << l;
    SHIPCK(ln_fwd(p->F(p->t[l]), C, C, nullptr, nullptr, p->F(p->hs[l]), C, p->F(p->hmu[l]),
                  p->F(p->hrs[l]), nvox(p->vol[l + 1]), st));
  }
  SCK(prep_weights(p));
  RB* R = p->rb;
  SCK(rb_fwd(p, R[0], src1(p->F(p->x_cl), p->ldx), nullptr));
  for (int i = 1; i < 4; ++i) {
    const int C = f << (i - 1);
    SCK(rb_fwd(p, R[i], src1(p->F(p->hs[i - 1]), C), p->F(p->hs[i - 1])));
  }
  SCK(rb_fwd(p, R[4], src1(p->F(p->hs[4]), 16 * f), p->F(p->hs[4])));
  const float* prev = p->F(R[4].out);
  const float* skip[NUP] = {p->F(p->hs[3]), p->F(R[3].out), p->F(R[2].out), p->F(R[1].out),
                            p->F(R[0].out)};
  for (int u = 0; u < NUP; ++u) {
    Up& U = p->up[u];
    float* upk = p->F(U.pk);
    SHIPCK(upconv_pack(p->P(U.w), upk, upk + upconv_pack_dgrad_offset(U.Cin, U.Cout, 8), U.Cin,
                       U.Cout, st, 8));
    SHIPCK(upconv_fwd(prev, upk, p->F(p->zeros), p->F(U.out), p->vol[U.Llow], U.Cin, U.Cout, st, 8));
    RB& r = R[5 + u];
    SCK(rb_fwd(p, r, Src2{p->F(U.out), skip[u], U.Cout, U.Cout, U.Cout}, nullptr));
    prev = p->F(r.out);
  }
  float* hp = p->F(p->head.pk);
  SHIPCK(head_pack(p->P(p->head.w), hp, hp + head_pack_dgrad_offset(f, p->K), f, p->K, st));
  SHIPCK(linear_fwd(prev, f, f, hp, p->P(p->head.b), logits, p->K, p->K, nvox(v0), nullptr, 0, st));
  return SPFF_OK;
}

int backward(spff_swin* p, const float* dl) {
  const spff_swin_cfg& c = p->cfg;
  const int f = p->f;
  const Vol& v0 = p->vol[0];
  hipStream_t st = p->st;
  RB* R = p->rb;
  float* wg = p->F(p->wg_ws);
  float* Gout = p->F(p->G_out);
  float* hp = p->F(p->head.pk);
  SHIPCK(linear_wgrad(p->F(R[9].out), f, f, dl, p->K, p->K, p->DP(p->head.w), p->DP(p->head.b),
                      nvox(v0), wg, st));
  SHIPCK(linear_dgrad(dl, p->K, p->K, hp + head_pack_dgrad_offset(f, p->K), Gout, f, f, nvox(v0),
                      nullptr, st));
  // decoders: dec1 (R9) <- up1 <- dec2 (R8) ... <- dec5 (R5) <- up5 <- enc10 (R4)
  float* dskip[NUP] = {p->F(p->d_hs[3]), p->F(p->d_enc[3]), p->F(p->d_enc[2]), p->F(p->d_enc[1]),
                       p->F(p->d_enc[0])};
  const float* skip[NUP] = {p->F(p->hs[3]), p->F(R[3].out), p->F(R[2].out), p->F(R[1].out),
                            p->F(R[0].out)};
  for (int u = NUP - 1; u >= 0; --u) {
    Up& U = p->up[u];
    RB& r = R[5 + u];
    float* dup = p->F(p->G_up);
    Dst2 dx{dup, dskip[u], U.Cout, U.Cout, U.Cout};
    SCK(rb_bwd(p, r, Gout, Src2{p->F(U.out), skip[u], U.Cout, U.Cout, U.Cout}, nullptr, &dx));
    const float* xlow = p->F(u == 0 ? R[4].out : R[5 + u - 1].out);
    SHIPCK(upconv_wgrad(xlow, dup, U.Cout, p->DP(U.w), p->F(p->dummy), p->vol[U.Llow], U.Cin, U.Cout,
                        wg, st, 8));
    float* upk = p->F(U.pk);
    SHIPCK(upconv_dgrad(dup, U.Cout, upk + upconv_pack_dgrad_offset(U.Cin, U.Cout, 8), Gout,
                        p->vol[U.Llow], U.Cin, U.Cout, st, 8));
  }
  // Gout = d enc10.out
  {
    Dst2 dx = dst1(p->F(p->d_hs[4]), 16 * f);
    SCK(rb_bwd(p, R[4], Gout, src1(p->F(p->hs[4]), 16 * f), p->F(p->hs[4]), &dx));
  }
  for (int i = 3; i >= 1; --i) {
    const int C = f << (i - 1);
    Dst2 dx = dst1(p->F(p->d_hs[i - 1]), C);
    SCK(rb_bwd(p, R[i], p->F(p->d_enc[i]), src1(p->F(p->hs[i - 1]), C), p->F(p->hs[i - 1]), &dx));
  }
  SCK(rb_bwd(p, R[0], p->F(p->d_enc[0]), src1(p->F(p->x_cl), p->ldx), nullptr, nullptr));
  // Swin: dT[l] = grad of t l = (stage l backward) + LN'(d hs l)
  for (int l = 4; l >= 0; --l) {
    const int C = f << l;
    const int64_t T = nvox(p->vol[l + 1]);
    float* dTl = p->F(p->dT[l]);
    if (l < 4) SCK(stage_bwd(p, p->stg[l], p->F(p->t[l]), p->F(p->dT[l + 1]), dTl));
    SHIPCK(ln_bwd(p->F(p->t[l]), C, C, nullptr, p->F(p->hmu[l]), p->F(p->hrs[l]), p->F(p->d_hs[l]), C,
                  dTl, C, l < 4 ? dTl : nullptr, C, nullptr, wg, T, st));
  }
  SHIPCK(patch_embed_wgrad(p->F(p->x_cl), p->ldx, c.in_ch, v0.D, v0.H, v0.W, v0.B, p->F(p->dT[0]), f,
                           p->DP(p->pe_w), p->DP(p->pe_b), wg, st));
  return SPFF_OK;
}

}  // namespace

// =================================================================== C ABI ==
extern "C" {

int spff_swin_create(const spff_swin_cfg* cfg, spff_swin** out) {
  if (!cfg || !out) return sfail(SPFF_EINVAL, "null argument");
  spff_swin* p = new spff_swin();
  p->cfg = *cfg;
  const int r = build(p);
  if (r != SPFF_OK) {
    delete p;
    return r;
  }
  *out = p;
  return SPFF_OK;
}

void spff_swin_destroy(spff_swin* p) { delete p; }

int spff_swin_num_params(const spff_swin* p) { return p ? (int)p->params.size() : 0; }

int spff_swin_param_info(const spff_swin* p, int i, const char** name, int* ndim,
                         int64_t shape[5], int64_t* offset, int64_t* numel) {
  if (!p || i < 0 || i >= (int)p->params.size()) return sfail(SPFF_EINVAL, "param index");
  const SEnt& e = p->params[i];
  if (name) *name = e.name.c_str();
  if (ndim) *ndim = (int)e.shape.size();
  if (shape)
    for (int k = 0; k < 5; ++k) shape[k] = k < (int)e.shape.size() ? e.shape[k] : 1;
  if (offset) *offset = e.off;
  if (numel) *numel = e.numel;
  return SPFF_OK;
}

int64_t spff_swin_param_floats(const spff_swin* p) { return p ? p->nparam : 0; }
size_t spff_swin_workspace_bytes(const spff_swin* p) { return p ? p->total : 0; }

int spff_swin_forward(spff_swin* p, const float* x, const float* params, float* logits, void* ws,
                      void* stream) {
  if (!p || !x || !params || !logits || !ws) return sfail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = nullptr;
  p->st = static_cast<hipStream_t>(stream);
  return forward(p, x, logits);
}

int spff_swin_backward(spff_swin* p, const float* dlogits, const float* params, float* dparams,
                       void* ws, void* stream) {
  if (!p || !dlogits || !params || !dparams || !ws) return sfail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = dparams;
  p->st = static_cast<hipStream_t>(stream);
  return backward(p, dlogits);
}

int spff_swin_saved_tensor(const spff_swin* p, void* ws, const char* name, const float** ptr,
                           int64_t* nv, int* ch) {
  if (!p || !ws || !name || !ptr) return sfail(SPFF_EINVAL, "null argument");
  const char* base = static_cast<const char*>(ws);
  const std::string n(name);
  auto ret = [&](size_t off, int64_t rows, int c) {
    *ptr = reinterpret_cast<const float*>(base + off);
    if (nv) *nv = rows;
    if (ch) *ch = c;
    return SPFF_OK;
  };
  const int f = p->f;
  for (int l = 0; l < 5; ++l) {
    const int64_t T = nvox(p->vol[l + 1]);
    if (n == "t" + std::to_string(l)) return ret(p->t[l], T, f << l);
    if (n == "hs" + std::to_string(l)) return ret(p->hs[l], T, f << l);
    if (n == "grad.t" + std::to_string(l)) return ret(p->dT[l], T, f << l);
  }
  for (int s = 0; s < NST; ++s) {
    const Stage& S = p->stg[s];
    const std::string pre = "stage" + std::to_string(s) + ".";
    const int64_t T = nvox(p->vol[S.L]);
    if (n == pre + "n1") return ret(S.n1, T, S.C);
    if (n == pre + "qkv") return ret(S.qkvb, T, 3 * S.C);
    if (n == pre + "O") return ret(S.O, T, S.C);
    if (n == pre + "x1") return ret(S.x1, T, S.C);
    if (n == pre + "hpre") return ret(S.hpre, T, S.hid);
    if (n == pre + "x2") return ret(S.x2, T, S.C);
    if (n == pre + "mn") return ret(S.mn, T / 8, 8 * S.C);
  }
  for (int i = 0; i < NRB; ++i) {
    const RB& r = p->rb[i];
    const int64_t V = nvox(p->vol[r.L]);
    if (n == r.name + ".y1") return ret(r.y1, V, r.C);
    if (n == r.name + ".a1") return ret(r.a1, V, r.C);
    if (n == r.name + ".y2") return ret(r.y2, V, r.C);
    if (r.has3 && n == r.name + ".y3") return ret(r.y3, V, r.C);
    if (n == r.name + ".out") return ret(r.out, V, r.C);
    for (int k = 0; k < 3; ++k) {
      if (k == 2 && !r.has3) break;
      const std::string j = std::to_string(k + 1);
      if (n == r.name + ".al" + j) return ret(r.st[k][2], p->cfg.batch, r.C);
      if (n == r.name + ".de" + j) return ret(r.st[k][3], p->cfg.batch, r.C);
    }
  }
  const char* upn[NUP] = {"up5", "up4", "up3", "up2", "up1"};
  for (int u = 0; u < NUP; ++u)
    if (n == upn[u]) return ret(p->up[u].out, nvox(p->vol[p->up[u].Llow - 1]), p->up[u].Cout);
  return sfail(SPFF_EINVAL, "unknown saved tensor " + n);
}

size_t spff_swin_loss_ws_bytes(int batch, int num_classes) {
  return dice_ce_ws_bytes(batch, num_classes);
}

int spff_swin_loss(const float* logits, const int64_t* labels, int batch, int64_t vox_per_sample,
                   int num_classes, int ignore_index, int include_bg, double ce_weight,
                   float* out4, float* dlogits, void* ws, void* stream) {
  if (!logits || !labels || !out4 || !dlogits || !ws) return sfail(SPFF_EINVAL, "null argument");
  SHIPCK(dice_ce_loss(logits, labels, batch, vox_per_sample, num_classes, ignore_index, include_bg,
                      ce_weight, out4, dlogits, ws, static_cast<hipStream_t>(stream)));
  return SPFF_OK;
}

}  // extern "C"
