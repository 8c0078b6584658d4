// 3D U-Net baseline variant (BASELINE config 3): the Cicek et al. 3D U-Net of
// the reference's "3DUNet" registry entry (config.py:283-311), behind
// LitCicek3DUNet_DepthAdapter_Published (models.py:756-853).
//
// Graph (Cicek3DUNet.forward, models.py:743-753), levels l = 0..4 halve D, H, W:
//   e1 = enc1(x); e2 = enc2(pool(e1)); e3 = enc3(pool(e2)); e4 = enc4(pool(e3))
//   b  = bott(pool(e4))
//   d4 = dec4([up4(b) | e4]); d3 = dec3([up3(d4) | e3]); d2 = dec2([up2(d3) | e2])
//   d1 = dec1([up1(d2) | e1]); logits = out(d1)
// Block (models.py:721-726): y1 = conv(x); a1 = relu(BN(y1)); y2 = conv(a1);
// out = relu(BN(y2)), Conv3d(3, padding 1, bias=False) since use_bn=True.
// The depth adapter (models.py:771-777) resamples the input's D to target_depth
// before the backbone and the logits back afterwards (misc.hip).
//
// Everything runs on the SPFF engine's kernels: the 3x3x3 convs of
// conv3d_x.hip / conv3d_wgx.hip (any SPFF_MATH_*), the per-(b,c,d) slab
// reductions of norm.hip finalised per channel for BatchNorm, act_apply /
// in_bwd_apply with ReLU's zero slope, the ConvTranspose GEMMs of gemm.hip with
// 8 sub-lattices, and the 2x2x2 max pool of misc.hip.  Saved for backward:
// y1, a1, y2, out per block, the pool argmax bytes and the statistics.
#include "spff_internal.h"
#include "spff.h"

#include <string>
#include <vector>

using namespace spff;

namespace {

int ufail(int code, const std::string& m) { return set_error(code, m.c_str()); }
#define UHIPCK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return ufail(SPFF_EHIP, std::string(#expr) + " -> " + hipGetErrorString(_e));        \
  } while (0)
#define UCK(expr)                   \
  do {                              \
    int _r = (expr);                \
    if (_r != SPFF_OK) return _r;   \
  } while (0)

constexpr int NLVL = 5, NBLK = 9, NUP = 4, NSUB = 8;
constexpr double BN_MOM = 0.1, BN_EPS = 1e-5;  // nn.BatchNorm3d defaults

struct UEnt {
  std::string name;
  std::vector<int64_t> shape;
  int64_t off, numel;
};

struct UBlk {
  std::string name;
  int lvl, Cin, C;
  int64_t w1 = -1, g1 = -1, b1 = -1, w2 = -1, g2 = -1, b2 = -1;  // params
  int64_t rm1 = -1, rv1 = -1, rm2 = -1, rv2 = -1;                // buffers
  size_t y1, a1, y2, out;
  size_t mean1, rstd1, al1, de1, mean2, rstd2, al2, de2;
  size_t pk[4] = {0, 0, 0, 0};  // batched conv images: w1 fwd, w2 fwd, w2 dgrad, w1 dgrad
};

struct UUp {
  int Cin, Cout, lvl_low;
  int64_t w, b;
  size_t pk, out;
};

inline int rup(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace

struct spff_unet3d {
  spff_unet3d_cfg cfg;
  Vol vol[NLVL];
  int f, K, ldx, Dt;
  std::vector<UEnt> params, bufs;
  int64_t nparam = 0, nbuf = 0;
  UBlk blk[NBLK];  // enc1..enc4, bott, dec4..dec1
  UUp up[NUP];     // up4, up3, up2, up1
  int64_t out_w = -1, out_b = -1;
  size_t head_pk = 0, x_cl = 0, pool[4] = {}, pidx[4] = {};
  size_t red_ws = 0, red_out = 0, kk1 = 0, kk2 = 0, wg_ws = 0, wt = 0;
  bool pkb = false;  // conv images packed in one batch at the forward start (b.pk)
  size_t wsl = 0;    // SPFF_MATH_F16X3 max |w| per conv, [NBLK][2] (batched plans)
  size_t G_out = 0, G_dy2 = 0, G_da1 = 0, G_dx = 0, dskip[4] = {}, logit_t = 0, dl_t = 0;
  size_t total = 0;
  bool last_training = true;
  // synchronised BatchNorm (spff_unet3d_set_sync_bn): the per-channel batch moments and the
  // backward's two per-channel sums are all-reduced (fp64) over the data-parallel group, so
  // every rank normalises with the GLOBAL batch statistics (torch.nn.SyncBatchNorm); world
  // 1 or no table: per-replica statistics, as DDP without SyncBN
  Coll co;
  size_t bnp = 0;  // fp64 per-channel partials [2][16 f]
  // per call
  char* ws = nullptr;
  const float* prm = nullptr;
  float* dprm = nullptr;
  float* buf = nullptr;
  hipStream_t st = nullptr;

  float* F(size_t off) const { return reinterpret_cast<float*>(ws + off); }
  const float* P(int64_t off) const { return off < 0 ? nullptr : prm + off; }
  float* DP(int64_t off) const { return off < 0 ? nullptr : dprm + off; }
  float* BF(int64_t off) const { return off < 0 || !buf ? nullptr : buf + off; }
  size_t alloc(size_t bytes) {
    size_t o = total;
    total += (bytes + 255) / 256 * 256;
    return o;
  }
  int64_t reg(const std::string& name, std::vector<int64_t> shape) {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    params.push_back(UEnt{name, shape, nparam, n});
    nparam += n;
    return nparam - n;
  }
  int64_t regb(const std::string& name, int64_t n) {
    bufs.push_back(UEnt{name, {n}, nbuf, n});
    nbuf += n;
    return nbuf - n;
  }
};

namespace {

void reg_block(spff_unet3d* p, UBlk& b) {
  const int C = b.C;
  // nn.Sequential(conv, BN, ReLU, conv, BN, ReLU): indices 0, 1, 3, 4
  b.w1 = p->reg(b.name + ".0.weight", {C, b.Cin, 3, 3, 3});
  b.g1 = p->reg(b.name + ".1.weight", {C});
  b.b1 = p->reg(b.name + ".1.bias", {C});
  b.w2 = p->reg(b.name + ".3.weight", {C, C, 3, 3, 3});
  b.g2 = p->reg(b.name + ".4.weight", {C});
  b.b2 = p->reg(b.name + ".4.bias", {C});
  b.rm1 = p->regb(b.name + ".1.running_mean", C);
  b.rv1 = p->regb(b.name + ".1.running_var", C);
  b.rm2 = p->regb(b.name + ".4.running_mean", C);
  b.rv2 = p->regb(b.name + ".4.running_var", C);
}

int build(spff_unet3d* p) {
  const spff_unet3d_cfg& c = p->cfg;
  if (c.batch < 1 || c.in_ch < 1 || c.depth < 1 || c.num_classes < 1 ||
      c.num_classes > SPFF_MAX_CLASSES)
    return ufail(SPFF_EINVAL, "invalid batch/in_ch/depth/num_classes (K must be 1..SPFF_MAX_CLASSES)");
  if (c.base < 8 || c.base % 8) return ufail(SPFF_EINVAL, "base must be a multiple of 8");
  if (c.in_ch > 64) return ufail(SPFF_EINVAL, "in_ch > 64 not supported");
  if (c.math < SPFF_MATH_F32 || c.math > SPFF_MATH_F16X3)
    return ufail(SPFF_EINVAL, "math must be one of SPFF_MATH_*");
  if (c.target_depth < 0) return ufail(SPFF_EINVAL, "target_depth must be >= 0");
  p->Dt = c.target_depth > 0 ? c.target_depth : c.depth;
  if (p->Dt % 16 || c.height % 16 || c.width % 16 || c.height < 16 || c.width < 16)
    return ufail(SPFF_ESHAPE,
                 "backbone D, H and W must be multiples of 16 (four MaxPool3d(2) whose outputs "
                 "torch.cat with the ConvTranspose3d outputs, models.py:743-752)");
  p->f = c.base;
  p->K = c.num_classes;
  p->ldx = rup(c.in_ch, 8);
  for (int l = 0; l < NLVL; ++l)
    p->vol[l] = Vol{c.batch, p->Dt >> l, c.height >> l, c.width >> l};
  const int f = p->f;
  const char* names[NBLK] = {"enc1", "enc2", "enc3", "enc4", "bott",
                             "dec4", "dec3", "dec2", "dec1"};
  const int lvl[NBLK] = {0, 1, 2, 3, 4, 3, 2, 1, 0};
  const int cin[NBLK] = {c.in_ch, f, 2 * f, 4 * f, 8 * f, 16 * f, 8 * f, 4 * f, 2 * f};
  const int cc[NBLK] = {f, 2 * f, 4 * f, 8 * f, 16 * f, 8 * f, 4 * f, 2 * f, f};
  for (int i = 0; i < NBLK; ++i) {
    UBlk& b = p->blk[i];
    b.name = names[i];
    b.lvl = lvl[i];
    b.Cin = cin[i];
    b.C = cc[i];
  }
  // registration order of Cicek3DUNet.__init__ (models.py:727-741)
  for (int i = 0; i < 5; ++i) reg_block(p, p->blk[i]);
  const char* upn[NUP] = {"up4", "up3", "up2", "up1"};
  for (int u = 0; u < NUP; ++u) {
    UUp& U = p->up[u];
    U.Cin = 16 * f >> u;
    U.Cout = 8 * f >> u;
    U.lvl_low = 4 - u;
    U.w = p->reg(std::string(upn[u]) + ".weight", {U.Cin, U.Cout, 2, 2, 2});
    U.b = p->reg(std::string(upn[u]) + ".bias", {U.Cout});
    reg_block(p, p->blk[5 + u]);
  }
  p->out_w = p->reg("out.weight", {p->K, f, 1, 1, 1});
  p->out_b = p->reg("out.bias", {p->K});

  // ---- workspace ----
  const Vol& v0 = p->vol[0];
  const int B = c.batch;
  p->x_cl = p->alloc(nvox(v0) * p->ldx * sizeof(float));
  size_t red_ws = 0, red_out = 0, wg = 0, wt = 0;
  for (int i = 0; i < NBLK; ++i) {
    UBlk& b = p->blk[i];
    const Vol& v = p->vol[b.lvl];
    const size_t act = nvox(v) * b.C * sizeof(float);
    b.y1 = p->alloc(act);
    b.a1 = p->alloc(act);
    b.y2 = p->alloc(act);
    b.out = p->alloc(act);
    const size_t bc = (size_t)B * b.C * sizeof(float);
    b.mean1 = p->alloc(bc); b.rstd1 = p->alloc(bc); b.al1 = p->alloc(bc); b.de1 = p->alloc(bc);
    b.mean2 = p->alloc(bc); b.rstd2 = p->alloc(bc); b.al2 = p->alloc(bc); b.de2 = p->alloc(bc);
    red_ws = std::max(red_ws, slab_reduce_ws_bytes(v, b.C, 2));
    red_out = std::max(red_out, (size_t)B * b.C * v.D * 2 * sizeof(float));
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, 3, b.Cin, b.C));
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, 3, b.C, b.C));
    wg = std::max(wg, conv3d_splitk_bytes(v, 3, b.Cin, b.C));
    wg = std::max(wg, conv3d_splitk_bytes(v, 3, b.C, b.C));
    wt = std::max(wt, conv3d_pack_bytes(3, b.Cin, b.C));
    wt = std::max(wt, conv3d_pack_bytes(3, b.C, b.C));
  }
  for (int l = 0; l < 4; ++l) {
    const Vol& vl = p->vol[l + 1];
    const int C = f << l;
    p->pool[l] = p->alloc(nvox(vl) * C * sizeof(float));
    p->pidx[l] = p->alloc(nvox(vl) * C);
  }
  for (int u = 0; u < NUP; ++u) {
    UUp& U = p->up[u];
    const Vol& vh = p->vol[U.lvl_low - 1];
    U.out = p->alloc(nvox(vh) * U.Cout * sizeof(float));
    U.pk = p->alloc(upconv_pack_floats(U.Cin, U.Cout, NSUB) * sizeof(float));
    wg = std::max(wg, upconv_wgrad_ws_bytes(p->vol[U.lvl_low], U.Cin, U.Cout, NSUB));
  }
  p->head_pk = p->alloc(head_pack_floats(f, p->K) * sizeof(float));
  wg = std::max(wg, head_wgrad_ws_bytes(nvox(v0), f, p->K));
  p->red_ws = p->alloc(red_ws);
  p->red_out = p->alloc(red_out);
  p->kk1 = p->alloc((size_t)B * 16 * f * sizeof(float));
  p->kk2 = p->alloc((size_t)B * 16 * f * sizeof(float));
  p->bnp = p->alloc((size_t)2 * 16 * f * sizeof(double));
  p->wg_ws = p->alloc(wg);
  p->pkb = conv3d_packs_batched(c.math);
  if (p->pkb) {
    for (int i = 0; i < NBLK; ++i) {
      UBlk& b = p->blk[i];
      b.pk[0] = p->alloc(conv3d_pack_bytes(3, b.Cin, b.C));
      b.pk[1] = p->alloc(conv3d_pack_bytes(3, b.C, b.C));
      b.pk[2] = p->alloc(conv3d_pack_bytes(3, b.C, b.C));
      if (i > 0) b.pk[3] = p->alloc(conv3d_pack_bytes(3, b.Cin, b.C));  // enc1's input: no dx
    }
    p->wsl = p->alloc(NBLK * 2 * sizeof(unsigned));
  } else {
    p->wt = p->alloc(wt);
  }
  size_t gmax = 0;  // max over levels of V_l * C_l (the bottleneck has 16 f channels)
  for (int l = 0; l < NLVL; ++l)
    gmax = std::max(gmax, (size_t)nvox(p->vol[l]) * (size_t)(f << l) * sizeof(float));
  p->G_out = p->alloc(gmax);
  p->G_dy2 = p->alloc(gmax);
  p->G_da1 = p->alloc(gmax);
  p->G_dx = p->alloc(gmax);
  for (int l = 0; l < 4; ++l)
    p->dskip[l] = p->alloc(nvox(p->vol[l]) * (f << l) * sizeof(float));
  if (p->Dt != c.depth) {
    p->logit_t = p->alloc(nvox(v0) * p->K * sizeof(float));
    p->dl_t = p->alloc(nvox(v0) * p->K * sizeof(float));
  }
  return SPFF_OK;
}

// BatchNorm3d over a conv output y (models.py:720): batch statistics + running
// update in training, running statistics in eval
int bn_fwd(spff_unet3d* p, const Vol& v, int C, size_t y, size_t mean, size_t rstd, size_t al,
           size_t de, int64_t g, int64_t b, int64_t rm, int64_t rv, bool training) {
  if (!training) {
    UHIPCK(bn_eval(p->BF(rm), p->BF(rv), p->P(g), p->P(b), p->F(mean), p->F(rstd), p->F(al),
                   p->F(de), BN_EPS, v.B, C, p->st));
    return SPFF_OK;
  }
  RedArgs a{};
  a.y = p->F(y);
  UHIPCK(slab_reduce(RED_SUM, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  if (p->co.on()) {  // SyncBN: global moments (same fp64 per-channel sums, then the group's)
    double* part = reinterpret_cast<double*>(p->ws + p->bnp);
    const double N = (double)nvox(v) * p->co.world;  // every rank runs the plan's shape
    UHIPCK(bn_partial(p->F(p->red_out), part, v, C, 1, p->st));
    UHIPCK(p->co.sum_f64(part, C, p->st));
    UHIPCK(bn_mean_fin(part, p->F(mean), v.B, C, N, p->st));
    a.mean = p->F(mean);
    UHIPCK(slab_reduce(RED_SQDEV, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
    UHIPCK(bn_partial(p->F(p->red_out), part, v, C, 1, p->st));
    UHIPCK(p->co.sum_f64(part, C, p->st));
    UHIPCK(bn_rstd_fin(part, p->P(g), p->P(b), p->F(mean), p->F(rstd), p->F(al), p->F(de),
                       p->BF(rm), p->BF(rv), BN_MOM, BN_EPS, v.B, C, N, p->st));
    return SPFF_OK;
  }
  UHIPCK(bn_mean(p->F(p->red_out), p->F(mean), v, C, p->st));
  a.mean = p->F(mean);
  UHIPCK(slab_reduce(RED_SQDEV, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  UHIPCK(bn_rstd(p->F(p->red_out), p->P(g), p->P(b), p->F(mean), p->F(rstd), p->F(al), p->F(de),
                 p->BF(rm), p->BF(rv), BN_MOM, BN_EPS, v, C, p->st));
  return SPFF_OK;
}

// batched plans: every conv's max |w| (f16x3) in one launch, then all 35 conv images
// (forward and input gradient) in one more, at the forward start -- the weights do not
// change between a step's forward and backward (the up-conv / head images are packed up
// front the same way).  Otherwise conv3d_pack before each conv (max + pack launches).
int prep_weights(spff_unet3d* p) {
  if (!p->pkb) return SPFF_OK;
  const int math = p->cfg.math;
  const bool f16 = math == SPFF_MATH_F16X3;
  unsigned* sl = reinterpret_cast<unsigned*>(p->ws + p->wsl);
  PrepJobs pj;
  PackJobs kj;
  if (f16) UHIPCK(spff::zero_async(sl, NBLK * 2 * sizeof(unsigned), p->st));
  for (int i = 0; i < NBLK; ++i) {
    UBlk& b = p->blk[i];
    unsigned* w1 = f16 ? sl + 2 * i : nullptr;
    unsigned* w2 = f16 ? sl + 2 * i + 1 : nullptr;
    bool ok = true;
    if (f16) {
      ok = ok && prep_absmax(&pj, p->P(b.w1), (int64_t)b.C * b.Cin * 27, w1);
      ok = ok && prep_absmax(&pj, p->P(b.w2), (int64_t)b.C * b.C * 27, w2);
    }
    ok = ok && conv3d_pack_job(&kj, p->P(b.w1), p->F(b.pk[0]), 3, b.Cin, b.C, false, w1);
    ok = ok && conv3d_pack_job(&kj, p->P(b.w2), p->F(b.pk[1]), 3, b.C, b.C, false, w2);
    ok = ok && conv3d_pack_job(&kj, p->P(b.w2), p->F(b.pk[2]), 3, b.C, b.C, true, w2);
    if (b.pk[3]) ok = ok && conv3d_pack_job(&kj, p->P(b.w1), p->F(b.pk[3]), 3, b.Cin, b.C, true, w1);
    if (!ok) return ufail(SPFF_EINVAL, "weight preparation table overflow");
  }
  UHIPCK(prep_run(pj, p->st));
  UHIPCK(conv3d_pack_many(kj, math, p->st));
  return SPFF_OK;
}
// conv k of block b (0: w1 fwd, 1: w2 fwd, 2: w2 dgrad, 3: w1 dgrad): its image (the
// batched one, else packed now into the scratch image) and its max |w| slot
int conv_image(spff_unet3d* p, const UBlk& b, int k, const Vol& v, const float** img,
               const unsigned** wmax) {
  const bool c1 = k == 0 || k == 3;
  const int bi = (int)(&b - p->blk);
  if (p->pkb) {
    if (!b.pk[k]) return ufail(SPFF_EINVAL, "no batched image for this conv");
    *img = p->F(b.pk[k]);
    *wmax = p->cfg.math == SPFF_MATH_F16X3
                ? reinterpret_cast<const unsigned*>(p->ws + p->wsl) + 2 * bi + (c1 ? 0 : 1)
                : nullptr;
    return SPFF_OK;
  }
  UHIPCK(conv3d_pack(p->P(c1 ? b.w1 : b.w2), p->F(p->wt), v, 3, c1 ? b.Cin : b.C, b.C, k >= 2,
                     p->cfg.math, p->st));
  *img = p->F(p->wt);
  *wmax = nullptr;
  return SPFF_OK;
}

int fwd_block(spff_unet3d* p, UBlk& b, const Src2& in, bool training) {
  const Vol& v = p->vol[b.lvl];
  const int C = b.C, math = p->cfg.math;
  const float* img;
  const unsigned* wmax;
  UCK(conv_image(p, b, 0, v, &img, &wmax));
  UHIPCK(conv3d_run(in, img, dst1(p->F(b.y1), C), v, 3, b.Cin, C, false, math, p->st,
                    p->F(p->wg_ws), nullptr, 0, wmax));
  UCK(bn_fwd(p, v, C, b.y1, b.mean1, b.rstd1, b.al1, b.de1, b.g1, b.b1, b.rm1, b.rv1, training));
  UHIPCK(act_apply(p->F(b.y1), p->F(b.a1), p->F(b.al1), p->F(b.de1), nullptr, nullptr, v, C,
                   p->st, 0.f));
  UCK(conv_image(p, b, 1, v, &img, &wmax));
  UHIPCK(conv3d_run(src1(p->F(b.a1), C), img, dst1(p->F(b.y2), C), v, 3, C, C, false, math,
                    p->st, p->F(p->wg_ws), nullptr, 0, wmax));
  UCK(bn_fwd(p, v, C, b.y2, b.mean2, b.rstd2, b.al2, b.de2, b.g2, b.b2, b.rm2, b.rv2, training));
  UHIPCK(act_apply(p->F(b.y2), p->F(b.out), p->F(b.al2), p->F(b.de2), nullptr, nullptr, v, C,
                   p->st, 0.f));
  return SPFF_OK;
}

// BatchNorm + ReLU backward: dy = rstd*gamma*(dr - k1 - xhat*k2), dr = g*[r > 0]
int bn_bwd(spff_unet3d* p, const Vol& v, int C, size_t y, const float* g, float* dy, size_t mean,
           size_t rstd, size_t al, size_t de, int64_t gamma, int64_t beta) {
  RedArgs a{};
  a.y = p->F(y); a.g = g; a.mean = p->F(mean); a.rstd = p->F(rstd);
  a.al = p->F(al); a.de = p->F(de); a.neg = 0.f;
  UHIPCK(slab_reduce(RED_BWD_IN, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  if (p->co.on() && p->last_training) {
    // SyncBN: k1, k2 from the group's sums; dgamma / dbeta are this rank's partial sums
    // (the flat gradient is SUM-all-reduced afterwards, like every other parameter's)
    double* part = reinterpret_cast<double*>(p->ws + p->bnp);
    UHIPCK(bn_partial(p->F(p->red_out), part, v, C, 2, p->st));
    UHIPCK(bn_bwd_dgb_part(part, p->DP(gamma), p->DP(beta), C, p->st));
    UHIPCK(p->co.sum_f64(part, 2 * (int64_t)C, p->st));
    UHIPCK(bn_bwd_fin(part, p->F(p->kk1), p->F(p->kk2), v.B, C, (double)nvox(v) * p->co.world,
                      p->st));
  } else {
    UHIPCK(bn_bwd_stats(p->F(p->red_out), p->DP(gamma), p->DP(beta), p->F(p->kk1), p->F(p->kk2),
                        v, C, p->st, p->last_training ? 0 : 1));
  }
  UHIPCK(in_bwd_apply(p->F(y), g, dy, p->F(mean), p->F(rstd), p->F(al), p->F(de), p->P(gamma),
                      nullptr, nullptr, p->F(p->kk1), p->F(p->kk2), v, C, p->st, 0.f));
  return SPFF_OK;
}

int bwd_block(spff_unet3d* p, UBlk& b, const float* dout, const Dst2* dx, const Src2& in) {
  const Vol& v = p->vol[b.lvl];
  const int C = b.C, math = p->cfg.math;
  float* dy2 = p->F(p->G_dy2);
  float* da1 = p->F(p->G_da1);
  UCK(bn_bwd(p, v, C, b.y2, dout, dy2, b.mean2, b.rstd2, b.al2, b.de2, b.g2, b.b2));
  UHIPCK(conv3d_wgrad(src1(p->F(b.a1), C), dy2, C, p->DP(b.w2), v, 3, C, C, math,
                      p->F(p->wg_ws), p->st));
  const float* img;
  const unsigned* wmax;
  UCK(conv_image(p, b, 2, v, &img, &wmax));
  UHIPCK(conv3d_run(src1(dy2, C), img, dst1(da1, C), v, 3, C, C, true, math, p->st,
                    p->F(p->wg_ws), nullptr, 0, wmax));
  UCK(bn_bwd(p, v, C, b.y1, da1, da1, b.mean1, b.rstd1, b.al1, b.de1, b.g1, b.b1));
  UHIPCK(conv3d_wgrad(in, da1, C, p->DP(b.w1), v, 3, b.Cin, C, math, p->F(p->wg_ws), p->st));
  if (dx) {
    UCK(conv_image(p, b, 3, v, &img, &wmax));
    UHIPCK(conv3d_run(src1(da1, C), img, *dx, v, 3, b.Cin, C, true, math, p->st,
                      p->F(p->wg_ws), nullptr, 0, wmax));
  }
  return SPFF_OK;
}

int forward(spff_unet3d* p, const float* x, float* logits, bool training) {
  const spff_unet3d_cfg& c = p->cfg;
  const int f = p->f;
  const Vol& v0 = p->vol[0];
  if (p->Dt != c.depth)  // _resize_depth_like (models.py:153-157)
    UHIPCK(resize_d_ncdhw_to_ndhwc(x, p->F(p->x_cl), c.batch, c.in_ch, c.depth, p->Dt, c.height,
                                   c.width, p->ldx, p->st));
  else
    UHIPCK(ncdhw_to_ndhwc(x, p->F(p->x_cl), v0, c.in_ch, p->ldx, p->st));
  UCK(prep_weights(p));
  UBlk* B = p->blk;
  Src2 in = src1(p->F(p->x_cl), p->ldx);
  for (int l = 0; l < 4; ++l) {
    UCK(fwd_block(p, B[l], in, training));
    UHIPCK(maxpool3_fwd(p->F(B[l].out), p->F(p->pool[l]),
                        reinterpret_cast<uint8_t*>(p->ws + p->pidx[l]), p->vol[l], f << l, p->st));
    in = src1(p->F(p->pool[l]), f << l);
  }
  UCK(fwd_block(p, B[4], in, training));
  const float* prev = p->F(B[4].out);
  for (int u = 0; u < NUP; ++u) {
    UUp& U = p->up[u];
    float* pk = p->F(U.pk);
    UHIPCK(upconv_pack(p->P(U.w), pk, pk + upconv_pack_dgrad_offset(U.Cin, U.Cout, NSUB), U.Cin,
                       U.Cout, p->st, NSUB));
    UHIPCK(upconv_fwd(prev, pk, p->P(U.b), p->F(U.out), p->vol[U.lvl_low], U.Cin, U.Cout, p->st,
                      NSUB, p->cfg.math));
    UBlk& d = B[5 + u];
    const UBlk& skip = B[3 - u];
    // torch.cat([up(x), skip], dim=1) read in place through the two-source view
    UCK(fwd_block(p, d, Src2{p->F(U.out), p->F(skip.out), U.Cout, U.Cout, U.Cout}, training));
    prev = p->F(d.out);
  }
  float* hp = p->F(p->head_pk);
  UHIPCK(head_pack(p->P(p->out_w), hp, hp + head_pack_dgrad_offset(f, p->K), f, p->K, p->st));
  float* lt = p->Dt != c.depth ? p->F(p->logit_t) : logits;
  UHIPCK(head_fwd(prev, hp, p->P(p->out_b), lt, nvox(v0), f, p->K, p->st, p->cfg.math));
  if (p->Dt != c.depth)  // _resize_logits_depth_like (models.py:159-163)
    UHIPCK(resize_d_rows(lt, logits, c.batch, p->K, p->Dt, c.depth, c.height, c.width, p->st));
  p->last_training = training;
  return SPFF_OK;
}

int backward(spff_unet3d* p, const float* dl) {
  const spff_unet3d_cfg& c = p->cfg;
  const int f = p->f;
  const int64_t V0 = nvox(p->vol[0]);
  UBlk* B = p->blk;
  const float* d16 = dl;
  if (p->Dt != c.depth) {
    UHIPCK(resize_d_rows_bwd(dl, p->F(p->dl_t), c.batch, p->K, p->Dt, c.depth, c.height,
                             c.width, p->st));
    d16 = p->F(p->dl_t);
  }
  float* hp = p->F(p->head_pk);
  UHIPCK(head_wgrad(p->F(B[8].out), d16, p->DP(p->out_w), p->DP(p->out_b), V0, f, p->K,
                    p->F(p->wg_ws), p->st));
  UHIPCK(head_dgrad(d16, hp + head_pack_dgrad_offset(f, p->K), p->F(p->G_out), V0, f, p->K,
                    p->st, p->cfg.math));
  for (int k = 0; k < NUP; ++k) {  // dec1 <- up1 <- dec2 ... <- up4
    const int bi = 8 - k, ui = 3 - k;
    UBlk& d = B[bi];
    UUp& U = p->up[ui];
    const int C = d.C, lvl = d.lvl;
    Dst2 dx{p->F(p->G_dx), p->F(p->dskip[lvl]), C, C, C};
    UCK(bwd_block(p, d, p->F(p->G_out), &dx,
                  Src2{p->F(U.out), p->F(B[lvl].out), C, C, C}));
    const Vol& low = p->vol[U.lvl_low];
    UHIPCK(upconv_wgrad(p->F(B[bi - 1].out), p->F(p->G_dx), C, p->DP(U.w), p->DP(U.b), low, U.Cin,
                        U.Cout, p->F(p->wg_ws), p->st, NSUB, p->cfg.math));
    float* pk = p->F(U.pk);
    UHIPCK(upconv_dgrad(p->F(p->G_dx), C, pk + upconv_pack_dgrad_offset(U.Cin, U.Cout, NSUB),
                        p->F(p->G_out), low, U.Cin, U.Cout, p->st, NSUB, p->cfg.math));
  }
  {
    Dst2 dx = dst1(p->F(p->G_dx), 8 * f);
    UCK(bwd_block(p, B[4], p->F(p->G_out), &dx, src1(p->F(p->pool[3]), 8 * f)));
  }
  for (int l = 3; l >= 0; --l) {
    const int C = f << l;
    UHIPCK(maxpool3_bwd_add(p->F(p->G_dx), reinterpret_cast<const uint8_t*>(p->ws + p->pidx[l]),
                            p->F(p->dskip[l]), C, p->F(p->dskip[l]), p->vol[l], C, p->st));
    if (l > 0) {
      Dst2 dx = dst1(p->F(p->G_dx), C / 2);
      UCK(bwd_block(p, B[l], p->F(p->dskip[l]), &dx, src1(p->F(p->pool[l - 1]), C / 2)));
    } else {
      UCK(bwd_block(p, B[0], p->F(p->dskip[0]), nullptr, src1(p->F(p->x_cl), p->ldx)));
    }
  }
  return SPFF_OK;
}

}  // namespace

// =================================================================== C ABI ==
extern "C" {

int spff_unet3d_create(const spff_unet3d_cfg* cfg, spff_unet3d** out) {
  if (!cfg || !out) return ufail(SPFF_EINVAL, "null argument");
  spff_unet3d* p = new spff_unet3d();
  p->cfg = *cfg;
  const int r = build(p);
  if (r != SPFF_OK) {
    delete p;
    return r;
  }
  *out = p;
  return SPFF_OK;
}

void spff_unet3d_destroy(spff_unet3d* p) { delete p; }

int spff_unet3d_num_params(const spff_unet3d* p) { return p ? (int)p->params.size() : 0; }

int spff_unet3d_param_info(const spff_unet3d* p, int i, const char** name, int* ndim,
                           int64_t shape[5], int64_t* offset, int64_t* numel) {
  if (!p || i < 0 || i >= (int)p->params.size()) return ufail(SPFF_EINVAL, "param index");
  const UEnt& e = p->params[i];
  if (name) *name = e.name.c_str();
  if (ndim) *ndim = (int)e.shape.size();
  if (shape)
    for (int k = 0; k < 5; ++k) shape[k] = k < (int)e.shape.size() ? e.shape[k] : 1;
  if (offset) *offset = e.off;
  if (numel) *numel = e.numel;
  return SPFF_OK;
}

int64_t spff_unet3d_param_floats(const spff_unet3d* p) { return p ? p->nparam : 0; }
int spff_unet3d_num_buffers(const spff_unet3d* p) { return p ? (int)p->bufs.size() : 0; }

int spff_unet3d_buffer_info(const spff_unet3d* p, int i, const char** name, int64_t* offset,
                            int64_t* numel) {
  if (!p || i < 0 || i >= (int)p->bufs.size()) return ufail(SPFF_EINVAL, "buffer index");
  const UEnt& e = p->bufs[i];
  if (name) *name = e.name.c_str();
  if (offset) *offset = e.off;
  if (numel) *numel = e.numel;
  return SPFF_OK;
}

int64_t spff_unet3d_buffer_floats(const spff_unet3d* p) { return p ? p->nbuf : 0; }
size_t spff_unet3d_workspace_bytes(const spff_unet3d* p) { return p ? p->total : 0; }

int spff_unet3d_forward(spff_unet3d* p, const float* x, const float* params, float* buffers,
                        int training, float* logits, void* ws, void* stream) {
  if (!p || !x || !params || !buffers || !logits || !ws) return ufail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = nullptr;
  p->buf = buffers;
  p->st = static_cast<hipStream_t>(stream);
  p->co.failed = nullptr;
  const int rc = forward(p, x, logits, training != 0);
  if (p->co.failed) return ufail(SPFF_ECOLL, std::string("SyncBN ") + p->co.failed + " failed");
  return rc;
}

int spff_unet3d_set_sync_bn(spff_unet3d* p, const spff_coll* coll, int world) {
  if (!p) return ufail(SPFF_EINVAL, "null plan");
  if (!coll || world <= 1) {
    p->co = Coll{};
    return SPFF_OK;
  }
  if (!coll->allreduce) return ufail(SPFF_EINVAL, "spff_coll needs allreduce");
  p->co = Coll{};
  p->co.world = world;
  p->co.ctx = coll->ctx;
  p->co.allreduce = coll->allreduce;
  p->co.halo = coll->halo;
  return SPFF_OK;
}

int spff_unet3d_backward(spff_unet3d* p, const float* dlogits, const float* params,
                         float* dparams, void* ws, void* stream) {
  if (!p || !dlogits || !params || !dparams || !ws) return ufail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = dparams;
  p->st = static_cast<hipStream_t>(stream);
  p->co.failed = nullptr;
  const int rc = backward(p, dlogits);
  if (p->co.failed) return ufail(SPFF_ECOLL, std::string("SyncBN ") + p->co.failed + " failed");
  return rc;
}

int spff_unet3d_saved_tensor(const spff_unet3d* p, void* ws, const char* name, const float** ptr,
                             int64_t* nv, int* ch) {
  if (!p || !ws || !name || !ptr) return ufail(SPFF_EINVAL, "null argument");
  const char* base = static_cast<const char*>(ws);
  const std::string n(name);
  auto ret = [&](size_t off, const Vol& v, int c) {
    *ptr = reinterpret_cast<const float*>(base + off);
    if (nv) *nv = nvox(v);
    if (ch) *ch = c;
    return SPFF_OK;
  };
  if (n == "x_cl") return ret(p->x_cl, p->vol[0], p->ldx);
  for (int i = 0; i < NBLK; ++i) {
    const UBlk& b = p->blk[i];
    const Vol& v = p->vol[b.lvl];
    if (n == b.name + ".y1") return ret(b.y1, v, b.C);
    if (n == b.name + ".a1") return ret(b.a1, v, b.C);
    if (n == b.name + ".y2") return ret(b.y2, v, b.C);
    if (n == b.name + ".out") return ret(b.out, v, b.C);
  }
  for (int l = 0; l < 4; ++l)
    if (n == "pool" + std::to_string(l + 1)) return ret(p->pool[l], p->vol[l + 1], p->f << l);
  const char* upn[NUP] = {"up4", "up3", "up2", "up1"};
  for (int u = 0; u < NUP; ++u)
    if (n == upn[u]) return ret(p->up[u].out, p->vol[p->up[u].lvl_low - 1], p->up[u].Cout);
  return ufail(SPFF_EINVAL, "unknown saved tensor " + n);
}

int spff_loss_ex(const float* logits, const int64_t* labels, int64_t nv, int K, int ignore,
                 double smooth, const int64_t* count_override, const float* class_weights,
                 int clamp_denominator, float* out4, float* dlogits, int64_t* conf, void* ws,
                 void* stream) {
  if (!logits || !labels || !out4 || !dlogits || !conf || !ws)
    return ufail(SPFF_EINVAL, "null argument");
  if (K < 1 || K > SPFF_MAX_CLASSES)
    return ufail(SPFF_EINVAL, "num_classes must be 1..SPFF_MAX_CLASSES");
  UHIPCK(loss_fwd(logits, labels, nv, K, ignore, smooth, count_override, out4, dlogits, conf,
                  static_cast<float*>(ws), static_cast<hipStream_t>(stream), class_weights,
                  clamp_denominator));
  return SPFF_OK;
}

}  // extern "C"
