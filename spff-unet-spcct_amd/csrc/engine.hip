// SPFF-UNet engine: plan (parameter + workspace layout), forward, backward and
// the C ABI of include/spff.h.
//
// Graph (reference UNet3D_SpectralCore.forward, models.py:693-701):
//   e1 = post0(enc1(x)); e2 = post1(enc2(pool(e1))); e3 = post2(enc3(pool(e2)))
//   b  = post3(bott(pool(e3)))
//   d3 = dec3([up3(b) | e3]); d2 = dec2([up2(d3) | e2]); d1 = dec1([up1(d2) | e1])
//   logits = out(d1)
// Block (models.py:1473-1478 + _post 684-685):
//   y1 = conv(x); a1 = lrelu(IN(y1)); y2 = conv(a1); out = lrelu(IN(y2))*P + Q
// with the gate algebra (EFiLM, FourierGate, SpectralSE, SE) folded into the
// per-(b,c,d) coefficients P, Q (gates.hip).  Saved for backward: y1, a1, y2,
// out and the (b,c)/(b,c,d) statistics -- everything else is recomputed.
#include "spff_internal.h"

#ifndef SPFF_OUTFUSE
// block outputs applied by the GEMMs that read them (ActRows) instead of a stored act_apply
// pass: 1 = dec1's, read by the head (forward GEMM + streaming weight gradient); 2 = also the
// bottleneck's and dec3 / dec2's, read by the up-convs; 0 = none.  Measured (round 3, one
// box, profiles/r03/ab/outfuse_kstats.txt): the up-conv loaders pay 5 loads per A float4 and
// the transform's VALU in kernels that are VALU-issue-bound already -- k_atb_x 0.64 -> 1.07,
// the up-conv forward 0.47 -> 0.69 ms/step against 0.16 ms/step of act_apply saved; the
// head's loaders +0.14 ms/step against dec1's 0.2 ms/step level-0 pass
#define SPFF_OUTFUSE 1
#endif
#ifndef SPFF_POOL_FOLD
// 1: the encoder blocks' output gradients (skip + MaxPool backward) are formed by their two
// readers (PoolAdd: the tail reduction, the IN-backward apply) instead of k_maxpool_bwd_add
#define SPFF_POOL_FOLD 1
#endif
#ifndef SPFF_RED_FUSE
#define SPFF_RED_FUSE 1  // 0 (A/B diagnostics): separate tail and IN-backward reductions
#endif
#include "spff.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace spff;


static thread_local std::string g_err;
static int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
namespace spff {
int set_error(int code, const char* msg) { return fail(code, msg); }
}
#define HIPCK(expr)                                                                        \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(SPFF_EHIP, std::string(#expr) + " -> " + hipGetErrorString(_e));         \
  } while (0)
// PROF: time one launch with HIP events on the plan's stream when enabled.
// PROFB also records the launch's compulsory HBM bytes (operands read once, result
// written once) for the roofline's traffic comparison.
#define PROF(P, CLS, FLOPS, expr) PROFB(P, CLS, FLOPS, 0.0, expr)
#define PROFB(P, CLS, FLOPS, BYTES, expr)                                                \
  do {                                                                                   \
    spff_plan* _p = (P);                                                                 \
    spff_plan::ProfRec* _r = _p->prof_on ? prof_slot(_p, (CLS), (FLOPS), (BYTES)) : nullptr; \
    if (_r) HIPCK(hipEventRecord(_r->a, _p->st));                                        \
    HIPCK(expr);                                                                         \
    if (_r) HIPCK(hipEventRecord(_r->b, _p->st));                                        \
  } while (0)
#define CK(expr)               \
  do {                         \
    int _r = (expr);           \
    if (_r != SPFF_OK) return _r; \
  } while (0)

namespace {

static inline int rup(int a, int b) { return (a + b - 1) / b * b; }

struct PEnt {
  std::string name;
  std::vector<int64_t> shape;
  int64_t off, numel;
};

struct ConvL {
  int Cin, Cout;
  int64_t w;
  int kpad_f, npad_f, kpad_d, npad_d;
};

struct Blk {
  std::string name;
  int lvl, Cin, C;
  bool novel, efilm, fgate, post_se, post_spec;
  ConvL c1, c2;
  int64_t g1 = -1, b1 = -1, g2 = -1, b2 = -1;
  int64_t fw0 = -1, fb0 = -1, fw2 = -1, fb2 = -1;
  int64_t mag = -1, mask = -1;
  int64_t sw0 = -1, sb0 = -1, sw2 = -1, sb2 = -1;
  int64_t pr0 = 0, pr1 = 0, se0 = 0, se1 = 0;  // flat ranges of the block's / SE parameters
  size_t y1, a1, y2, out;
  size_t mean1, rstd1, al1, de1, mean2, rstd2, al2, de2;
  size_t Sa, t, bt, hid, s1, g1s, sg2, p, h, e, P, Q;
  size_t spec = 0;  // sharded plans: full-depth s1 spectrum [B][L][2] (fp64)
  bool fa = false;  // conv2 reads y1 through the IN affine (a1 never stored)
  bool fout = false;  // out never stored: its GEMM consumers apply it to y2 (ActRows)
  size_t pk[4] = {0, 0, 0, 0};  // batched conv images: c1 fwd, c2 fwd, c2 dgrad, c1 dgrad
  size_t PT = 0, QT = 0;  // fout + gates: P, Q as [B][D][C]
  bool tail() const { return efilm || fgate || post_se || post_spec; }
};

struct UpL {
  int Cin, Cout, lvl_low;
  int64_t w, b;
  size_t pk, out;
  // _cat trilinear fallback (models.py:687-691): 2 x the low level's H / W differs from
  // the skip's (odd extents floor in the pools).  raw = the up-conv output at 2H x 2W
  // (resized into out); in the backward it holds the resized-back gradient.
  bool rs = false;
  size_t raw = 0;
};

}  // namespace

struct spff_plan {
  spff_cfg cfg;
  Vol vol[4];
  int f, KD, ldx, K;
  int efh = 32, efp = 16, fphase = 0;  // EnergyFiLM3D(hidden, pe_dims), learn_phase
  bool lean = false;  // SPFF_MEM_LEAN layout: a1 / out / up-conv outputs live in the
                      // gradient scratch and are recomputed in the backward
  std::vector<PEnt> params;
  int64_t nparam = 0;
  Blk blk[7];
  UpL up[3];  // up3, up2, up1
  int64_t out_w = -1, out_b = -1;
  size_t head_pk = 0;
  size_t x_cl = 0, pool[3] = {0, 0, 0}, pidx[3] = {0, 0, 0};
  size_t red_ws = 0, red_out = 0, red_out4 = 0, gscr = 0, Abuf = 0, Bbuf = 0, kk1 = 0, kk2 = 0,
         wg_ws = 0, wt = 0, cst = 0;
  bool pkb = false;  // conv images packed in one batch at the forward start (b.pk)
  size_t wcur = 0;   // the image the next conv3d_run reads (b.pk[k] or the scratch wt)
  size_t fsl = 0;  // SPFF_MATH_F16X3 operand maxima, 8 slots per block (f16_slot), then
                   // two per-launch slots of the sharded plans' weight gradients
  size_t G_out = 0, G_dy2 = 0, G_da1 = 0, G_dx = 0, dskip[3] = {0, 0, 0};
  size_t part_d = 0;  // sharded plans: fp64 IN partials [B][C][2]
  // height-sharded plans (spff_cfg.shard_axis = SPFF_SHARD_HEIGHT, hshard.hip): the
  // boundary-row staging slab (the convs read the neighbours' rows in place) and the gate
  // parameter gradients of ranks other than 0 (the gates are evaluated replicated)
  bool hsh = false;
  int hmul = 1;  // global / local rows
  size_t hst = 0, gdum = 0;
  size_t total = 0;
  Coll co;             // sharding group (world 1: unsharded)
  bool coll_set = false;
  spff_grad_ready_fn grad_fn = nullptr;  // data-parallel gradient-ready hook
  void* grad_ctx = nullptr;
  float* pe_dev = nullptr;
  std::vector<float> pe_host;
  // optional HIP-event timing of the MFMA kernels (bench.py roofline)
  struct ProfRec { hipEvent_t a, b; int cls; double flops, bytes; };
  std::vector<ProfRec> prof;
  size_t prof_n = 0;
  bool prof_on = false;
  int dbg_stop = -1;  // debug: stop backward after this many blocks (-1 = off)
  bool efilm_ready = false;  // this forward's EFiLM coefficients are computed (all blocks)
  bool keep_out = false;  // debug: store the fused block outputs too (saved views)
  bool pool_fold = SPFF_POOL_FOLD;  // PoolAdd in the encoder backward (debug key 2: off)
  bool bst_fuse = true;  // conv1's IN-backward sums in the dgrad epilogue (debug key 3: off)
  // per call
  char* ws = nullptr;
  const float* prm = nullptr;
  float* dprm = nullptr;
  hipStream_t st = nullptr;
  // depth-sharded plans: side stream + events of the halo exchange that overlaps the
  // interior depth tiles of the next convolution (conv_halo)
  hipStream_t st2 = nullptr;
  hipEvent_t ev_in = nullptr, ev_halo = nullptr;
  // the conv input whose halo exchange halo_begin already put on st2 (ev_halo marks it)
  const float* halo_early = nullptr;

  float* F(size_t off) const { return reinterpret_cast<float*>(ws + off); }
  const float* P(int64_t off) const { return off < 0 ? nullptr : prm + off; }
  float* DP(int64_t off) const { return off < 0 ? nullptr : dprm + off; }
  size_t alloc(size_t bytes) {
    size_t o = total;
    total += (bytes + 255) / 256 * 256;
    return o;
  }
  // a conv input of a halo'd (depth-sharded) plan: one neighbour slice of up to
  // slice_bytes before and after the interior; returns the interior offset
  size_t alloc_halo(size_t bytes, size_t slice_bytes) {
    if (!vol[0].dh) return alloc(bytes);
    return alloc(bytes + 2 * slice_bytes) + slice_bytes;
  }
  double* D64(size_t off) const { return reinterpret_cast<double*>(ws + off); }
  int64_t reg(const std::string& name, std::vector<int64_t> shape) {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    params.push_back(PEnt{name, shape, nparam, n});
    int64_t o = nparam;
    nparam += n;
    return o;
  }
};

// compulsory HBM bytes of one conv launch: both activations once + the fp32 weights
static double cbytes(double V, int Cin, int Cout, int T) {
  return 4.0 * (V * Cin + V * Cout + (double)T * Cin * Cout);
}

constexpr int F16_SHARD_SLOTS = 7 * 8;

static spff_plan::ProfRec* prof_slot(spff_plan* p, int cls, double flops, double bytes) {
  if (p->prof_n == p->prof.size()) {
    spff_plan::ProfRec r;
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return nullptr;
    p->prof.push_back(r);
  }
  spff_plan::ProfRec* r = &p->prof[p->prof_n++];
  r->cls = cls;
  r->flops = flops;
  r->bytes = bytes;
  return r;
}

namespace {

void reg_block(spff_plan* p, Blk& b) {
  const std::string a = b.novel ? "pre" : "b1", bb = b.novel ? "body" : "b2";
  const int KD = p->KD, C = b.C;
  b.pr0 = p->nparam;
  b.c1.w = p->reg(b.name + "." + a + ".0.weight", {C, b.Cin, KD, 3, 3});
  b.g1 = p->reg(b.name + "." + a + ".1.weight", {C});
  b.b1 = p->reg(b.name + "." + a + ".1.bias", {C});
  b.c2.w = p->reg(b.name + "." + bb + ".0.weight", {C, C, KD, 3, 3});
  b.g2 = p->reg(b.name + "." + bb + ".1.weight", {C});
  b.b2 = p->reg(b.name + "." + bb + ".1.bias", {C});
  if (b.efilm) {
    b.fw0 = p->reg(b.name + ".efilm.mlp.0.weight", {p->efh, p->efp, 1});
    b.fb0 = p->reg(b.name + ".efilm.mlp.0.bias", {p->efh});
    b.fw2 = p->reg(b.name + ".efilm.mlp.2.weight", {2 * C, p->efh, 1});
    b.fb2 = p->reg(b.name + ".efilm.mlp.2.bias", {2 * C});
  }
  if (b.fgate) {
    b.mag = p->reg(b.name + ".fgate.mag_scale", {1});
    b.mask = p->reg(b.name + ".fgate.freq_mask", {1, 1, p->co.D_glob / 2 + 1, 1, 1});
  }
  b.pr1 = p->nparam;
}

void conv_dims(ConvL& c, int Cin, int Cout) {
  c.Cin = Cin;
  c.Cout = Cout;
  c.kpad_f = rup(Cin, 8);
  c.npad_f = rup(Cout, conv3d_bn(Cout));
  c.kpad_d = rup(Cout, 8);
  c.npad_d = rup(Cin, conv3d_bn(Cin));
}

size_t conv_pack_bytes(const ConvL& c, int KD) { return conv3d_pack_bytes(KD, c.Cin, c.Cout); }

void host_pe(int D, int P, std::vector<float>& pe) {
  // models.py:1495-1503 in fp32: h = max(1, P / 2) frequencies, denom = exp(i * (-ln(1e4)/h)),
  // pe = [sin(pos*denom); cos(pos*denom)] (2 h rows), and a zero row when that is < P (odd P)
  const int h = std::max(1, P / 2);
  pe.assign((size_t)P * D, 0.f);
  const float cst = (float)(-std::log(10000.0) / (double)h);
  for (int i = 0; i < h; ++i) {
    const float denom = std::exp((float)i * cst);
    for (int d = 0; d < D; ++d) {
      const float arg = (float)d * denom;
      if (i < P) pe[(size_t)i * D + d] = std::sin(arg);
      if (h + i < P) pe[(size_t)(h + i) * D + d] = std::cos(arg);
    }
  }
}

int build_plan(spff_plan* p) {
  const spff_cfg& c = p->cfg;
  if (c.batch < 1 || c.in_ch < 1 || c.depth < 1 || c.num_classes < 1 ||
      c.num_classes > SPFF_MAX_CLASSES)
    return fail(SPFF_EINVAL, "invalid batch/in_ch/depth/num_classes (K must be 1..SPFF_MAX_CLASSES)");
  if (c.base < 8 || c.base % 8)
    return fail(SPFF_EINVAL, "base must be a multiple of 8");
  if (c.ksd != 1 && c.ksd != 3) return fail(SPFF_EINVAL, "ksd must be 1 or 3");
  if (c.height < 8 || c.width < 8)
    return fail(SPFF_ESHAPE, "H and W must be >= 8 (three (1,2,2) pools)");
  if (c.in_ch > 1024) return fail(SPFF_EINVAL, "in_ch > 1024 not supported");
  if (c.math < SPFF_MATH_F32 || c.math > SPFF_MATH_F16X3)
    return fail(SPFF_EINVAL, "math must be one of SPFF_MATH_*");
  if (c.memory_mode < SPFF_MEM_AUTO || c.memory_mode > SPFF_MEM_LEAN)
    return fail(SPFF_EINVAL, "memory_mode must be one of SPFF_MEM_*");
  p->efh = c.efilm_hidden > 0 ? c.efilm_hidden : 32;
  p->efp = c.efilm_pe_dims > 0 ? c.efilm_pe_dims : 16;
  p->fphase = c.fgate_learn_phase != 0;
  // (pe_dims 1 would give the reference a 2-row code for a 1-channel Conv1d: it raises)
  if (c.efilm_hidden < 0 || c.efilm_pe_dims < 0 || p->efh > EFH_MAX || p->efp < 2 ||
      p->efp > EFP_MAX)
    return fail(SPFF_EINVAL, "efilm_hidden must be 1..64 and efilm_pe_dims 2..32 (0: 32, 16)");
  p->lean = c.memory_mode == SPFF_MEM_LEAN ||
            (c.memory_mode == SPFF_MEM_AUTO &&
             (int64_t)c.batch * c.depth * c.height * c.width >= (int64_t(1) << 26));
  const int world = c.shard_world > 1 ? c.shard_world : 1;
  const bool hsh = world > 1 && c.shard_axis == SPFF_SHARD_HEIGHT;
  if (world > 1) {
    if (c.shard_axis != SPFF_SHARD_DEPTH && c.shard_axis != SPFF_SHARD_HEIGHT)
      return fail(SPFF_EINVAL, "shard_axis must be SPFF_SHARD_DEPTH or SPFF_SHARD_HEIGHT");
    if (!hsh && c.batch != 1) return fail(SPFF_EINVAL, "depth-sharded plans take batch == 1");
    if (hsh && (c.height % 8 || c.width % 8))
      return fail(SPFF_ESHAPE, "height-sharded plans take local height and width multiples of 8");
    if (c.shard_rank < 0 || c.shard_rank >= world) return fail(SPFF_EINVAL, "bad shard_rank");
  }
  p->hsh = hsh;
  p->hmul = hsh ? world : 1;
  p->co.world = world;
  p->co.rank = world > 1 ? c.shard_rank : 0;
  p->co.D_glob = hsh ? c.depth : c.depth * world;
  p->co.d_off = hsh ? 0 : p->co.rank * c.depth;
  p->f = c.base;
  p->KD = c.ksd;
  p->K = c.num_classes;
  p->ldx = rup(c.in_ch, 8);
  const int dh = (world > 1 && !hsh && c.ksd == 3) ? 1 : 0;
  for (int l = 0; l < 4; ++l) {
    p->vol[l] = Vol{c.batch, c.depth, c.height >> l, c.width >> l};
    p->vol[l].dh = dh;
  }
  const int f = p->f;
  const char* names[7] = {"enc1", "enc2", "enc3", "bott", "dec3", "dec2", "dec1"};
  const int lvl[7] = {0, 1, 2, 3, 2, 1, 0};
  const int cin[7] = {c.in_ch, f, 2 * f, 4 * f, 8 * f, 4 * f, 2 * f};
  const int cc[7] = {f, 2 * f, 4 * f, 8 * f, 4 * f, 2 * f, f};
  for (int i = 0; i < 7; ++i) {
    Blk& b = p->blk[i];
    b.name = names[i];
    b.lvl = lvl[i];
    b.Cin = cin[i];
    b.C = cc[i];
    b.efilm = c.use_efilm != 0;
    b.fgate = c.use_fgate != 0;
    b.novel = b.efilm || b.fgate;
    b.post_se = i < 4 && c.use_se;
    b.post_spec = i < 4 && c.use_specse;
    b.fa = conv3d_fuses_act(c.math, b.C);
    // the bottleneck and decoder outputs feed only the up-convs and the head (GEMMs)
    b.fout = (SPFF_OUTFUSE >= 2 ? i >= 3 : SPFF_OUTFUSE == 1 && i == 6) && !p->lean &&
             b.C % 4 == 0;
    conv_dims(b.c1, b.Cin, b.C);
    conv_dims(b.c2, b.C, b.C);
  }
  // parameter registration in reference state-dict order (models.py:655-681)
  reg_block(p, p->blk[0]);
  reg_block(p, p->blk[1]);
  reg_block(p, p->blk[2]);
  reg_block(p, p->blk[3]);
  const int upc[3][3] = {{8 * f, 4 * f, 2}, {4 * f, 2 * f, 1}, {2 * f, f, 0}};
  const char* upn[3] = {"up3", "up2", "up1"};
  for (int u = 0; u < 3; ++u) {
    UpL& U = p->up[u];
    U.Cin = upc[u][0];
    U.Cout = upc[u][1];
    U.lvl_low = upc[u][2] + 1;
    const Vol& vl = p->vol[U.lvl_low];
    const Vol& vh = p->vol[U.lvl_low - 1];
    U.rs = 2 * vl.H != vh.H || 2 * vl.W != vh.W;
    U.w = p->reg(std::string(upn[u]) + ".weight", {U.Cin, U.Cout, 1, 2, 2});
    U.b = p->reg(std::string(upn[u]) + ".bias", {U.Cout});
    reg_block(p, p->blk[4 + u]);
  }
  p->out_w = p->reg("out.weight", {p->K, f, 1, 1, 1});
  p->out_b = p->reg("out.bias", {p->K});
  if (c.use_se) {
    const int chs[4] = {f, 2 * f, 4 * f, 8 * f};
    for (int i = 0; i < 4; ++i) {
      const int C = chs[i], h = se_hidden(C);
      const std::string pre = "se." + std::to_string(i) + ".fc.";
      Blk& b = p->blk[i];
      b.se0 = p->nparam;
      b.sw0 = p->reg(pre + "0.weight", {h, C, 1, 1, 1});
      b.sb0 = p->reg(pre + "0.bias", {h});
      b.sw2 = p->reg(pre + "2.weight", {C, h, 1, 1, 1});
      b.sb2 = p->reg(pre + "2.bias", {C});
      b.se1 = p->nparam;
    }
  }

  // ---- workspace layout ----
  const int B = c.batch, D = c.depth;
  const Vol& v0 = p->vol[0];
  const auto slice = [&](const Vol& v, int C) { return (size_t)v.H * v.W * C * sizeof(float); };
  p->x_cl = p->alloc_halo(nvox(v0) * p->ldx * sizeof(float), slice(v0, p->ldx));
  size_t red_ws = 0, red_out = 0, red_out4 = 0, gs = 0, bcd = 0, wg = 0, wt = 0, cst = 0;
  size_t hst = 0, gd = 0;
  for (int i = 0; i < 7; ++i) {
    Blk& b = p->blk[i];
    const Vol& v = p->vol[b.lvl];
    const size_t act = nvox(v) * b.C * sizeof(float);
    // with the fused input activation conv2 reads y1 (halo'd when sharded), not a1
    b.y1 = b.fa ? p->alloc_halo(act, slice(v, b.C)) : p->alloc(act);
    b.y2 = p->alloc(act);
    if (!p->lean) {
      if (!b.fa) b.a1 = p->alloc_halo(act, slice(v, b.C));
      b.out = p->alloc_halo(act, slice(v, b.C));
    } else if (i == 3) {
      b.out = p->alloc(act);  // the bottleneck output (up3's input) is kept: 1/64 size
    }
    const size_t bc = (size_t)B * b.C * sizeof(float);
    b.mean1 = p->alloc(bc); b.rstd1 = p->alloc(bc); b.al1 = p->alloc(bc); b.de1 = p->alloc(bc);
    b.mean2 = p->alloc(bc); b.rstd2 = p->alloc(bc); b.al2 = p->alloc(bc); b.de2 = p->alloc(bc);
    const size_t bcdz = (size_t)B * b.C * D * sizeof(float);
    if (b.tail()) {
      b.Sa = p->alloc(bcdz);
      b.P = p->alloc(bcdz);
      b.Q = p->alloc(bcdz);
      if (b.fout) {
        b.PT = p->alloc(bcdz);
        b.QT = p->alloc(bcdz);
      }
      b.s1 = p->alloc((size_t)B * D * 4);
      b.g1s = p->alloc((size_t)B * D * 4);
      b.sg2 = p->alloc((size_t)B * D * 4);
      b.p = p->alloc(bc);
      b.e = p->alloc(bc);
      b.h = p->alloc((size_t)B * se_hidden(b.C) * 4);
      b.t = p->alloc((size_t)b.C * D * 4);
      b.bt = p->alloc((size_t)b.C * D * 4);
      b.hid = p->alloc((size_t)p->efh * D * 4);
      if (world > 1 && !hsh)
        b.spec = p->alloc((size_t)B * (p->co.D_glob / 2 + 1) * 2 * sizeof(double));
    }
    red_ws = std::max(red_ws, slab_reduce_ws_bytes(v, b.C, b.tail() && SPFF_RED_FUSE ? 6 : 2));
    red_out = std::max(red_out, (size_t)B * b.C * D * 2 * sizeof(float));
    if (b.tail() && SPFF_RED_FUSE)
      red_out4 = std::max(red_out4, (size_t)B * b.C * D * 4 * sizeof(float));
    gs = std::max(gs, world > 1 && !hsh ? gates_sh_scratch_bytes(v, b.C, p->co.D_glob)
                                        : gates_scratch_bytes(v, b.C));
    if (hsh) {  // the boundary-row staging slab of the widest conv input at this level
      hst = std::max(hst, hstage_floats(v, hrows_ld(std::max(b.Cin, b.C))));
      gd = std::max(gd, (size_t)(b.pr1 - (b.b2 + b.C)) + (size_t)(b.se1 - b.se0));
    }
    bcd = std::max(bcd, bcdz);
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, p->KD, b.Cin, b.C));
    wg = std::max(wg, conv3d_wgrad_ws_bytes(v, p->KD, b.C, b.C));
    wg = std::max(wg, conv3d_splitk_bytes(v, p->KD, b.Cin, b.C));
    wg = std::max(wg, conv3d_splitk_bytes(v, p->KD, b.C, b.C));
    wt = std::max(wt, conv_pack_bytes(b.c1, p->KD));
    wt = std::max(wt, conv_pack_bytes(b.c2, p->KD));
    cst = std::max(cst, conv3d_stats_bytes(v, p->KD, b.Cin, b.C));
    cst = std::max(cst, conv3d_stats_bytes(v, p->KD, b.C, b.C));
  }
  for (int l = 0; l < 3; ++l) {
    const Vol& vl = p->vol[l + 1];
    const int C = f << l;  // channels of e_{l+1} pooled
    p->pool[l] = p->alloc_halo(nvox(vl) * C * sizeof(float), slice(vl, C));
    p->pidx[l] = p->alloc(nvox(vl) * C);
  }
  for (int u = 0; u < 3; ++u) {
    UpL& U = p->up[u];
    const Vol& vh = p->vol[U.lvl_low - 1];
    if (!p->lean) U.out = p->alloc_halo(nvox(vh) * U.Cout * sizeof(float), slice(vh, U.Cout));
    U.pk = p->alloc(upconv_pack_floats(U.Cin, U.Cout) * sizeof(float));
    if (U.rs) U.raw = p->alloc(nvox(p->vol[U.lvl_low]) * 4 * U.Cout * sizeof(float));
    wg = std::max(wg, upconv_wgrad_ws_bytes(p->vol[U.lvl_low], U.Cin, U.Cout));
  }
  p->head_pk = p->alloc(head_pack_floats(f, p->K) * sizeof(float));
  wg = std::max(wg, head_wgrad_ws_bytes(nvox(v0), f, p->K));
  p->red_ws = p->alloc(red_ws);
  p->red_out = p->alloc(red_out);
  p->red_out4 = p->alloc(red_out4);
  p->gscr = p->alloc(gs);
  p->Abuf = p->alloc(bcd);
  p->Bbuf = p->alloc(bcd);
  p->kk1 = p->alloc((size_t)B * 8 * f * sizeof(float));
  p->kk2 = p->alloc((size_t)B * 8 * f * sizeof(float));
  p->wg_ws = p->alloc(wg);
  // (the lean layout keeps the one scratch image: it trades time for the smallest footprint)
  p->pkb = !p->lean && conv3d_packs_batched(p->cfg.math);
  if (p->pkb) {
    for (int i = 0; i < 7; ++i) {
      Blk& b = p->blk[i];
      b.pk[0] = p->alloc(conv_pack_bytes(b.c1, p->KD));
      b.pk[1] = p->alloc(conv_pack_bytes(b.c2, p->KD));
      b.pk[2] = p->alloc(conv_pack_bytes(b.c2, p->KD));
      if (i > 0) b.pk[3] = p->alloc(conv_pack_bytes(b.c1, p->KD));  // enc1's input: no dx
    }
  } else {
    p->wt = p->alloc(wt);
  }
  p->fsl = p->alloc((F16_SHARD_SLOTS + 2) * sizeof(unsigned));
  p->cst = p->alloc(cst);
  // gradient scratch, sized for level 0 ([V0][f]); a level-l tensor of the path
  // (V0 / 4^l voxels x f 2^l channels) fills 1 / 2^l of a buffer.  Halo'd (level-0
  // slice = the largest) so any of them can hold a conv input.
  const size_t gbytes = nvox(v0) * f * sizeof(float);
  p->G_out = p->alloc_halo(gbytes, slice(v0, f));
  p->G_dy2 = p->alloc_halo(gbytes, slice(v0, f));
  p->G_da1 = p->alloc_halo(gbytes, slice(v0, f));
  p->G_dx = p->alloc_halo(gbytes, slice(v0, f));
  // skip gradients: dskip0 needs a level-0 buffer of its own; dskip1 (alive from
  // dec2's input gradient to enc2's backward) and dskip2 (dec3 -> enc3) sit in the
  // upper halves of G_dx / G_out, which only level-0 tensors reach (dec1, before)
  p->dskip[0] = p->alloc(gbytes);
  p->dskip[1] = p->G_dx + gbytes / 2;
  p->dskip[2] = p->G_out + gbytes / 2;
  if (p->lean) {
    // forward placement of the unsaved tensors (lifetimes in DESIGN.md §2):
    //   enc1 a1/out -> G_da1 (out alive until dec1's first conv)
    //   enc2 a1/out -> G_dy2 [lower half]     enc3 a1/out -> G_out [lower quarter]
    //   bott a1, dec3 a1, dec2 a1, up3/up2/up1 outputs -> G_dx (each dead before the next)
    //   dec3 out -> G_dy2 upper half (enc2's output still alive below it)
    //   dec2 out -> G_dy2 (enc2's output dead)   dec1 a1 -> G_da1   dec1 out -> G_out
    Blk* B = p->blk;
    B[0].a1 = B[0].out = p->G_da1;
    B[1].a1 = B[1].out = p->G_dy2;
    B[2].a1 = B[2].out = p->G_out;
    B[3].a1 = p->G_dx;
    B[4].a1 = p->G_dx; B[4].out = p->G_dy2 + gbytes / 2;
    B[5].a1 = p->G_dx; B[5].out = p->G_dy2;
    B[6].a1 = p->G_da1; B[6].out = p->G_out;
    for (int u = 0; u < 3; ++u) p->up[u].out = p->G_dx;
  }
  if (world > 1) p->part_d = p->alloc((size_t)B * 8 * f * 2 * sizeof(double));
  if (hsh) {
    p->hst = p->alloc(hst * sizeof(float));
    p->gdum = p->alloc(std::max<size_t>(gd, 1) * sizeof(float));
  }

  if (c.use_efilm && efilm_fwd_lds(p->efh, p->efp, c.depth) > 160 * 1024)
    return fail(SPFF_EINVAL, "(efilm_hidden + efilm_pe_dims) x depth x 4 B exceeds 160 KiB of LDS");
  host_pe(p->co.D_glob, p->efp, p->pe_host);  // global depths; a slab reads columns d_off + d  // uploaded on the first forward (plan creation needs no GPU)
  return SPFF_OK;
}

int ensure_pe(spff_plan* p) {
  if (p->pe_dev) return SPFF_OK;
  HIPCK(hipMalloc(&p->pe_dev, p->pe_host.size() * sizeof(float)));
  HIPCK(hipMemcpy(p->pe_dev, p->pe_host.data(), p->pe_host.size() * sizeof(float),
                  hipMemcpyHostToDevice));
  return SPFF_OK;
}

GateParams gate_params(const spff_plan* p, const Blk& b) {
  GateParams g;
  g.pe = p->pe_dev;
  g.pe_pitch = p->co.D_glob;
  g.d_off = p->co.d_off;
  g.efh = p->efh;
  g.efp = p->efp;
  g.fphase = p->fphase;
  g.fw0 = b.efilm ? p->P(b.fw0) : nullptr;
  g.fb0 = b.efilm ? p->P(b.fb0) : nullptr;
  g.fw2 = b.efilm ? p->P(b.fw2) : nullptr;
  g.fb2 = b.efilm ? p->P(b.fb2) : nullptr;
  g.mask = b.fgate ? p->P(b.mask) : nullptr;
  g.mag = b.fgate ? p->P(b.mag) : nullptr;
  g.sw0 = b.post_se ? p->P(b.sw0) : nullptr;
  g.sb0 = b.post_se ? p->P(b.sb0) : nullptr;
  g.sw2 = b.post_se ? p->P(b.sw2) : nullptr;
  g.sb2 = b.post_se ? p->P(b.sb2) : nullptr;
  g.specse = b.post_spec ? 1 : 0;
  g.efilm_ready = p->efilm_ready;
  return g;
}

GateSaved gate_saved(const spff_plan* p, const Blk& b) {
  GateSaved s;
  s.t = p->F(b.t); s.bt = p->F(b.bt); s.hid = p->F(b.hid);
  s.s1 = p->F(b.s1); s.g1 = p->F(b.g1s); s.sg2 = p->F(b.sg2);
  s.p = p->F(b.p); s.h = p->F(b.h); s.e = p->F(b.e);
  s.P = p->F(b.P); s.Q = p->F(b.Q);
  s.PT = b.fout ? p->F(b.PT) : nullptr;
  s.QT = b.fout ? p->F(b.QT) : nullptr;
  s.spec = p->co.on() ? p->D64(b.spec) : nullptr;
  return s;
}

// the rows of block b's output as its GEMM consumers apply them (b.fout)
ActRows act_rows(const spff_plan* p, const Blk& b) {
  const Vol& v = p->vol[b.lvl];
  ActRows a;
  a.y = p->F(b.y2);
  a.al = p->F(b.al2);
  a.de = p->F(b.de2);
  a.PT = b.tail() ? p->F(b.PT) : nullptr;
  a.QT = b.tail() ? p->F(b.QT) : nullptr;
  a.D = v.D;
  a.HW = v.H * v.W;
  return a;
}

// one D-slice halo per side for a conv input of a depth-sharded plan (no-op otherwise)
int halo(spff_plan* p, const float* interior, const Vol& v, int C, hipStream_t st = nullptr) {
  if (!v.dh) return SPFF_OK;
  if (!st) st = p->st;
  const int64_t sl = (int64_t)v.H * v.W * C;
  float* in = const_cast<float*>(interior);
  if (p->co.rank == 0) HIPCK(spff::zero_async(in - sl, sl * sizeof(float), st));
  if (p->co.rank == p->co.world - 1)
    HIPCK(spff::zero_async(in + v.D * sl, sl * sizeof(float), st));
  if (p->co.do_halo(in, sl, v.D, st) != 0) return fail(SPFF_ECOLL, "halo exchange failed");
  return SPFF_OK;
}
int halo_src(spff_plan* p, const Src2& x, const Vol& v, hipStream_t st = nullptr) {
  CK(halo(p, x.p0, v, x.ld0, st));
  if (x.p1 != x.p0) CK(halo(p, x.p1, v, x.ld1, st));
  return SPFF_OK;
}
// ---- height-sharded plans (hshard.hip): the convs read the neighbours' rows in place ----
// x's boundary rows 0 and H - 1 -> the neighbours, theirs -> the staging slab's recv
// slices; *xr = x reading them as its stencil rows -1 / H (zero at the global ends).
// On stream st (the side stream when the exchange overlaps a conv's interior tiles).
int hrows_exchange(spff_plan* p, const Src2& x, const Vol& v, int cin, Src2* xr,
                   hipStream_t st) {
  const int ldr = hrows_ld(cin);
  float* stg = p->F(p->hst);
  const int64_t S = (int64_t)v.B * v.D * v.W * ldr;
  HIPCK(hrows_pack(x, cin, stg + S, v, ldr, st));
  if (p->co.do_halo(stg + S, S, 2, st) != 0) return fail(SPFF_ECOLL, "row halo exchange failed");
  *xr = x;
  xr->rlo = p->co.rank > 0 ? stg : nullptr;
  xr->rhi = p->co.rank < p->co.world - 1 ? stg + 3 * S : nullptr;
  xr->ldr = ldr;
  return SPFF_OK;
}
// the side stream st2 and its events (created at the first overlapped exchange)
int side_stream(spff_plan* p) {
  if (p->st2) return SPFF_OK;
  HIPCK(hipStreamCreateWithFlags(&p->st2, hipStreamNonBlocking));
  HIPCK(hipEventCreateWithFlags(&p->ev_in, hipEventDisableTiming));
  HIPCK(hipEventCreateWithFlags(&p->ev_halo, hipEventDisableTiming));
  return SPFF_OK;
}
// a height-sharded 3x3x3 conv: the row exchange on the side stream st2 beside the H tiles
// that read no boundary row, then the first and last H tiles (conv3d_splits_height); else
// exchange, then convolve.  The ranks at both global ends still exchange (their single
// neighbour), so every rank runs the same collective sequence.
int conv_h(spff_plan* p, int cls, double flops, double bytes, const Src2& x, const Dst2& y,
           const Vol& v, int Cin_w, int Cout_w, bool dgrad, const unsigned* wmax) {
  const int cin = dgrad ? Cout_w : Cin_w, KD = p->KD, math = p->cfg.math;
  Src2 xr;
  const bool ovl = conv3d_splits_height(v, KD, Cin_w, Cout_w, dgrad, math);
  if (!ovl) {
    CK(hrows_exchange(p, x, v, cin, &xr, p->st));
    PROFB(p, cls, flops, bytes,
          conv3d_run(xr, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st,
                     p->F(p->wg_ws), nullptr, 0, wmax));
    return SPFF_OK;
  }
  CK(side_stream(p));
  HIPCK(hipEventRecord(p->ev_in, p->st));  // x is final (and the previous conv is done
  HIPCK(hipStreamWaitEvent(p->st2, p->ev_in, 0));  //   reading the staging slab)
  CK(hrows_exchange(p, x, v, cin, &xr, p->st2));
  HIPCK(hipEventRecord(p->ev_halo, p->st2));
  PROFB(p, cls, flops, bytes,
        conv3d_run(xr, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st,
                   p->F(p->wg_ws), nullptr, 3, wmax));
  HIPCK(hipStreamWaitEvent(p->st, p->ev_halo, 0));
  PROFB(p, cls, 0.0, 0.0,
        conv3d_run(xr, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st,
                   p->F(p->wg_ws), nullptr, 4, wmax));
  return SPFF_OK;
}
// weight gradient of a 3x3x3 conv (height-sharded: x's stencil rows from the neighbours;
// dy is read at the local rows only)
int conv_wgrad(spff_plan* p, double flops, double bytes, const Src2& x, const float* dy, float* dw,
               const Vol& v, int Cin, int Cout, const unsigned* xmax = nullptr,
               const unsigned* ymax = nullptr) {
  Src2 xr = x;
  if (p->hsh) CK(hrows_exchange(p, x, v, Cin, &xr, p->st));
  if (p->cfg.math == SPFF_MATH_F16X3 && (!xmax || !ymax)) {
    // sharded plans: the operand maxima of this launch (x with the halo slices / boundary
    // rows it reads, dy), timed as class 7 like the unsharded plans' precomputed ones
    unsigned* sl = reinterpret_cast<unsigned*>(p->ws + p->fsl) + F16_SHARD_SLOTS;
    HIPCK(spff::zero_async(sl, 2 * sizeof(unsigned), p->st));
    PROFB(p, 7, 0.0, 4.0 * (double)nvox(v) * Cin, absmax_src(xr, v, Cin, true, sl, p->st));
    PROFB(p, 7, 0.0, 4.0 * (double)nvox(v) * Cout,
          absmax_src(src1(dy, Cout), v, Cout, false, sl + 1, p->st));
    xmax = sl;
    ymax = sl + 1;
  }
  PROFB(p, 2, flops, bytes,
        conv3d_wgrad(xr, dy, Cout, dw, v, p->KD, Cin, Cout, p->cfg.math, p->F(p->wg_ws), p->st,
                     xmax, ymax));
  return SPFF_OK;
}

// depth-sharded plans: start the halo exchange of the next dgrad's input on st2 as soon
// as that input is final, so that it runs beside the weight gradient enqueued before the
// dgrad (which reads the same tensor at the local slices only), not just beside the
// dgrad's interior tiles; conv_halo then only waits for ev_halo.
int halo_begin(spff_plan* p, const float* x, const Vol& v, int C) {
  if (p->hsh || !v.dh) return SPFF_OK;
  CK(side_stream(p));
  HIPCK(hipEventRecord(p->ev_in, p->st));
  HIPCK(hipStreamWaitEvent(p->st2, p->ev_in, 0));
  CK(halo(p, x, v, C, p->st2));
  HIPCK(hipEventRecord(p->ev_halo, p->st2));
  p->halo_early = x;
  return SPFF_OK;
}

// halo exchange of x + the 3x3x3 convolution reading it.  Depth-sharded plans whose
// conv can split its depth tiles run the exchange on the side stream st2 while the
// interior depth tiles (which read no halo slice) compute on st, then the first and
// last depth tiles after it; otherwise exchange, then convolve.  cls / flops / bytes:
// the PROFB record of the launch (the interior launch carries the FLOPs, the
// boundary one adds its time to the same class).
// (wmax: the f16_slot max |w| of an unsharded SPFF_MATH_F16X3 plan, else null; the input's
// scale is per (tile, chunk), inside the conv kernel)
int conv_halo(spff_plan* p, int cls, double flops, double bytes, const Src2& x, const Dst2& y,
              const Vol& v, int Cin_w, int Cout_w, bool dgrad, float* stats,
              const unsigned* wmax = nullptr, const BStat* bst = nullptr) {
  if (p->hsh) {
    if (bst) return fail(SPFF_EINVAL, "fused IN-backward sums: unsharded plans only");
    return conv_h(p, cls, flops, bytes, x, y, v, Cin_w, Cout_w, dgrad, wmax);
  }
  if (bst && v.dh) return fail(SPFF_EINVAL, "fused IN-backward sums: unsharded plans only");
  const int KD = p->KD, math = p->cfg.math;
  const bool ovl = v.dh && !stats && conv3d_splits_depth(v, KD, Cin_w, Cout_w, dgrad, math);
  const bool early = p->halo_early && p->halo_early == x.p0 && x.p1 == x.p0;
  p->halo_early = nullptr;
  if (!ovl) {
    if (early)
      HIPCK(hipStreamWaitEvent(p->st, p->ev_halo, 0));
    else
      CK(halo_src(p, x, v));
    PROFB(p, cls, flops, bytes,
          conv3d_run(x, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st, p->F(p->wg_ws),
                     stats, 0, wmax, bst));
    return SPFF_OK;
  }
  if (!early) {
    CK(side_stream(p));
    HIPCK(hipEventRecord(p->ev_in, p->st));  // x is final
    HIPCK(hipStreamWaitEvent(p->st2, p->ev_in, 0));
    CK(halo_src(p, x, v, p->st2));
    HIPCK(hipEventRecord(p->ev_halo, p->st2));
  }
  PROFB(p, cls, flops, bytes,
        conv3d_run(x, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st, p->F(p->wg_ws),
                   nullptr, 1, wmax));
  HIPCK(hipStreamWaitEvent(p->st, p->ev_halo, 0));
  PROFB(p, cls, 0.0, 0.0,
        conv3d_run(x, p->F(p->wcur), y, v, KD, Cin_w, Cout_w, dgrad, math, p->st, p->F(p->wg_ws),
                   nullptr, 2, wmax));
  return SPFF_OK;
}

int in_stats(spff_plan* p, const Vol& v, int C, size_t y, size_t mean, size_t rstd, size_t al,
             size_t de, int64_t gamma, int64_t beta) {
  RedArgs a{};
  a.y = p->F(y);
  const bool sh = p->co.on();
  double* pd = sh ? p->D64(p->part_d) : nullptr;
  const double N = (double)p->co.D_glob * v.H * p->hmul * v.W;
  PROFB(p, 4, 0.0, 4.0 * (double)nvox(v) * C,
        slab_reduce(RED_SUM, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  if (sh) {  // per-(b,c) sums over the slab -> group sum -> global mean
    HIPCK(in_partial(p->F(p->red_out), pd, v, C, 1, p->st));
    HIPCK(p->co.sum_f64(pd, (int64_t)v.B * C, p->st));
    HIPCK(in_mean_fin(pd, p->F(mean), v.B * C, N, p->st));
  } else {
    HIPCK(in_mean(p->F(p->red_out), p->F(mean), v, C, p->st));
  }
  a.mean = p->F(mean);
  PROFB(p, 4, 0.0, 4.0 * (double)nvox(v) * C,
        slab_reduce(RED_SQDEV, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
  if (sh) {
    HIPCK(in_partial(p->F(p->red_out), pd, v, C, 1, p->st));
    HIPCK(p->co.sum_f64(pd, (int64_t)v.B * C, p->st));
    HIPCK(in_rstd_fin(pd, p->P(gamma), p->P(beta), p->F(mean), p->F(rstd), p->F(al), p->F(de),
                      v.B, C, N, p->st));
  } else {
    HIPCK(in_rstd(p->F(p->red_out), p->P(gamma), p->P(beta), p->F(mean), p->F(rstd), p->F(al),
                  p->F(de), v, C, p->st));
  }
  return SPFF_OK;
}

// IN backward statistics from p->red_out = per-(b,c,d) [sum dr, sum dr*xhat]
int in_bwd(spff_plan* p, const Vol& v, int C, int64_t gamma, int64_t beta) {
  if (!p->co.on())
    return in_bwd_stats(p->F(p->red_out), p->P(gamma), p->DP(gamma), p->DP(beta), p->F(p->kk1),
                        p->F(p->kk2), v, C, p->st) == hipSuccess
               ? SPFF_OK
               : fail(SPFF_EHIP, "in_bwd_stats");
  double* pd = p->D64(p->part_d);
  HIPCK(in_partial(p->F(p->red_out), pd, v, C, 2, p->st));
  HIPCK(in_bwd_dgb(pd, p->DP(gamma), p->DP(beta), v.B, C, p->st));  // local partial grads
  HIPCK(p->co.sum_f64(pd, (int64_t)v.B * C * 2, p->st));
  HIPCK(in_bwd_fin(pd, p->F(p->kk1), p->F(p->kk2), v.B * C,
                   (double)p->co.D_glob * v.H * p->hmul * v.W, p->st));
  return SPFF_OK;
}

// conv2's input: a1 = lrelu(IN(y1)) -- read from y1 through the IN affine when the
// conv kernels fuse it (a1 is then never stored), else the materialised a1
Src2 act_src(const spff_plan* p, const Blk& b) {
  if (!b.fa) return src1(p->F(b.a1), b.C);
  Src2 s = src1(p->F(b.y1), b.C);
  s.al = p->F(b.al1);
  s.de = p->F(b.de1);
  s.zlo = p->co.on() && p->co.rank == 0;
  s.zhi = p->co.on() && p->co.rank == p->co.world - 1;
  return s;
}

// SPFF_MATH_F16X3 on an unsharded plan: the per-tensor operand maxima (float bits, the fp16
// planes' scale) of the weights and of the weight gradients' operands (the fwd/dgrad
// kernels scale their input per tile themselves), precomputed once per step and shared by
// the launches that read the tensor: per block, slot F16_W1 / F16_W2 max |w| and F16_A1 a
// parameter bound on a1 = lrelu(IN(y1)) (act_bound), all in one batch at the forward start;
// F16_OUT from the block-output apply (act_apply[_pool]) as it writes out; the block input:
// an encoder's is the previous block's pooled output, bounded by its F16_OUT; a decoder's
// [up | skip] (F16_IN) from the up-conv GEMM as it stores the up part, max-ed with the skip
// encoder's F16_OUT; the first block's a pass over the network input; F16_DY2 / F16_DA1
// from in_bwd_apply as it writes them.  Sharded plans compute the weight gradients' per
// launch (their operands also span halo slices / boundary rows that arrive later).
enum { F16_IN = 0, F16_A1, F16_DY2, F16_DA1, F16_W1, F16_W2, F16_OUT };
unsigned* f16_slot(const spff_plan* p, const Blk& b, int k) {
  if (p->cfg.math != SPFF_MATH_F16X3 || p->co.on() || p->hsh) return nullptr;
  return reinterpret_cast<unsigned*>(p->ws + p->fsl) + 8 * (int)(&b - p->blk) + k;
}
// the slot bounding block b's first-conv input (see above; null: not f16x3 / sharded)
const unsigned* f16_in_slot(const spff_plan* p, const Blk& b) {
  const int bi = (int)(&b - p->blk);
  if (bi >= 1 && bi <= 3) return f16_slot(p, p->blk[bi - 1], F16_OUT);
  return f16_slot(p, b, F16_IN);
}
int f16_in_max(spff_plan* p, const Blk& b, const Src2& in, const Vol& v) {
  unsigned* sl = f16_slot(p, b, F16_IN);
  const int bi = (int)(&b - p->blk);
  // encoders 2-4: the previous block's output max; decoders: the up-conv GEMM filled it as
  // it stored [up | ...] (max-ed with the skip encoder's output max, upconv_out)
  if (!sl || bi >= 1) return SPFF_OK;
  PROFB(p, 7, 0.0, 4.0 * (double)nvox(v) * b.Cin, absmax_src(in, v, b.Cin, false, sl, p->st));
  return SPFF_OK;
}
// max |w| of conv 1 / 2 of block b for the conv kernels (SPFF_MATH_F16X3): batched plans
// fill slot F16_W1 / F16_W2 whatever the sharding (weights are replicated); the others
// pass f16_slot (null on sharded plans: conv3d_pack fills the image's own slot)
const unsigned* w_slot(const spff_plan* p, const Blk& b, int k) {
  if (p->cfg.math != SPFF_MATH_F16X3) return nullptr;
  if (!p->pkb) return f16_slot(p, b, k);
  return reinterpret_cast<const unsigned*>(p->ws + p->fsl) + 8 * (int)(&b - p->blk) + k;
}
// the parameter-derived operand data of a step, at the forward start.  Batched plans: the
// maxima and bounds in one launch (prep_run), then every conv image -- forward and input
// gradient, all 27 -- in one more (conv3d_pack_many); the weights do not change between
// the forward and the backward of a step (the up-conv / head images are packed up front
// the same way).  Otherwise per-tensor launches and conv3d_pack before each conv.
int f16_param_slots(spff_plan* p) {
  const int T = 9 * p->KD;
  const int math = p->cfg.math;
  if (p->pkb) {
    PrepJobs pj;
    PackJobs kj;
    double bytes = 0.0;
    if (math == SPFF_MATH_F16X3)
      HIPCK(spff::zero_async(p->ws + p->fsl, 7 * 8 * sizeof(unsigned), p->st));
    for (int i = 0; i < 7; ++i) {
      Blk& b = p->blk[i];
      const Vol& v = p->vol[b.lvl];
      unsigned* w1 = const_cast<unsigned*>(w_slot(p, b, F16_W1));
      unsigned* w2 = const_cast<unsigned*>(w_slot(p, b, F16_W2));
      bool ok = true;
      if (math == SPFF_MATH_F16X3) {
        ok = ok && prep_absmax(&pj, p->P(b.c1.w), (int64_t)b.C * b.Cin * T, w1);
        ok = ok && prep_absmax(&pj, p->P(b.c2.w), (int64_t)b.C * b.C * T, w2);
        bytes += 4.0 * b.C * (b.Cin + b.C) * T;
        if (unsigned* a1 = f16_slot(p, b, F16_A1)) {
          ok = ok && prep_act_bound(&pj, p->P(b.g1), p->P(b.b1), b.C, (double)v.D * v.H * v.W, a1);
          bytes += 8.0 * b.C;
        }
      }
      ok = ok && conv3d_pack_job(&kj, p->P(b.c1.w), p->F(b.pk[0]), p->KD, b.Cin, b.C, false, w1);
      ok = ok && conv3d_pack_job(&kj, p->P(b.c2.w), p->F(b.pk[1]), p->KD, b.C, b.C, false, w2);
      ok = ok && conv3d_pack_job(&kj, p->P(b.c2.w), p->F(b.pk[2]), p->KD, b.C, b.C, true, w2);
      if (b.pk[3])
        ok = ok && conv3d_pack_job(&kj, p->P(b.c1.w), p->F(b.pk[3]), p->KD, b.Cin, b.C, true, w1);
      if (!ok) return fail(SPFF_EINVAL, "weight preparation table overflow");
    }
    if (pj.n) PROFB(p, 7, 0.0, bytes, prep_run(pj, p->st));
    HIPCK(conv3d_pack_many(kj, math, p->st));
    return SPFF_OK;
  }
  if (!f16_slot(p, p->blk[0], 0)) return SPFF_OK;
  HIPCK(spff::zero_async(p->ws + p->fsl, 7 * 8 * sizeof(unsigned), p->st));
  for (int i = 0; i < 7; ++i) {
    const Blk& b = p->blk[i];
    const Vol& v = p->vol[b.lvl];
    PROFB(p, 7, 0.0, 4.0 * b.C * b.Cin * T,
          absmax_f32(p->P(b.c1.w), (int64_t)b.C * b.Cin * T, f16_slot(p, b, F16_W1), p->st));
    PROFB(p, 7, 0.0, 4.0 * b.C * b.C * T,
          absmax_f32(p->P(b.c2.w), (int64_t)b.C * b.C * T, f16_slot(p, b, F16_W2), p->st));
    PROFB(p, 7, 0.0, 8.0 * b.C, act_bound(p->P(b.g1), p->P(b.b1), b.C, (double)v.D * v.H * v.W,
                    f16_slot(p, b, F16_A1), p->st));
  }
  return SPFF_OK;
}
// the image of conv k of block b (0: c1 fwd, 1: c2 fwd, 2: c2 dgrad, 3: c1 dgrad) for the
// next conv3d_run: the batched one, else packed now into the scratch image
int conv_image(spff_plan* p, const Blk& b, int k, const Vol& v) {
  if (p->pkb) {
    p->wcur = b.pk[k];
    return p->wcur ? SPFF_OK : fail(SPFF_EINVAL, "no batched image for this conv");
  }
  const bool c1 = k == 0 || k == 3;
  HIPCK(conv3d_pack(p->P(c1 ? b.c1.w : b.c2.w), p->F(p->wt), v, p->KD, c1 ? b.Cin : b.C, b.C,
                    k >= 2, p->cfg.math, p->st, f16_slot(p, b, c1 ? F16_W1 : F16_W2)));
  p->wcur = p->wt;
  return SPFF_OK;
}

// pool >= 0: encoder block b's output also feeds MaxPool3d((1,2,2)) into p->pool[pool]
// (the output apply and the pool run as one pass where H and W are even)
int fwd_block(spff_plan* p, Blk& b, const Src2& in, int pool = -1) {
  const Vol& v = p->vol[b.lvl];
  const int C = b.C, KD = p->KD;
  const int math = p->cfg.math;
  CK(conv_image(p, b, 0, v));
  const double V = (double)nvox(v), T = 9.0 * KD;
  CK(f16_in_max(p, b, in, v));
  // InstanceNorm statistics fused into the conv epilogue where the split kernel
  // runs unsharded without split-K; otherwise the two slab_reduce passes
  const bool fuse1 = !p->co.on() && conv3d_fuses_stats(v, KD, b.Cin, C, math);
  CK(conv_halo(p, 0, 2.0 * V * b.Cin * C * T, cbytes(V, b.Cin, C, T), in, dst1(p->F(b.y1), C), v,
               b.Cin, C, false, fuse1 ? p->F(p->cst) : nullptr, w_slot(p, b, F16_W1)));
  if (fuse1)
    HIPCK(conv3d_in_stats_fin(p->F(p->cst), v, KD, b.Cin, C, math, p->P(b.g1), p->P(b.b1),
                              p->F(b.mean1), p->F(b.rstd1), p->F(b.al1), p->F(b.de1), p->st));
  else
    CK(in_stats(p, v, C, b.y1, b.mean1, b.rstd1, b.al1, b.de1, b.g1, b.b1));
  if (!b.fa)
    PROFB(p, 5, 0.0, 8.0 * (double)nvox(v) * C,
          act_apply(p->F(b.y1), p->F(b.a1), p->F(b.al1), p->F(b.de1), nullptr, nullptr, v, C,
                    p->st));
  CK(conv_image(p, b, 1, v));
  const Src2 in2 = act_src(p, b);
  const bool fuse2 = !p->co.on() && conv3d_fuses_stats(v, KD, C, C, math);
  CK(conv_halo(p, 0, 2.0 * V * C * C * T, cbytes(V, C, C, T), in2, dst1(p->F(b.y2), C), v, C, C,
               false, fuse2 ? p->F(p->cst) : nullptr, w_slot(p, b, F16_W2)));
  if (fuse2)
    HIPCK(conv3d_in_stats_fin(p->F(p->cst), v, KD, C, C, math, p->P(b.g2), p->P(b.b2), p->F(b.mean2),
                              p->F(b.rstd2), p->F(b.al2), p->F(b.de2), p->st));
  else
    CK(in_stats(p, v, C, b.y2, b.mean2, b.rstd2, b.al2, b.de2, b.g2, b.b2));
  if (b.tail()) {
    RedArgs a{};
    a.y = p->F(b.y2);
    a.al = p->F(b.al2);
    a.de = p->F(b.de2);
    PROFB(p, 4, 0.0, 4.0 * (double)nvox(v) * C,
        slab_reduce(RED_ACT, a, v, C, p->F(b.Sa), p->F(p->red_ws), p->st));
    GateParams gp = gate_params(p, b);
    GateSaved sv = gate_saved(p, b);
    if (p->hsh) {  // partial (h, w) sums of the local rows -> global; gates replicated
      HIPCK(p->co.sum_f32(p->F(b.Sa), (int64_t)v.B * C * v.D, p->st));
      Vol vg = v;
      vg.H *= p->hmul;
      HIPCK(gates_fwd(gp, p->F(b.Sa), sv, vg, C, p->F(p->gscr), p->st));
    } else if (p->co.on())
      HIPCK(gates_fwd_sh(gp, p->F(b.Sa), sv, v, C, p->F(p->gscr), p->co, p->st));
    else
      HIPCK(gates_fwd(gp, p->F(b.Sa), sv, v, C, p->F(p->gscr), p->st));
  }
  const float* P = b.tail() ? p->F(b.P) : nullptr;
  const float* Q = b.tail() ? p->F(b.Q) : nullptr;
  if (b.fout && !p->keep_out) return SPFF_OK;  // applied by the up-conv / head GEMMs
  if (pool >= 0 && !((v.H | v.W) & 1)) {
    // read y2, write out + pooled + argmax bytes: 4C + 4C + C + C / 4 bytes per voxel
    PROFB(p, 5, 0.0, 9.25 * (double)nvox(v) * C,
          act_apply_pool(p->F(b.y2), p->F(b.out), p->F(b.al2), p->F(b.de2), P, Q,
                         p->F(p->pool[pool]),
                         reinterpret_cast<uint8_t*>(p->ws + p->pidx[pool]), v, C, p->st, 0.01f,
                         f16_slot(p, b, F16_OUT)));
    return SPFF_OK;
  }
  PROFB(p, 5, 0.0, 8.0 * (double)nvox(v) * C,
        act_apply(p->F(b.y2), p->F(b.out), p->F(b.al2), p->F(b.de2), P, Q, v, C, p->st, 0.01f,
                  f16_slot(p, b, F16_OUT)));
  if (pool >= 0)
    HIPCK(maxpool_fwd(p->F(b.out), p->F(p->pool[pool]),
                      reinterpret_cast<uint8_t*>(p->ws + p->pidx[pool]), v, C, p->st));
  return SPFF_OK;
}

Src2 src2(const float* a, const float* b, int C) { return Src2{a, b, C, C, C}; }

// up-conv of block src's output into U.out at the skip's resolution (through U.raw and
// the _cat trilinear resize when the pooled extents were odd)
// (amax / also: the decoder block input's f16x3 slot, filled by the GEMM as it stores the
// up part and max-ed with the skip encoder's output max; null on the lean recompute)
int upconv_out(spff_plan* p, const UpL& U, const Blk& src, unsigned* amax = nullptr,
               const unsigned* also = nullptr) {
  const Vol& low = p->vol[U.lvl_low];
  const ActRows act = act_rows(p, src);
  PROF(p, 3, 2.0 * nvox(low) * U.Cin * 4.0 * U.Cout,
       upconv_fwd(p->F(src.out), p->F(U.pk), p->P(U.b), p->F(U.rs ? U.raw : U.out), low, U.Cin,
                  U.Cout, p->st, 4, p->cfg.math, src.fout ? &act : nullptr, amax, also));
  if (U.rs) {
    const Vol& vh = p->vol[U.lvl_low - 1];
    Vol vr = low;
    vr.H *= 2;
    vr.W *= 2;
    HIPCK(resize_hw_fwd(p->F(U.raw), p->F(U.out), vr, vh.H, vh.W, U.Cout, p->st));
  }
  return SPFF_OK;
}

// block output out = lrelu(y2 * al2 + de2) [* P + Q] into dst (lean recompute)
int recompute_out(spff_plan* p, const Blk& b, float* dst) {
  const Vol& v = p->vol[b.lvl];
  PROFB(p, 5, 0.0, 8.0 * (double)nvox(v) * b.C,
        act_apply(p->F(b.y2), dst, p->F(b.al2), p->F(b.de2), b.tail() ? p->F(b.P) : nullptr,
                  b.tail() ? p->F(b.Q) : nullptr, v, b.C, p->st));
  return SPFF_OK;
}

// lean plans: rebuild the first conv's input [up | skip] of decoder block bi for its
// weight gradient -- called once that block's dout (G_out) and dy2 (G_dy2) are dead:
// the previous decoder's output (up-conv input) at its forward place, the up-conv
// output into G_dx, the encoder skip into G_out, plus their halos when sharded
int lean_dec_input(spff_plan* p, int bi, Src2* in) {
  Blk* B = p->blk;
  const Blk& d = B[bi];
  const Blk& skip = B[6 - bi];
  const Blk& prev = B[bi - 1];
  UpL& U = p->up[bi - 4];
  if (bi - 1 >= 4) CK(recompute_out(p, prev, p->F(prev.out)));
  CK(upconv_out(p, U, prev));
  CK(recompute_out(p, skip, p->F(p->G_out)));
  *in = src2(p->F(U.out), p->F(p->G_out), d.C);
  return halo_src(p, *in, p->vol[d.lvl]);
}

// height-sharded ranks other than 0: the block's replicated gate parameter gradients go
// to scratch and their dparams ranges are zeroed (the flat gradient is SUM-reduced)
int hsh_gate_grads(spff_plan* p, const Blk& b, GateGrads& gg) {
  if (p->co.rank == 0) return SPFF_OK;
  const int64_t g0 = b.b2 + b.C, span = b.pr1 - g0;
  float* dum = p->F(p->gdum);
  auto mv = [&](float*& q, int64_t off, bool se) {
    if (q) q = se ? dum + span + (off - b.se0) : dum + (off - g0);
  };
  mv(gg.fw0, b.fw0, false); mv(gg.fb0, b.fb0, false); mv(gg.fw2, b.fw2, false);
  mv(gg.fb2, b.fb2, false); mv(gg.mask, b.mask, false); mv(gg.mag, b.mag, false);
  mv(gg.sw0, b.sw0, true); mv(gg.sb0, b.sb0, true); mv(gg.sw2, b.sw2, true);
  mv(gg.sb2, b.sb2, true);
  if (span > 0) HIPCK(spff::zero_async(p->DP(g0), span * sizeof(float), p->st));
  if (b.se1 > b.se0)
    HIPCK(spff::zero_async(p->DP(b.se0), (b.se1 - b.se0) * sizeof(float), p->st));
  return SPFF_OK;
}

int bwd_block(spff_plan* p, Blk& b, const float* dout, const Dst2* dx, const Src2& in_saved,
              int dec_bi = -1, PoolAdd pa = {}) {
  const Vol& v = p->vol[b.lvl];
  const int C = b.C, KD = p->KD;
  Src2 in = in_saved;
  const float* A = nullptr;
  const float* Bc = nullptr;
  if (b.tail()) {
    RedArgs a{};
    a.y = p->F(b.y2);
    a.g = dout;
    a.al = p->F(b.al2);
    a.de = p->F(b.de2);
    a.mean = p->F(b.mean2);
    a.rstd = p->F(b.rstd2);
    a.pa = pa;
    // (SPFF_RED_FUSE: the IN-backward sums of y2 in the same pass, RED_BWD_TAIL6)
    PROFB(p, 4, 0.0, 8.0 * (double)nvox(v) * C,
          SPFF_RED_FUSE ? slab_reduce(RED_BWD_TAIL6, a, v, C, p->F(p->red_out), p->F(p->red_ws),
                                      p->st, p->F(p->red_out4))
                        : slab_reduce(RED_BWD_TAIL, a, v, C, p->F(p->red_out), p->F(p->red_ws),
                                      p->st));
    GateParams gp = gate_params(p, b);
    GateSaved sv = gate_saved(p, b);
    GateGrads gg;
    gg.fw0 = b.efilm ? p->DP(b.fw0) : nullptr;
    gg.fb0 = b.efilm ? p->DP(b.fb0) : nullptr;
    gg.fw2 = b.efilm ? p->DP(b.fw2) : nullptr;
    gg.fb2 = b.efilm ? p->DP(b.fb2) : nullptr;
    gg.mask = b.fgate ? p->DP(b.mask) : nullptr;
    gg.mag = b.fgate ? p->DP(b.mag) : nullptr;
    gg.sw0 = b.post_se ? p->DP(b.sw0) : nullptr;
    gg.sb0 = b.post_se ? p->DP(b.sb0) : nullptr;
    gg.sw2 = b.post_se ? p->DP(b.sw2) : nullptr;
    gg.sb2 = b.post_se ? p->DP(b.sb2) : nullptr;
    if (p->hsh) {
      // the per-(b,c,d) sums of dout, dout*a2 summed over the group; every rank then
      // derives the same A, Bc and gate parameter gradients -- rank 0 keeps the latter
      HIPCK(p->co.sum_f32(p->F(p->red_out), (int64_t)v.B * C * v.D * 2, p->st));
      CK(hsh_gate_grads(p, b, gg));
      Vol vg = v;
      vg.H *= p->hmul;
      HIPCK(gates_bwd(gp, sv, p->F(b.Sa), p->F(p->red_out), gg, p->F(p->Abuf), p->F(p->Bbuf), vg,
                      C, p->F(p->gscr), p->st));
    } else if (p->co.on())
      HIPCK(gates_bwd_sh(gp, sv, p->F(b.Sa), p->F(p->red_out), gg, p->F(p->Abuf), p->F(p->Bbuf),
                         v, C, p->F(p->gscr), p->co, p->st));
    else
      HIPCK(gates_bwd(gp, sv, p->F(b.Sa), p->F(p->red_out), gg, p->F(p->Abuf), p->F(p->Bbuf), v,
                      C, p->F(p->gscr), p->st));
    A = p->F(p->Abuf);
    Bc = p->F(p->Bbuf);
  }
  float* dy2 = p->F(p->G_dy2);
  float* da1 = p->F(p->G_da1);
  // PoolAdd reads the pooled gradient (in G_dx) up to this block's IN-backward apply of dy2;
  // only the block's last dgrad (into dx) may overwrite it, so neither dy2 nor da1 may live
  // there (a placement change would corrupt the encoder gradients silently)
  if (pa.dp && (pa.dp == dy2 || pa.dp == da1))
    return fail(SPFF_EINVAL, "PoolAdd gradient aliases a scratch the block writes first");
  {
    RedArgs a{};
    a.y = p->F(b.y2); a.g = dout; a.mean = p->F(b.mean2); a.rstd = p->F(b.rstd2);
    a.al = p->F(b.al2); a.de = p->F(b.de2); a.A = A; a.Bc = Bc; a.pa = pa;
    if (b.tail() && SPFF_RED_FUSE)
      HIPCK(in_sums_from_tail(p->F(p->red_out4), A, Bc, p->F(p->red_out),
                              (int64_t)v.B * C * v.D, p->st));
    else
      PROFB(p, 4, 0.0, 8.0 * (double)nvox(v) * C,
            slab_reduce(RED_BWD_IN, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
    CK(in_bwd(p, v, C, b.g2, b.b2));
    PROFB(p, 6, 0.0, 12.0 * (double)nvox(v) * C,
          in_bwd_apply(p->F(b.y2), dout, dy2, p->F(b.mean2), p->F(b.rstd2), p->F(b.al2),
                       p->F(b.de2), p->P(b.g2), A, Bc, p->F(p->kk1), p->F(p->kk2), v, C, p->st,
                       0.01f, f16_slot(p, b, F16_DY2), pa));
  }
  const double V = (double)nvox(v), T = 9.0 * KD;
  Src2 a1 = act_src(p, b);  // (fused: y1 and its halo as the forward left them)
  if (p->lean && !b.fa) {  // a1 = lrelu(IN(y1)) again, into the buffer da1 overwrites next
    PROFB(p, 5, 0.0, 8.0 * (double)nvox(v) * C,
          act_apply(p->F(b.y1), da1, p->F(b.al1), p->F(b.de1), nullptr, nullptr, v, C, p->st));
    CK(halo(p, da1, v, C));
    a1 = src1(da1, C);
  }
  CK(halo_begin(p, dy2, v, C));  // dgrad input: its exchange beside the weight gradient
  CK(conv_wgrad(p, 2.0 * V * C * C * T, cbytes(V, C, C, T), a1, dy2, p->DP(b.c2.w), v, C, C,
                f16_slot(p, b, F16_A1), f16_slot(p, b, F16_DY2)));
  const int math = p->cfg.math;
  CK(conv_image(p, b, 2, v));
  // the IN-backward sums of conv1 (sum dr, sum dr xhat over da1, y1) in the epilogue of the
  // input-gradient conv that writes da1 (BStat), instead of a RED_BWD_IN pass over both
  const bool bfuse = p->bst_fuse && !p->co.on() && !p->hsh &&
                     conv3d_fuses_bwd_stats(v, KD, C, C, math);
  BStat bs;
  if (bfuse) {
    bs.y = p->F(b.y1);
    bs.al = p->F(b.al1);
    bs.de = p->F(b.de1);
    bs.mean = p->F(b.mean1);
    bs.rstd = p->F(b.rstd1);
    bs.out = p->F(p->cst);
    bs.ld = C;
  }
  // (compulsory bytes: + y1, which the fused epilogue reads once)
  CK(conv_halo(p, 1, 2.0 * V * C * C * T, cbytes(V, C, C, T) + (bfuse ? 4.0 * V * C : 0.0),
               src1(dy2, C), dst1(da1, C), v, C, C, true, nullptr, w_slot(p, b, F16_W2),
               bfuse ? &bs : nullptr));
  {
    RedArgs a{};
    a.y = p->F(b.y1); a.g = da1; a.mean = p->F(b.mean1); a.rstd = p->F(b.rstd1);
    a.al = p->F(b.al1); a.de = p->F(b.de1);
    if (bfuse) {
      HIPCK(conv3d_in_bwd_stats_fin(p->F(p->cst), v, KD, C, C, math, p->DP(b.g1), p->DP(b.b1),
                                    p->F(p->kk1), p->F(p->kk2), p->st));
    } else {
      PROFB(p, 4, 0.0, 8.0 * (double)nvox(v) * C,
            slab_reduce(RED_BWD_IN, a, v, C, p->F(p->red_out), p->F(p->red_ws), p->st));
      CK(in_bwd(p, v, C, b.g1, b.b1));
    }
    PROFB(p, 6, 0.0, 12.0 * (double)nvox(v) * C,
          in_bwd_apply(p->F(b.y1), da1, da1, p->F(b.mean1), p->F(b.rstd1), p->F(b.al1),
                       p->F(b.de1), p->P(b.g1), nullptr, nullptr, p->F(p->kk1), p->F(p->kk2), v,
                       C, p->st, 0.01f, f16_slot(p, b, F16_DA1)));
  }
  if (p->lean && dec_bi >= 0) CK(lean_dec_input(p, dec_bi, &in));
  if (dx) CK(halo_begin(p, da1, v, C));
  CK(conv_wgrad(p, 2.0 * V * b.Cin * C * T, cbytes(V, b.Cin, C, T), in, da1, p->DP(b.c1.w), v,
                b.Cin, C, f16_in_slot(p, b), f16_slot(p, b, F16_DA1)));
  if (dx) {
    CK(conv_image(p, b, 3, v));
    CK(conv_halo(p, 1, 2.0 * V * b.Cin * C * T, cbytes(V, b.Cin, C, T), src1(da1, C), *dx, v,
                 b.Cin, C, true, nullptr, w_slot(p, b, F16_W1)));
  }
  return SPFF_OK;
}

// report dparams[a, b) final to the gradient-ready hook (no-op without one)
int grad_ready(spff_plan* p, int64_t a, int64_t b) {
  if (!p->grad_fn || b <= a) return SPFF_OK;
  if (p->grad_fn(p->grad_ctx, a, b - a, p->st) != 0) return fail(SPFF_EHIP, "gradient hook failed");
  return SPFF_OK;
}
int block_grads_ready(spff_plan* p, const Blk& b) {
  CK(grad_ready(p, b.pr0, b.pr1));
  return grad_ready(p, b.se0, b.se1);
}

int forward(spff_plan* p, const float* x, float* logits) {
  const int f = p->f;
  const spff_cfg& c = p->cfg;
  {  // every block's EnergyFiLM coefficients in one launch (parameters only)
    EfilmJobs jobs;
    jobs.H = p->efh;
    jobs.P = p->efp;
    for (int i = 0; i < 7; ++i) {
      const Blk& b = p->blk[i];
      if (!b.efilm) continue;
      jobs.j[jobs.n++] = EfilmJob{p->P(b.fw0), p->P(b.fb0), p->P(b.fw2), p->P(b.fb2),
                                  p->F(b.t), p->F(b.bt), p->F(b.hid), b.C};
    }
    p->efilm_ready = false;
    HIPCK(efilm_fwd_all(p->pe_dev + p->co.d_off, p->co.D_glob, jobs, c.depth, p->st));
    p->efilm_ready = jobs.n > 0;
  }
  CK(f16_param_slots(p));
  HIPCK(ncdhw_to_ndhwc(x, p->F(p->x_cl), p->vol[0], c.in_ch, p->ldx, p->st));
  Blk* B = p->blk;
  CK(fwd_block(p, B[0], src1(p->F(p->x_cl), p->ldx), 0));
  CK(fwd_block(p, B[1], src1(p->F(p->pool[0]), f), 1));
  CK(fwd_block(p, B[2], src1(p->F(p->pool[1]), 2 * f), 2));
  CK(fwd_block(p, B[3], src1(p->F(p->pool[2]), 4 * f)));
  const Blk* prev = &B[3];
  for (int u = 0; u < 3; ++u) {
    UpL& U = p->up[u];
    float* pk = p->F(U.pk);
    HIPCK(upconv_pack(p->P(U.w), pk, pk + upconv_pack_dgrad_offset(U.Cin, U.Cout), U.Cin, U.Cout,
                      p->st));
    Blk& d = B[4 + u];
    const Blk& skip = B[2 - u];
    CK(upconv_out(p, U, *prev, f16_slot(p, d, F16_IN), f16_slot(p, skip, F16_OUT)));
    CK(fwd_block(p, d, src2(p->F(U.out), p->F(skip.out), U.Cout)));
    prev = &d;
  }
  float* hp = p->F(p->head_pk);
  HIPCK(head_pack(p->P(p->out_w), hp, hp + head_pack_dgrad_offset(f, p->K), f, p->K, p->st));
  const ActRows hact = act_rows(p, *prev);
  PROF(p, 3, 2.0 * nvox(p->vol[0]) * f * p->K,
       head_fwd(p->F(prev->out), hp, p->P(p->out_b), logits, nvox(p->vol[0]), f, p->K, p->st,
                p->cfg.math, prev->fout ? &hact : nullptr));
  return SPFF_OK;
}

int backward(spff_plan* p, const float* dl) {
  const int f = p->f;
  Blk* B = p->blk;
  const int64_t V0 = nvox(p->vol[0]);
  float* hp = p->F(p->head_pk);
  const ActRows hact = act_rows(p, B[6]);
  PROF(p, 3, 2.0 * V0 * f * p->K,
       head_wgrad(p->F(B[6].out), dl, p->DP(p->out_w), p->DP(p->out_b), V0, f, p->K,
                  p->F(p->wg_ws), p->st, B[6].fout ? &hact : nullptr));
  CK(grad_ready(p, p->out_w, p->out_b + p->K));
  PROF(p, 3, 2.0 * V0 * f * p->K,
       head_dgrad(dl, hp + head_pack_dgrad_offset(f, p->K), p->F(p->G_out), V0, f, p->K,
                  p->st, p->cfg.math));
  // decoder: dec1 (B[6]) <- up1 (up[2]) <- dec2 ... ; skip grads go to dskip[l]
  for (int k = 0; k < 3; ++k) {
    const int bi = 6 - k;          // dec1, dec2, dec3
    const int ui = 2 - k;          // up1, up2, up3
    Blk& d = B[bi];
    UpL& U = p->up[ui];
    const int C = d.C;             // = U.Cout = skip channels
    const int lvl = d.lvl;
    Dst2 dx{p->F(p->G_dx), p->F(p->dskip[lvl]), C, C, C};
    CK(bwd_block(p, d, p->F(p->G_out), &dx, src2(p->F(U.out), p->F(B[lvl].out), C), bi));
    CK(block_grads_ready(p, d));
    if (p->dbg_stop == k + 1) return SPFF_OK;
    const Blk& ub = (ui == 0) ? B[3] : B[bi - 1];  // the up-conv's input block
    const ActRows uact = act_rows(p, ub);
    const Vol& low = p->vol[U.lvl_low];
    const float* gup = p->F(p->G_dx);
    if (U.rs) {  // back through the _cat resize to the up-conv's 2H x 2W grid
      Vol vr = low;
      vr.H *= 2;
      vr.W *= 2;
      HIPCK(resize_hw_bwd(p->F(p->G_dx), p->F(U.raw), vr, p->vol[lvl].H, p->vol[lvl].W, C,
                          p->st));
      gup = p->F(U.raw);
    }
    PROF(p, 3, 2.0 * nvox(low) * U.Cin * 4.0 * U.Cout,
         upconv_wgrad(p->F(ub.out), gup, C, p->DP(U.w), p->DP(U.b), low, U.Cin, U.Cout,
                      p->F(p->wg_ws), p->st, 4, p->cfg.math, ub.fout ? &uact : nullptr));
    CK(grad_ready(p, U.w, U.b + U.Cout));
    float* pk = p->F(U.pk);
    PROF(p, 3, 2.0 * nvox(low) * U.Cin * 4.0 * U.Cout,
         upconv_dgrad(gup, C, pk + upconv_pack_dgrad_offset(U.Cin, U.Cout),
                      p->F(p->G_out), low, U.Cin, U.Cout, p->st, 4, p->cfg.math));
  }
  // bottleneck + encoder
  {
    Dst2 dx = dst1(p->F(p->G_dx), 4 * f);
    CK(bwd_block(p, B[3], p->F(p->G_out), &dx, src1(p->F(p->pool[2]), 4 * f)));
    CK(block_grads_ready(p, B[3]));
  }
  for (int l = 2; l >= 0; --l) {
    const int C = f << l;
    // the block's output gradient = skip gradient + the pool's backward of G_dx, formed by
    // its two readers (PoolAdd) -- G_dx is overwritten only by this block's last dgrad
    PoolAdd pa;
    pa.dp = p->F(p->G_dx);
    pa.idx = reinterpret_cast<const uint8_t*>(p->ws + p->pidx[l]);
    if (!p->pool_fold) {
      HIPCK(maxpool_bwd_add(pa.dp, pa.idx, p->F(p->dskip[l]), C, p->F(p->dskip[l]), p->vol[l], C,
                            p->st));
      pa = PoolAdd{};
    }
    if (l > 0) {
      Dst2 dx = dst1(p->F(p->G_dx), C / 2);
      CK(bwd_block(p, B[l], p->F(p->dskip[l]), &dx, src1(p->F(p->pool[l - 1]), C / 2), -1, pa));
    } else {
      CK(bwd_block(p, B[0], p->F(p->dskip[0]), nullptr, src1(p->F(p->x_cl), p->ldx), -1, pa));
    }
    CK(block_grads_ready(p, B[l]));
  }
  return SPFF_OK;
}

}  // namespace

// =================================================================== C ABI ==
extern "C" {

const char* spff_last_error(void) { return g_err.c_str(); }

int spff_plan_create(const spff_cfg* cfg, spff_plan** out) {
  if (!cfg || !out) return fail(SPFF_EINVAL, "null argument");
  spff_plan* p = new spff_plan();
  p->cfg = *cfg;
  int r = build_plan(p);
  if (r != SPFF_OK) {
    if (p->pe_dev) (void)hipFree(p->pe_dev);
    delete p;
    return r;
  }
  *out = p;
  return SPFF_OK;
}

int spff_plan_set_coll(spff_plan* p, const spff_coll* coll) {
  if (!p || !coll) return fail(SPFF_EINVAL, "null argument");
  if (!coll->allreduce || !coll->halo) return fail(SPFF_EINVAL, "spff_coll needs allreduce and halo");
  p->co.ctx = coll->ctx;
  p->co.allreduce = coll->allreduce;
  p->co.halo = coll->halo;
  p->coll_set = true;
  return SPFF_OK;
}

int spff_plan_set_grad_hook(spff_plan* p, spff_grad_ready_fn fn, void* ctx) {
  if (!p) return fail(SPFF_EINVAL, "null plan");
  p->grad_fn = fn;
  p->grad_ctx = ctx;
  return SPFF_OK;
}

void spff_plan_destroy(spff_plan* p) {
  if (!p) return;
  for (auto& r : p->prof) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  if (p->pe_dev) (void)hipFree(p->pe_dev);
  if (p->ev_in) (void)hipEventDestroy(p->ev_in);
  if (p->ev_halo) (void)hipEventDestroy(p->ev_halo);
  if (p->st2) (void)hipStreamDestroy(p->st2);
  delete p;
}

int spff_num_params(const spff_plan* p) { return p ? (int)p->params.size() : 0; }

int spff_param_info(const spff_plan* p, int i, const char** name, int* ndim, int64_t shape[5],
                    int64_t* offset, int64_t* numel) {
  if (!p || i < 0 || i >= (int)p->params.size()) return fail(SPFF_EINVAL, "param index");
  const PEnt& e = p->params[i];
  if (name) *name = e.name.c_str();
  if (ndim) *ndim = (int)e.shape.size();
  if (shape)
    for (int k = 0; k < 5; ++k) shape[k] = k < (int)e.shape.size() ? e.shape[k] : 1;
  if (offset) *offset = e.off;
  if (numel) *numel = e.numel;
  return SPFF_OK;
}

int64_t spff_param_floats(const spff_plan* p) { return p ? p->nparam : 0; }
size_t spff_workspace_bytes(const spff_plan* p) { return p ? p->total : 0; }

// a step that failed because a shard-group callback returned non-zero (e.g. a peer
// that timed out) reports SPFF_ECOLL and which callback, whatever status the failing
// kernel-level call surfaced
static int coll_status(spff_plan* p, int rc, const char* what) {
  if (rc == SPFF_OK || !p->co.failed) return rc;
  return fail(SPFF_ECOLL, std::string(what) + ": shard-group collective (spff_coll." +
                              p->co.failed + ") failed; the step's outputs are undefined (" +
                              g_err + ")");
}

int spff_forward(spff_plan* p, const float* x, const float* params, float* logits, void* ws,
                 void* stream) {
  if (!p || !x || !params || !logits || !ws) return fail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = nullptr;
  p->st = static_cast<hipStream_t>(stream);
  if (p->co.on() && !p->coll_set)
    return fail(SPFF_EINVAL, "depth-sharded plan: call spff_plan_set_coll first");
  CK(ensure_pe(p));
  p->co.failed = nullptr;
  p->halo_early = nullptr;  // never carried over from a step that failed after halo_begin
  const int rc = forward(p, x, logits);
  p->halo_early = nullptr;
  return coll_status(p, rc, "spff_forward");
}

int spff_backward(spff_plan* p, const float* dlogits, const float* params, float* dparams,
                  void* ws, void* stream) {
  if (!p || !dlogits || !params || !dparams || !ws) return fail(SPFF_EINVAL, "null argument");
  p->ws = static_cast<char*>(ws);
  p->prm = params;
  p->dprm = dparams;
  p->st = static_cast<hipStream_t>(stream);
  if (p->co.on() && !p->coll_set)
    return fail(SPFF_EINVAL, "depth-sharded plan: call spff_plan_set_coll first");
  p->co.failed = nullptr;
  p->halo_early = nullptr;  //  a stale early halo would skip an exchange
  const int rc = backward(p, dlogits);
  p->halo_early = nullptr;
  return coll_status(p, rc, "spff_backward");
}

int spff_saved_tensor(const spff_plan* p, void* ws, const char* name, const float** ptr,
                      int64_t* nv, int* ch) {
  if (!p || !ws || !name || !ptr) return fail(SPFF_EINVAL, "null argument");
  const char* base = static_cast<const char*>(ws);
  const std::string n(name);
  auto ret = [&](size_t off, const Vol& v, int c) {
    *ptr = reinterpret_cast<const float*>(base + off);
    if (nv) *nv = nvox(v);
    if (ch) *ch = c;
    return SPFF_OK;
  };
  if (n == "x_cl") return ret(p->x_cl, p->vol[0], p->ldx);
  if (n.rfind("grad.", 0) == 0) {  // backward scratch, sized as level-0 [V0][f]
    const size_t off = n == "grad.out" ? p->G_out : n == "grad.dy2" ? p->G_dy2 :
                       n == "grad.da1" ? p->G_da1 : n == "grad.dx" ? p->G_dx : 0;
    if (off) return ret(off, p->vol[0], p->f);
    for (int l = 0; l < 3; ++l)  // total gradient at encoder output l after a backward
      if (n == "grad.dskip" + std::to_string(l)) return ret(p->dskip[l], p->vol[l], p->f << l);
  }
  for (int i = 0; i < 7; ++i) {
    const Blk& b = p->blk[i];
    const Vol& v = p->vol[b.lvl];
    if (n == b.name + ".y1") return ret(b.y1, v, b.C);
    if (n == b.name + ".a1") {
      if (b.fa)
        return fail(SPFF_EINVAL, "a1 is not stored: conv2 applies lrelu(IN(y1)) as it loads y1");
      return ret(b.a1, v, b.C);
    }
    if (n == b.name + ".y2") return ret(b.y2, v, b.C);
    if (n == b.name + ".out") {
      if (b.fout && !p->keep_out)
        return fail(SPFF_EINVAL, "out is not stored: the up-conv / head GEMMs apply it as they "
                                 "read y2 (spff_debug_set key 1 stores it too)");
      return ret(b.out, v, b.C);
    }
    // per-(b,c) normalisation of the IN that follows conv 1 / 2: r = y*al + de
    const Vol bv{v.B, 1, 1, 1};
    if (n == b.name + ".al1") return ret(b.al1, bv, b.C);
    if (n == b.name + ".de1") return ret(b.de1, bv, b.C);
    if (n == b.name + ".al2") return ret(b.al2, bv, b.C);
    if (n == b.name + ".de2") return ret(b.de2, bv, b.C);
  }
  for (int l = 0; l < 3; ++l) {
    if (n == "pool" + std::to_string(l + 1)) return ret(p->pool[l], p->vol[l + 1], p->f << l);
    // the max-pool's argmax bytes [V_low][C] (k = 2 dh + dw of the 2 x 2 window): uint8
    if (n == "pool" + std::to_string(l + 1) + ".idx")
      return ret(p->pidx[l], p->vol[l + 1], p->f << l);
  }
  const char* upn[3] = {"up3", "up2", "up1"};
  for (int u = 0; u < 3; ++u)
    if (n == upn[u]) return ret(p->up[u].out, p->vol[p->up[u].lvl_low - 1], p->up[u].Cout);
  return fail(SPFF_EINVAL, "unknown saved tensor " + n);
}

int spff_debug_set(spff_plan* p, int key, int value) {
  if (!p) return fail(SPFF_EINVAL, "null plan");
  if (key == 0) p->dbg_stop = value;
  if (key == 1) p->keep_out = value != 0;  // store the GEMM-applied block outputs too
  if (key == 2) p->pool_fold = value != 0;  // 0: k_maxpool_bwd_add pass instead of PoolAdd
  if (key == 3) p->bst_fuse = value != 0;   // 0: conv1's IN-backward sums by a slab_reduce pass
  return SPFF_OK;
}

int spff_prof_enable(spff_plan* p, int on) {
  if (!p) return fail(SPFF_EINVAL, "null plan");
  p->prof_on = on != 0;
  p->prof_n = 0;
  return SPFF_OK;
}

int spff_prof_collect(spff_plan* p, double* out, int nclass) {
  if (!p || !out) return fail(SPFF_EINVAL, "null argument");
  for (int i = 0; i < 4 * nclass; ++i) out[i] = 0.0;
  for (size_t i = 0; i < p->prof_n; ++i) {
    spff_plan::ProfRec& r = p->prof[i];
    HIPCK(hipEventSynchronize(r.b));
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, r.a, r.b));
    if (r.cls < nclass) {
      out[4 * r.cls + 0] += ms;
      out[4 * r.cls + 1] += r.flops;
      out[4 * r.cls + 2] += 1.0;
      out[4 * r.cls + 3] += r.bytes;
    }
  }
  p->prof_n = 0;
  return SPFF_OK;
}

// ---- op-level up-convolution (tests / INTEGRATION): ws = [forward pack | dgrad pack |
// wgrad partial slabs]
size_t spff_upconv_ws_bytes(int B, int D, int H, int W, int cin, int cout) {
  const Vol low{B, D, H, W};
  return upconv_pack_floats(cin, cout) * sizeof(float) + 256 +
         upconv_wgrad_ws_bytes(low, cin, cout);
}
static int upconv_args(int cin, int cout, int math) {
  if (cin % 4 || cout % 4 || cin <= 0 || cout <= 0)
    return fail(SPFF_EINVAL, "cin and cout must be positive multiples of 4");
  if (math < SPFF_MATH_F32 || math > SPFF_MATH_F16X3) return fail(SPFF_EINVAL, "bad math");
  return SPFF_OK;
}
int spff_upconv_fwd(const float* x, const float* w, const float* b, float* y, int B, int D, int H,
                    int W, int cin, int cout, int math, void* ws, void* stream) {
  if (!x || !w || !b || !y || !ws) return fail(SPFF_EINVAL, "null argument");
  CK(upconv_args(cin, cout, math));
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* wf = static_cast<float*>(ws);
  HIPCK(upconv_pack(w, wf, wf + upconv_pack_dgrad_offset(cin, cout), cin, cout, s));
  HIPCK(upconv_fwd(x, wf, b, y, Vol{B, D, H, W}, cin, cout, s, 4, math));
  return SPFF_OK;
}
int spff_upconv_dgrad(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                      int cin, int cout, int math, void* ws, void* stream) {
  if (!dy || !w || !dx || !ws) return fail(SPFF_EINVAL, "null argument");
  CK(upconv_args(cin, cout, math));
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* wf = static_cast<float*>(ws);
  HIPCK(upconv_pack(w, wf, wf + upconv_pack_dgrad_offset(cin, cout), cin, cout, s));
  HIPCK(upconv_dgrad(dy, cout, wf + upconv_pack_dgrad_offset(cin, cout), dx, Vol{B, D, H, W}, cin,
                     cout, s, 4, math));
  return SPFF_OK;
}
int spff_upconv_wgrad(const float* x, const float* dy, float* dw, float* db, int B, int D, int H,
                      int W, int cin, int cout, int math, void* ws, void* stream) {
  if (!x || !dy || !dw || !db || !ws) return fail(SPFF_EINVAL, "null argument");
  CK(upconv_args(cin, cout, math));
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(ws) + upconv_pack_floats(cin, cout) + 64;
  HIPCK(upconv_wgrad(x, dy, cout, dw, db, Vol{B, D, H, W}, cin, cout, part, s, 4, math));
  return SPFF_OK;
}

int spff_conv_prof_enable(int on) {
  conv_prof_enable(on != 0);
  return SPFF_OK;
}

int spff_conv_prof_collect(double* out, int nclass) {
  if (!out || nclass < 0) return fail(SPFF_EINVAL, "null argument");
  HIPCK(conv_prof_collect(out, nclass));
  return SPFF_OK;
}

size_t spff_loss_ws_bytes(int64_t nv, int K) { return loss_ws_bytes(nv, K); }

int spff_loss(const float* logits, const int64_t* labels, int64_t nv, int K, int ignore,
              double smooth, const int64_t* count_override, float* out4, float* dlogits,
              int64_t* conf, void* ws, void* stream) {
  if (!logits || !labels || !out4 || !dlogits || !conf || !ws)
    return fail(SPFF_EINVAL, "null argument");
  if (K < 1 || K > SPFF_MAX_CLASSES) return fail(SPFF_EINVAL, "num_classes must be 1..SPFF_MAX_CLASSES");
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIPCK(loss_fwd(logits, labels, nv, K, ignore, smooth, count_override, out4, dlogits, conf,
                 static_cast<float*>(ws), s));
  return SPFF_OK;
}

int spff_confusion(const float* logits, const int64_t* labels, int64_t nv, int K, int ignore,
                   int64_t* conf, void* stream) {
  if (!logits || !labels || !conf) return fail(SPFF_EINVAL, "null argument");
  if (K < 1 || K > SPFF_MAX_CLASSES) return fail(SPFF_EINVAL, "num_classes must be 1..SPFF_MAX_CLASSES");
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIPCK(confusion_only(logits, labels, nv, K, ignore, conf, s));
  return SPFF_OK;
}

int spff_count_valid(const int64_t* labels, int64_t nv, int ignore, int64_t* count, void* stream) {
  if (!labels || !count) return fail(SPFF_EINVAL, "null argument");
  HIPCK(count_valid(labels, nv, ignore, count, static_cast<hipStream_t>(stream)));
  return SPFF_OK;
}

int spff_scale(float* x, int64_t n, const float* scale, void* stream) {
  if (!x || !scale) return fail(SPFF_EINVAL, "null argument");
  HIPCK(scale_by_dev(x, n, scale, static_cast<hipStream_t>(stream)));
  return SPFF_OK;
}

int spff_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   int64_t n, double lr, double beta1, double beta2, double eps,
                   double weight_decay, int decoupled, int64_t step, void* stream) {
  if (n > 0 && (!params || !grads || !exp_avg || !exp_avg_sq))
    return fail(SPFF_EINVAL, "null argument");
  if (step < 1) return fail(SPFF_EINVAL, "step must be >= 1");
  HIPCK(adam_step(params, grads, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay,
                  decoupled, step, static_cast<hipStream_t>(stream)));
  return SPFF_OK;
}

// ---- op-level conv entry points ----
static size_t conv_op_pack_floats(int cin, int cout, int ksd) {
  ConvL c;
  conv_dims(c, cin, cout);
  return conv_pack_bytes(c, ksd) / sizeof(float);
}

size_t spff_conv3d_ws_bytes(int B, int D, int H, int W, int cin, int cout, int ksd) {
  Vol v{B, D, H, W};
  return conv_op_pack_floats(cin, cout, ksd) * sizeof(float) + 256 +
         conv3d_wgrad_ws_bytes(v, ksd, cin, cout);
}

int spff_conv3d_fwd_ex(const float* x, int ldx, const float* w, float* y, int B, int D, int H,
                       int W, int cin, int cout, int ksd, int math, void* ws, void* stream) {
  if (!x || !w || !y || !ws) return fail(SPFF_EINVAL, "null argument");
  if (ldx % 4 || ldx < cin) return fail(SPFF_EINVAL, "ldx must be >= cin and a multiple of 4");
  if (cout % 4) return fail(SPFF_EINVAL, "cout must be a multiple of 4");
  if (math < SPFF_MATH_F32 || math > SPFF_MATH_F16X3) return fail(SPFF_EINVAL, "bad math");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Vol v{B, D, H, W};
  HIPCK(conv3d_pack(w, ws, v, ksd, cin, cout, false, math, s));
  HIPCK(conv3d_run(src1(x, ldx), ws, dst1(y, cout), v, ksd, cin, cout, false, math, s));
  return SPFF_OK;
}

int spff_conv3d_fwd(const float* x, int ldx, const float* w, float* y, int B, int D, int H, int W,
                    int cin, int cout, int ksd, void* ws, void* stream) {
  return spff_conv3d_fwd_ex(x, ldx, w, y, B, D, H, W, cin, cout, ksd, SPFF_MATH_F32, ws, stream);
}

int spff_conv3d_dgrad_ex(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                         int cin, int cout, int ksd, int math, void* ws, void* stream) {
  if (!dy || !w || !dx || !ws) return fail(SPFF_EINVAL, "null argument");
  if (cout % 4 || cin % 4) return fail(SPFF_EINVAL, "channels must be multiples of 4");
  if (math < SPFF_MATH_F32 || math > SPFF_MATH_F16X3) return fail(SPFF_EINVAL, "bad math");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Vol v{B, D, H, W};
  HIPCK(conv3d_pack(w, ws, v, ksd, cin, cout, true, math, s));
  HIPCK(conv3d_run(src1(dy, cout), ws, dst1(dx, cin), v, ksd, cin, cout, true, math, s));
  return SPFF_OK;
}

int spff_conv3d_dgrad(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                      int cin, int cout, int ksd, void* ws, void* stream) {
  return spff_conv3d_dgrad_ex(dy, w, dx, B, D, H, W, cin, cout, ksd, SPFF_MATH_F32, ws, stream);
}

int spff_conv3d_wgrad_ex(const float* x, int ldx, const float* dy, float* dw, int B, int D,
                         int H, int W, int cin, int cout, int ksd, int math, void* ws,
                         void* stream) {
  if (!x || !dy || !dw || !ws) return fail(SPFF_EINVAL, "null argument");
  if (ldx % 4 || ldx < cin || cout % 4) return fail(SPFF_EINVAL, "bad channel strides");
  if (math < SPFF_MATH_F32 || math > SPFF_MATH_F16X3) return fail(SPFF_EINVAL, "bad math");
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(ws) + conv_op_pack_floats(cin, cout, ksd) + 64;
  HIPCK(conv3d_wgrad(src1(x, ldx), dy, cout, dw, Vol{B, D, H, W}, ksd, cin, cout, math, part,
                     s));
  return SPFF_OK;
}

int spff_conv3d_wgrad(const float* x, int ldx, const float* dy, float* dw, int B, int D, int H,
                      int W, int cin, int cout, int ksd, void* ws, void* stream) {
  return spff_conv3d_wgrad_ex(x, ldx, dy, dw, B, D, H, W, cin, cout, ksd, SPFF_MATH_F32, ws,
                              stream);
}

}  // extern "C"
