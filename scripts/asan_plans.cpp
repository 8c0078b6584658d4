// Host-side sanitizer driver for the C ABI ("an ASan/UBSan CPU build of
// the C ABI").  Built by scripts/asan_build.sh with the host half of every HIP
// translation unit under -fsanitize=address,undefined; runs with no GPU and makes no
// device call: it creates and destroys a plan for every BASELINE.json configuration
// (and the sharded / ragged / ablation variants), walks the flat parameter layout,
// sizes every workspace, resolves every saved-tensor name against a dummy workspace
// pointer, and checks that malformed configurations are rejected with an error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "spff.h"

static int g_fail = 0;
#define EXPECT(c, ...)                              \
  do {                                              \
    if (!(c)) {                                     \
      std::fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);            \
      std::fprintf(stderr, "\n");                   \
      ++g_fail;                                     \
    }                                               \
  } while (0)

static spff_cfg cfg_of(int B, int Cin, int D, int H, int W, int K, int base = 32, int world = 1,
                       int rank = 0, int axis = 0, int mem = SPFF_MEM_AUTO, int math = SPFF_MATH_BF16X6,
                       int efilm = 1, int fgate = 1, int se = 1, int specse = 1) {
  spff_cfg c;
  std::memset(&c, 0, sizeof c);
  c.batch = B; c.in_ch = Cin; c.depth = D; c.height = H; c.width = W;
  c.num_classes = K; c.base = base; c.ksd = 3;
  c.use_efilm = efilm; c.use_fgate = fgate; c.use_se = se; c.use_specse = specse;
  c.math = math; c.shard_world = world; c.shard_rank = rank; c.shard_axis = axis;
  c.memory_mode = mem;
  return c;
}

static const char* kSaved[] = {
    "x_cl", "grad.out", "grad.dy2", "grad.da1", "grad.dx", "enc1.y1", "enc1.y2", "enc1.out",
    "enc1.a1", "enc1.al1", "enc1.de1", "enc1.al2", "enc1.de2", "enc2.y1", "enc3.y2", "bott.y1",
    "bott.out", "dec3.y1", "dec3.out", "dec2.y2", "dec1.y1", "dec1.out", "pool1", "pool2",
    "pool3", "up3", "up2", "up1", "no.such.tensor"};

static void plan_case(const char* tag, const spff_cfg& c) {
  spff_plan* p = nullptr;
  const int rc = spff_plan_create(&c, &p);
  EXPECT(rc == SPFF_OK && p, "%s: spff_plan_create rc %d (%s)", tag, rc, spff_last_error());
  if (!p) return;
  const int n = spff_num_params(p);
  EXPECT(n > 0, "%s: %d params", tag, n);
  int64_t end = 0;
  for (int i = 0; i < n; ++i) {
    const char* name = nullptr;
    int nd = 0;
    int64_t shape[5] = {0, 0, 0, 0, 0}, off = -1, numel = -1;
    EXPECT(spff_param_info(p, i, &name, &nd, shape, &off, &numel) == SPFF_OK, "%s: param %d", tag, i);
    int64_t prod = 1;
    for (int k = 0; k < nd; ++k) prod *= shape[k];
    EXPECT(name && std::strlen(name) > 0 && nd >= 1 && nd <= 5 && prod == numel && off == end,
           "%s: param %d %s layout", tag, i, name ? name : "?");
    end = off + numel;
  }
  EXPECT(end == spff_param_floats(p), "%s: flat size", tag);
  const char* nm = nullptr;
  int nd = 0;
  int64_t sh[5], off, numel;
  EXPECT(spff_param_info(p, n, &nm, &nd, sh, &off, &numel) != SPFF_OK, "%s: index past end", tag);
  EXPECT(spff_param_info(p, -1, &nm, &nd, sh, &off, &numel) != SPFF_OK, "%s: negative index", tag);
  const size_t ws = spff_workspace_bytes(p);
  EXPECT(ws > 0, "%s: workspace", tag);
  // saved-tensor lookups are pointer arithmetic on the workspace (never dereferenced)
  static char dummy[16];
  for (const char* s : kSaved) {
    const float* ptr = nullptr;
    int64_t nv = 0;
    int ch = 0;
    if (spff_saved_tensor(p, dummy, s, &ptr, &nv, &ch) == SPFF_OK) {
      const size_t o = (size_t)((const char*)ptr - dummy);
      EXPECT(o + (size_t)nv * ch * 4 <= ws, "%s: saved %s [%zu + %lld] outside the workspace",
             tag, s, o, (long long)nv * ch * 4);
    }
  }
  EXPECT(spff_saved_tensor(p, dummy, "no.such.tensor", nullptr, nullptr, nullptr) != SPFF_OK,
         "%s: unknown saved name", tag);
  std::printf("  %-44s params %3d  floats %9lld  workspace %8.2f GiB\n", tag, n,
              (long long)spff_param_floats(p), ws / 1073741824.0);
  spff_plan_destroy(p);
}

static void reject(const char* tag, const spff_cfg& c) {
  spff_plan* p = nullptr;
  const int rc = spff_plan_create(&c, &p);
  EXPECT(rc != SPFF_OK && !p, "%s: malformed config accepted", tag);
  if (p) spff_plan_destroy(p);
}

int main() {
  std::printf("SPFF plans (BASELINE.json configs and variants):\n");
  plan_case("config1 registry 1x1x5x64x64 K9", cfg_of(1, 1, 5, 64, 64, 9));
  plan_case("config2 headline 2x5x128^3 K13", cfg_of(2, 5, 128, 128, 128, 13));
  plan_case("config2 f32", cfg_of(2, 5, 128, 128, 128, 13, 32, 1, 0, 0, SPFF_MEM_AUTO, SPFF_MATH_F32));
  plan_case("config2 lean", cfg_of(2, 5, 128, 128, 128, 13, 32, 1, 0, 0, SPFF_MEM_LEAN));
  plan_case("config4 whole 1x5x512^3 (lean)", cfg_of(1, 5, 512, 512, 512, 13));
  for (int r : {0, 3, 7})
    plan_case(("config4 depth-shard 8 rank " + std::to_string(r)).c_str(),
              cfg_of(1, 5, 64, 512, 512, 13, 32, 8, r, SPFF_SHARD_DEPTH));
  for (int r : {0, 1})
    plan_case(("registry height-shard 2 rank " + std::to_string(r)).c_str(),
              cfg_of(1, 1, 5, 256, 512, 13, 32, 2, r, SPFF_SHARD_HEIGHT));
  plan_case("ragged 1x5x4x18x20 (trilinear _cat)", cfg_of(1, 5, 4, 18, 20, 9, 8));
  plan_case("ablation no efilm/fgate", cfg_of(1, 5, 8, 32, 32, 9, 8, 1, 0, 0, 0, 1, 0, 0, 1, 1));
  plan_case("ablation no se/specse", cfg_of(1, 5, 8, 32, 32, 9, 8, 1, 0, 0, 0, 1, 1, 1, 0, 0));
  reject("H < 8", cfg_of(1, 1, 5, 4, 64, 13));
  plan_case("K 40 base 24 (fx5)", cfg_of(1, 5, 6, 24, 24, 40, 24));
  {
    spff_cfg g = cfg_of(1, 5, 8, 16, 16, 9, 8);
    g.efilm_hidden = 24;
    g.efilm_pe_dims = 11;
    g.fgate_learn_phase = 1;
    plan_case("gates hidden 24 pe_dims 11 learn_phase (fx6)", g);
    g.efilm_hidden = 65;
    reject("efilm hidden 65", g);
    g.efilm_hidden = 24;
    g.efilm_pe_dims = 1;
    reject("efilm pe_dims 1", g);
  }
  reject("K > SPFF_MAX_CLASSES", cfg_of(1, 1, 5, 64, 64, SPFF_MAX_CLASSES + 1));
  reject("base 20", cfg_of(1, 1, 5, 64, 64, 13, 20));
  reject("depth shard batch 2", cfg_of(2, 1, 8, 64, 64, 13, 32, 2, 0, SPFF_SHARD_DEPTH));
  reject("height shard 60 rows", cfg_of(1, 1, 5, 60, 512, 13, 32, 2, 0, SPFF_SHARD_HEIGHT));
  reject("bad shard axis", cfg_of(1, 1, 5, 64, 512, 13, 32, 2, 0, 2));
  reject("rank >= world", cfg_of(1, 5, 64, 64, 64, 13, 32, 2, 2, SPFF_SHARD_DEPTH));
  EXPECT(spff_plan_create(nullptr, nullptr) != SPFF_OK, "null cfg");
  spff_plan_destroy(nullptr);
  EXPECT(spff_loss_ws_bytes(2LL * 128 * 128 * 128, 13) > 0, "loss ws");
  EXPECT(spff_conv3d_ws_bytes(2, 128, 128, 128, 32, 32, 3) >= 0, "conv ws");

  std::printf("3DUNet (BASELINE configs[2]):\n");
  {
    spff_unet3d_cfg c;
    std::memset(&c, 0, sizeof c);
    c.batch = 4; c.in_ch = 1; c.depth = 5; c.height = 96; c.width = 96;
    c.target_depth = 16; c.num_classes = 13; c.base = 32; c.math = SPFF_MATH_BF16X6;
    spff_unet3d* u = nullptr;
    EXPECT(spff_unet3d_create(&c, &u) == SPFF_OK && u, "unet3d create: %s", spff_last_error());
    if (u) {
      int64_t end = 0;
      for (int i = 0; i < spff_unet3d_num_params(u); ++i) {
        const char* name; int nd; int64_t sh[5], off, numel;
        EXPECT(spff_unet3d_param_info(u, i, &name, &nd, sh, &off, &numel) == SPFF_OK && off == end,
               "unet3d param %d", i);
        end = off + numel;
      }
      EXPECT(end == spff_unet3d_param_floats(u), "unet3d flat size");
      int64_t bend = 0;
      for (int i = 0; i < spff_unet3d_num_buffers(u); ++i) {
        const char* name; int64_t off, numel;
        EXPECT(spff_unet3d_buffer_info(u, i, &name, &off, &numel) == SPFF_OK && off == bend,
               "unet3d buffer %d", i);
        bend = off + numel;
      }
      EXPECT(bend == spff_unet3d_buffer_floats(u), "unet3d buffer size");
      std::printf("  4x1x5x96^2 -> 16: params %lld, workspace %.2f GiB\n",
                  (long long)spff_unet3d_param_floats(u), spff_unet3d_workspace_bytes(u) / 1073741824.0);
      spff_unet3d_destroy(u);
    }
    c.height = 90;  // not a multiple of 16
    u = nullptr;
    EXPECT(spff_unet3d_create(&c, &u) != SPFF_OK && !u, "unet3d H 90 accepted");
    if (u) spff_unet3d_destroy(u);
  }

  std::printf("SwinUNETR (BASELINE configs[4]):\n");
  {
    spff_swin_cfg c;
    std::memset(&c, 0, sizeof c);
    c.batch = 2; c.in_ch = 1; c.depth = 128; c.height = 128; c.width = 128;
    c.num_classes = 13; c.feature_size = 12; c.window = 7;
    c.heads[0] = 1; c.heads[1] = 2; c.heads[2] = 4; c.heads[3] = 8;
    c.mlp_ratio = 2.0f; c.math = SPFF_MATH_BF16X6;
    spff_swin* s = nullptr;
    EXPECT(spff_swin_create(&c, &s) == SPFF_OK && s, "swin create: %s", spff_last_error());
    if (s) {
      int64_t end = 0;
      for (int i = 0; i < spff_swin_num_params(s); ++i) {
        const char* name; int nd; int64_t sh[5], off, numel;
        EXPECT(spff_swin_param_info(s, i, &name, &nd, sh, &off, &numel) == SPFF_OK && off == end,
               "swin param %d", i);
        end = off + numel;
      }
      EXPECT(end == spff_swin_param_floats(s), "swin flat size");
      std::printf("  2x1x128^3: params %lld, workspace %.2f GiB\n", (long long)spff_swin_param_floats(s),
                  spff_swin_workspace_bytes(s) / 1073741824.0);
      spff_swin_destroy(s);
    }
    EXPECT(spff_swin_loss_ws_bytes(2, 13) > 0, "swin loss ws");
  }
  std::printf(g_fail ? "asan_plans: %d FAILURES\n" : "asan_plans: ok\n", g_fail);
  return g_fail ? 1 : 0;
}
