// 3x3x3 convolution weight gradient on the bf16 matrix cores with the exact
// 3-plane (bf16x6) or 2-plane (bf16x3) operand split of conv3d_x.hip.
//
// Replaces the weight gradient of nn.Conv3d(cin, cout, (ksd,3,3),
// padding=(ksd//2,1,1), bias=False) (reference models.py:616-618):
//   dW[co][ci][tap] = sum_v x[v + off(tap)][ci] * dy[v][co].
//
// MFMA v_mfma_f32_32x32x16_bf16: rows = (tap, ci) -- a 32-row block is 8 chunks
// of 4 input channels, each chunk at its own tap -- cols = 32 out channels,
// k = 16 voxels (one W-row of the 1 x 8 x 16 voxel tile).  Both operands need
// the voxel axis in their k slots while the LDS images are channel-last
// ([plane][pos][CI] halo, [plane][voxel][32] dy tile, exactly as global memory):
// ds_read_b64_tr_b16 gathers them transposed -- every lane supplies the address
// of 4 contiguous channels of one voxel, so each row's tap offset and each
// chunk's channel base are free per lane and no shifted copies are needed.
// Blocks pair taps whose halo offsets differ by 4 (mod 8) positions, so the
// two 16-lane groups of a 32-lane half read disjoint bank ranges.
//
// 256 threads (4 waves), two workgroups per CU (76 KB LDS each) so one
// workgroup's staging (fp32 loads, exact split, LDS stores) overlaps the other's
// MFMAs; the next tile's halo / dy are register-prefetched during the current
// tile's MFMAs.  Output: the fp32 partial slabs of conv3d.hip's wgrad
// ([split][tap][kpad][npad]), summed in fixed order by k_wgrad_reduce.
#include "spff_internal.h"
#include "bf16split.h"

#include <type_traits>
#include <vector>

#ifndef SPFF_XCDMAP
#define SPFF_XCDMAP 1  // 0: split-fastest block order (A/B diagnostics)
#endif
#ifndef SPFF_WX16
#define SPFF_WX16 1  // 1: v_mfma_f32_16x16x32_bf16 wgrad (k_conv3d_wgrad_x16), 0: 32x32x16
#endif
#ifndef SPFF_WXUNROLL
#define SPFF_WXUNROLL 4  // k-step (W-row pair) loop unroll of k_conv3d_wgrad_x16
#endif
#ifndef SPFF_WXRING4
#define SPFF_WXRING4 1  // f16x3 3x3x3 wgrad: 4-slot plane ring + double dy buffer (one barrier)
#endif
#ifndef SPFF_WXUNROLL2
// the same for two-plane operands (bf16x3, f16x3): unrolled 4 deep the compiler hoists the
// fragment reads of later k-steps (fewer MFMAs per step) into 256 VGPRs + 11-23 spilled;
// 2 deep: 218 VGPRs, no spill
#define SPFF_WXUNROLL2 2
#endif

namespace spff {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int rup(int a, int b) { return cdiv(a, b) * b; }

namespace {
constexpr int WX_TH = 8, WX_TW = 16, WX_TV = WX_TH * WX_TW, WX_CO = 32, WX_MAXBLK = 16;

// (tap, channel base) of the 8 four-channel chunks of each 32-row block
struct WxTable {
  signed char tap[WX_MAXBLK][8];   // -1: padding chunk (computed, never stored)
  signed char ci0[WX_MAXBLK][8];
  int nblk;
};

__device__ __forceinline__ unsigned short bfbits(__bf16 v) {
  return __builtin_bit_cast(unsigned short, v);
}
template <int NS>
__device__ __forceinline__ void split4(const float4& v, uint2 (&o)[nplanes(NS)]) {
  split4_pk<NS>(v, o);  // bf16split.h
}

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
__device__ __forceinline__ i16x4 tr_read(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
}
__device__ __forceinline__ bf16x8 frag(const i16x4& lo, const i16x4& hi) {
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
}  // namespace

template <int KD, int CI, int NS, int NJMAX>
__global__ __launch_bounds__(256, 2) void k_conv3d_wgrad_x(
    Src2 x, const float* __restrict__ dy, int lddy, float* __restrict__ part, Vol vol, int Cin,
    int kpad, int Cout, int npad, int tilesH, int tilesW, int ntiles, int tps, WxTable tb) {
  constexpr int HD = KD, HH = WX_TH + 2, HWD = WX_TW + 2;
  constexpr int NPOS = HD * HH * HWD;
  constexpr int T = KD * 9;
  constexpr int CQ = CI / 4;                              // float4 per halo position
  constexpr int NH = (NPOS * CQ + 255) / 256;              // halo float4 per thread
  constexpr int NY = WX_TV * (WX_CO / 4) / 256;            // dy float4 per thread (= 4)
  __shared__ __attribute__((aligned(16))) unsigned short Xs[NS * NPOS * CI];
  __shared__ __attribute__((aligned(16))) unsigned short Ys[NS * WX_TV * WX_CO];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, h = g >> 1, q = (lane & 15) >> 2, pq = lane & 3;
  // XCD-aware order: blocks b and b + 8 share an XCD, so XCD group b % 8 runs the
  // (ci, co) blocks of one voxel range back to back -- every x / dy tile is fetched
  // from HBM once and re-read by the other channel blocks from that XCD's L2
  const int nci = kpad / CI, ncb = nci * (npad / WX_CO);
  const int rk = blockIdx.x >> 3;
  const int nsp8 = gridDim.x / ncb;
  const int cb = SPFF_XCDMAP ? rk % ncb : (int)(blockIdx.x / nsp8);
  const int split = SPFF_XCDMAP ? (rk / ncb) * 8 + (blockIdx.x & 7) : (int)(blockIdx.x % nsp8);
  if (split * tps >= ntiles) return;  // padding block (uniform)
  const int ci_base = (cb % nci) * CI, co0 = (cb / nci) * WX_CO;
  const int D = vol.D, H = vol.H, W = vol.W;

  // blocks of this wave: wave, wave + 4, ...; nj of them (uniform per wave)
  const int nj = (tb.nblk - wave + 3) / 4;
  // lane-constant A addresses (elements, plane 0, k-step 0, read 0) per block
  int aoff[NJMAX];
#pragma unroll
  for (int j = 0; j < NJMAX; ++j) {
    const int blk = wave + 4 * j;
    const int c4 = 4 * (g & 1) + pq;
    int t = blk < tb.nblk ? tb.tap[blk][c4] : -1;
    const int ci0 = blk < tb.nblk ? tb.ci0[blk][c4] : 0;
    if (t < 0) t = 0;  // padding chunk: any valid address
    const int kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
    aoff[j] = ((kd * HH + kh) * HWD + kw + 8 * h + q) * CI + ci0;
  }
  // B: row q of the read = voxel 8h + 4s + q of k-step j; cols co 16(g&1) + 4pq
  const int boff = (8 * h + q) * WX_CO + 16 * (g & 1) + 4 * pq;

  f32x16 acc[NJMAX];
#pragma unroll
  for (int j = 0; j < NJMAX; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  float4 hreg[NH], yreg[NY];
  float4 xal = make_float4(1.f, 1.f, 1.f, 1.f), xde = make_float4(0.f, 0.f, 0.f, 0.f);
  auto fetch = [&](int tile) {
    // depth-fastest tile order: a split's consecutive tiles share two of their three
    // halo planes, which the previous tile has just brought into L2
    int t = tile;
    const int d0 = t % D; t /= D;
    const int twi = t % tilesW; t /= tilesW;
    const int thi = t % tilesH;
    const int b = t / tilesH;
    const int h0 = thi * WX_TH, w0 = twi * WX_TW;
    if (x.al) {  // fused input activation: this tile's batch, this thread's 4 channels
      // (256 threads, CQ | 256: the thread's channel group is the same for every k)
      const int c = ci_base + 4 * (tid % CQ);
      if (c < Cin) {
        xal = *reinterpret_cast<const float4*>(x.al + (int64_t)b * x.ld0 + c);
        xde = *reinterpret_cast<const float4*>(x.de + (int64_t)b * x.ld0 + c);
      }
    }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int i = tid + 256 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NPOS * CQ) {
        const int c4 = i % CQ, pos = i / CQ;
        const int hw = pos % HWD, t2 = pos / HWD, hh = t2 % HH, hd = t2 / HH;
        const int gd = d0 + hd - KD / 2, gh = h0 + hh - 1, gw = w0 + hw - 1;
        const int c = ci_base + 4 * c4;
        if ((unsigned)(gd + vol.dh) < (unsigned)(D + 2 * vol.dh) && (unsigned)gh < (unsigned)H &&
            (unsigned)gw < (unsigned)W && c < Cin && !((gd < 0 && x.zlo) || (gd >= D && x.zhi))) {
          const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
          const float* p =
              c < x.split ? x.p0 + vox * x.ld0 + c : x.p1 + vox * x.ld1 + (c - x.split);
          v = *reinterpret_cast<const float4*>(p);
          if (x.al) {
            v.x = v.x * xal.x + xde.x; v.x = v.x > 0.f ? v.x : 0.01f * v.x;
            v.y = v.y * xal.y + xde.y; v.y = v.y > 0.f ? v.y : 0.01f * v.y;
            v.z = v.z * xal.z + xde.z; v.z = v.z > 0.f ? v.z : 0.01f * v.z;
            v.w = v.w * xal.w + xde.w; v.w = v.w > 0.f ? v.w : 0.01f * v.w;
          }
        }
      }
      hreg[k] = v;
    }
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = tid + 256 * k;
      const int c4 = i % (WX_CO / 4), kv = i / (WX_CO / 4);
      const int gh = h0 + kv / WX_TW, gw = w0 + kv % WX_TW;
      const int c = co0 + 4 * c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gh < H && gw < W && c < Cout) {
        const int64_t vox = (((int64_t)b * D + d0) * H + gh) * W + gw;
        v = *reinterpret_cast<const float4*>(dy + vox * lddy + c);
      }
      yreg[k] = v;
    }
  };
  auto stash = [&](bool negate) {
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int i = tid + 256 * k;
      if (i < NPOS * CQ) {
        uint2 o[NS];
        split4<NS>(hreg[k], o);
#pragma unroll
        for (int p = 0; p < NS; ++p)
          *reinterpret_cast<uint2*>(Xs + p * NPOS * CI + 4 * i) = o[p];
      }
    }
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = tid + 256 * k;
      uint2 o[NS];
      const float4 yv = negate ? make_float4(-yreg[k].x, -yreg[k].y, -yreg[k].z, -yreg[k].w)
                               : yreg[k];
      split4<NS>(yv, o);
#pragma unroll
      for (int p = 0; p < NS; ++p)
        *reinterpret_cast<uint2*>(Ys + p * WX_TV * WX_CO + 4 * i) = o[p];
    }
  };

  auto compute = [&](auto NJc) {
    constexpr int NJ = decltype(NJc)::value;
#pragma unroll 2
    for (int ks = 0; ks < WX_TH; ++ks) {
      bf16x8 bq[NS];
#pragma unroll
      for (int p = 0; p < NS; ++p) {
        const unsigned short* yb = Ys + p * WX_TV * WX_CO + ks * WX_TW * WX_CO + boff;
        bq[p] = frag(tr_read(yb), tr_read(yb + 4 * WX_CO));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        bf16x8 aq[NS];
#pragma unroll
        for (int p = 0; p < NS; ++p) {
          const unsigned short* xb = Xs + p * NPOS * CI + ks * HWD * CI + aoff[j];
          aq[p] = frag(tr_read(xb), tr_read(xb + 4 * CI));
        }
        f32x16 c = acc[j];
        if constexpr (NS == 3) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[1], bq[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[0], bq[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[2], bq[0], c, 0, 0, 0);
        }
        if constexpr (NS >= 2) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[0], bq[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[1], bq[0], c, 0, 0, 0);
        }
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[0], bq[0], c, 0, 0, 0);
        acc[j] = c;
      }
    }
  };

  const int tbeg = split * tps;
  const int tend = min(ntiles, tbeg + tps);
  if (tbeg < tend) fetch(tbeg);
  for (int tile = tbeg; tile < tend; ++tile) {
    // sign-alternating accumulation (conv3d_x.hip): odd tiles stage -dy and the
    // accumulators flip sign at every tile boundary, so the bf16 MFMA's one-sided
    // rounding of the small split products cancels between consecutive tiles
    if (tile != tbeg) {
#pragma unroll
      for (int j = 0; j < NJMAX; ++j) acc[j] = -acc[j];
    }
    __syncthreads();  // previous compute done reading LDS
    stash(((tile - tbeg) & 1) != 0);
    __syncthreads();
    if (tile + 1 < tend) fetch(tile + 1);
    if (nj == NJMAX) compute(std::integral_constant<int, NJMAX>{});
    else if constexpr (NJMAX > 1) compute(std::integral_constant<int, NJMAX - 1>{});
  }

  if (tend > tbeg && ((tend - 1 - tbeg) & 1)) {
#pragma unroll
    for (int j = 0; j < NJMAX; ++j) acc[j] = -acc[j];
  }

  // partial slab [split][tap][kpad][npad]: row i = chunk (i/4) channel i%4, col = co
#pragma unroll
  for (int j = 0; j < NJMAX; ++j) {
    const int blk = wave + 4 * j;
    if (j >= nj || blk >= tb.nblk) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * h;  // h = lane >> 5
      const int c4 = i >> 2;
      const int t = tb.tap[blk][c4];
      if (t < 0) continue;
      const int ci = ci_base + tb.ci0[blk][c4] + (i & 3);
      part[(((int64_t)split * T + t) * kpad + ci) * npad + co0 + (lane & 31)] = acc[j][r];
    }
  }
}

// ------------------------------------------------- 16x16x32 wgrad (X16) --
// CO (16 or 32): the Cout block of a workgroup; 16 for Cout <= 16 (the SwinUNETR's C = 12
// convs ran 12 of 32 columns)
// Same tiles, staging and partial slabs as k_conv3d_wgrad_x; the MFMA is
// v_mfma_f32_16x16x32_bf16: rows = 16 (tap, channel) -- one tap x 16 channels
// (CI 16) or two taps x 8 (CI 8), so 27 x 16 = 432 rows are 27 blocks with no
// padding, 7 / 7 / 7 / 6 over the 4 waves (the 32-row schedule pads to 448 and
// gives one wave 128 rows) -- cols = 16 Cout (two col blocks of the 32),
// k = 32 voxels = two W-rows of the 1 x 8 x 16 tile.
// k-group g (lanes 16g..16g+15) takes W-row 2ks + (g >> 1), w = 8s + 4(g & 1) + q
// for read s = 0, 1 and transpose row q: a 32-lane half then reads 8 consecutive
// halo positions (conflict-free on the channel-last [pos][CI] image), and B reads
// 8 consecutive voxels of the dy image whose 16-byte chunks are XOR-swizzled by
// voxel bit 2 (chunk ^= ((v >> 2) & 1) << 1) so those 8 rows of 64 B hit 64
// distinct banks.
// HR: height-sharded input (the stencil's rows h = -1 / h = H from Src2::rlo / rhi, as in
// k_conv3d_fwd_x); a separate instantiation
// ACT: x is y1 read through the fused input activation (x.al / x.de: lrelu(IN(y1)), the
// 32-channel convs of conv3d_fuses_act) -- a separate instantiation, so the plain kernels
// carry neither its per-tile coefficient loads nor its validity bookkeeping
template <int KD, int CI, int NS, int NJMAX, bool HR, int CO, bool ACT>
__global__ __launch_bounds__(256, 2) void k_conv3d_wgrad_x16(
    Src2 x, const float* __restrict__ dy, int lddy, float* __restrict__ part, Vol vol, int Cin,
    int kpad, int Cout, int npad, int tilesH, int tilesW, int ntiles, int tps, int nblk,
    const unsigned* __restrict__ xmx, const unsigned* __restrict__ ymx) {
  constexpr int HD = KD, HH = WX_TH + 2, HWD = WX_TW + 2;
  constexpr int NPOS = HD * HH * HWD;
  constexpr int T = KD * 9;
  constexpr int CQ = CI / 4;                              // float4 per halo position
  constexpr int PPOS = HH * HWD;                           // positions per depth plane
  constexpr int NP = (PPOS * CQ + 255) / 256;              // plane float4 per thread
  constexpr int NY = WX_TV * (CO / 4) / 256;            // dy float4 per thread (= 4)
  constexpr int NCB = CO / 16;                          // 16-wide col blocks (2)
  // operand planes; HF: two fp16 planes of the scaled operands (NS_F16, bf16split.h)
  constexpr int NPL = nplanes(NS);
  constexpr bool HF = NS == NS_F16;
  // R4 (f16x3, 3x3x3, SPFF_WXRING4): a 4-slot plane ring and two dy buffers (78 KB, still two
  // workgroups per CU), so the next tile's plane and dy go to slots the current tile does
  // not read: one barrier per tile instead of the write-after-read pair
  constexpr bool R4 = HF && KD == 3 && SPFF_WXRING4;
  constexpr int NSL = R4 ? 4 : KD;           // plane slots of the halo ring
  constexpr int NPOSA = NSL * PPOS;          // halo image positions per split plane
  constexpr int YB = NPL * WX_TV * CO;       // one dy buffer (elements)
  __shared__ __attribute__((aligned(16))) unsigned short Xs[NPL * NPOSA * CI];
  __shared__ __attribute__((aligned(16))) unsigned short Ys[(R4 ? 2 : 1) * YB];
  int ybuf = 0;  // dy buffer of the current tile (R4)
  // HF: x scaled by 2^ex (*xmx: max |x|), dy by 2^ey (*ymx: max |dy|)
  const int ex = HF ? f16_scale_exp(*xmx) : 0;
  const int ey = HF ? f16_scale_exp(*ymx) : 0;
  const float sx = exp2i(ex), sy = exp2i(ey);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int nci = kpad / CI, ncb = nci * (npad / CO);
  const int rk = blockIdx.x >> 3;
  const int nsp8 = gridDim.x / ncb;
  const int cbk = SPFF_XCDMAP ? rk % ncb : (int)(blockIdx.x / nsp8);
  const int split = SPFF_XCDMAP ? (rk / ncb) * 8 + (blockIdx.x & 7) : (int)(blockIdx.x % nsp8);
  if (split * tps >= ntiles) return;  // padding block (uniform)
  const int ci_base = (cbk % nci) * CI, co0 = (cbk / nci) * CO;
  const int D = vol.D, H = vol.H, W = vol.W;

  // row blocks of this wave: wave, wave + 4, ...; nj of them (uniform per wave)
  const int nj = (nblk - wave + 3) / 4;
  // lane-constant A address (elements; plane 0, k-step 0, read 0) per block: transpose
  // column block pq = rows 4pq..4pq+3 of the block = tap (16 blk + 4pq) / CI, channels
  // (16 blk + 4pq) % CI ..; transpose row q = voxel (W-row g >> 1, w 4(g & 1) + q)
  int aoff[NJMAX];
#pragma unroll
  for (int j = 0; j < NJMAX; ++j) {
    const int r0 = 16 * (wave + 4 * j) + 4 * pq;
    int t = r0 / CI;
    const int ch0 = r0 % CI;
    if (t >= T) t = 0;  // padding rows: any valid address (never stored)
    const int kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
    aoff[j] = ((kd * HH + kh + (g >> 1)) * HWD + kw + 4 * (g & 1) + q) * CI + ch0;
  }
  // B: voxel (W-row g >> 1, w 4(g & 1) + q), co 16 cb + 4 pq, chunk-swizzled
  const int bsw = CO == 32 ? (g & 1) << 1 : 0;  // (16-wide rows: 32 B, no swizzle)
  const int bv = (g >> 1) * WX_TW + 4 * (g & 1) + q;
  int boff[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
    boff[cb] = bv * CO + (((2 * cb + (pq >> 1)) ^ bsw) << 3) + 4 * (pq & 1);

  f32x4 acc[NJMAX][NCB];
#pragma unroll
  for (int j = 0; j < NJMAX; ++j)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[j][cb][r] = 0.f;

  // Rolling depth-plane halo: tiles run depth-fastest, so tile d0 + 1 of the same
  // (b, h, w) column needs only ONE new plane (gd = d0 + 1 + KD / 2) beside the KD - 1
  // it shares with tile d0.  Plane gd lives in slot (gd + 3) % KD of the halo image; the
  // register pipeline carries one plane (+ dy) per tile, and a column's first tile
  // stages its other KD - 1 planes synchronously.
  float4 hreg[NP], yreg[NY];
  float4 xal = make_float4(1.f, 1.f, 1.f, 1.f), xde = make_float4(0.f, 0.f, 0.f, 0.f);
  struct TileXY { int d0, b, h0, w0; };
  auto tile_xy = [&](int tile) {
    TileXY r;
    int t = tile;
    r.d0 = t % D; t /= D;
    const int twi = t % tilesW; t /= tilesW;
    const int thi = t % tilesH;
    r.b = t / tilesH;
    r.h0 = thi * WX_TH;
    r.w0 = twi * WX_TW;
    return r;
  };
  // (the fused input activation is applied at the store, not here: applied to each load as
  // it arrived, it made the prefetch wait for every load in turn before the MFMAs)
  unsigned hm = 0;  // bit k: hreg[k] is a valid (not padding) position
  auto load_plane = [&](const TileXY& tx, int gd, float4 (&r)[NP], unsigned& m) {
    m = 0;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = tid + 256 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < PPOS * CQ) {
        const int c4 = i % CQ, pos = i / CQ;
        const int hw = pos % HWD, hh = pos / HWD;
        const int b = tx.b, gh = tx.h0 + hh - 1, gw = tx.w0 + hw - 1;
        const int c = ci_base + 4 * c4;
        bool hin = (unsigned)gh < (unsigned)H;
        if constexpr (HR) hin = hin || (gh == -1 && x.rlo) || (gh == H && x.rhi);
        if ((unsigned)(gd + vol.dh) < (unsigned)(D + 2 * vol.dh) && hin &&
            (unsigned)gw < (unsigned)W && c < Cin && !((gd < 0 && x.zlo) || (gd >= D && x.zhi))) {
          const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
          const float* p =
              c < x.split ? x.p0 + vox * x.ld0 + c : x.p1 + vox * x.ld1 + (c - x.split);
          if constexpr (HR) {
            if ((unsigned)gh >= (unsigned)H)
              p = (gh < 0 ? x.rlo : x.rhi) + (((int64_t)b * D + gd) * W + gw) * x.ldr + c;
          }
          v = *reinterpret_cast<const float4*>(p);
          m |= 1u << k;
        }
      }
      r[k] = v;
    }
  };
  auto store_plane = [&](int gd, const float4 (&r)[NP], unsigned m) {
    unsigned short* dst = Xs + (R4 ? ((gd + 4) & 3) : ((gd + 3) % KD)) * PPOS * CI;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = tid + 256 * k;
      if (i < PPOS * CQ) {
        uint2 o[NPL];
        float4 v = r[k];
        if (ACT && ((m >> k) & 1u)) {  // lrelu(IN(y)) of valid positions (padding stays 0)
          v.x = v.x * xal.x + xde.x; v.x = v.x > 0.f ? v.x : 0.01f * v.x;
          v.y = v.y * xal.y + xde.y; v.y = v.y > 0.f ? v.y : 0.01f * v.y;
          v.z = v.z * xal.z + xde.z; v.z = v.z > 0.f ? v.z : 0.01f * v.z;
          v.w = v.w * xal.w + xde.w; v.w = v.w > 0.f ? v.w : 0.01f * v.w;
        }
        if constexpr (HF) v = make_float4(v.x * sx, v.y * sx, v.z * sx, v.w * sx);
        split4<NS>(v, o);
#pragma unroll
        for (int p = 0; p < NPL; ++p)
          *reinterpret_cast<uint2*>(dst + p * NPOSA * CI + 4 * i) = o[p];
      }
    }
  };
  auto fetch = [&](int tile) {
    const TileXY tx = tile_xy(tile);
    if constexpr (ACT) {
      // the fused activation's coefficients of this tile's batch and this thread's 4
      // channels, loaded unconditionally from a clamped channel, so no branch merge waits
      // for them here -- store_plane does
      const int c = ci_base + 4 * (tid % CQ);
      const int64_t o = (int64_t)tx.b * x.ld0 + (c < Cin ? c : 0);
      xal = *reinterpret_cast<const float4*>(x.al + o);
      xde = *reinterpret_cast<const float4*>(x.de + o);
    }
    load_plane(tx, tx.d0 + KD / 2, hreg, hm);
    const int b = tx.b, d0 = tx.d0, h0 = tx.h0, w0 = tx.w0;
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = tid + 256 * k;
      const int c4 = i % (CO / 4), kv = i / (CO / 4);
      const int gh = h0 + kv / WX_TW, gw = w0 + kv % WX_TW;
      const int c = co0 + 4 * c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gh < H && gw < W && c < Cout) {
        const int64_t vox = (((int64_t)b * D + d0) * H + gh) * W + gw;
        v = *reinterpret_cast<const float4*>(dy + vox * lddy + c);
      }
      yreg[k] = v;
    }
  };
  auto stash = [&](int d0, bool negate, int yb) {
    store_plane(d0 + KD / 2, hreg, hm);
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int i = tid + 256 * k;
      const int c4 = i % (CO / 4), kv = i / (CO / 4);
      uint2 o[NPL];
      const float ys = HF ? (negate ? -sy : sy) : (negate ? -1.f : 1.f);
      const float4 yv = make_float4(yreg[k].x * ys, yreg[k].y * ys, yreg[k].z * ys, yreg[k].w * ys);
      split4<NS>(yv, o);
      const int off = kv * CO + (((c4 >> 1) ^ (CO == 32 ? ((kv >> 2) & 1) << 1 : 0)) << 3) + 4 * (c4 & 1);
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        *reinterpret_cast<uint2*>(Ys + yb * YB + p * WX_TV * CO + off) = o[p];
    }
  };

  auto compute = [&](auto NJc, int d0) {
    constexpr int NJ = decltype(NJc)::value;
    // aoff[j] addresses plane kd as slot kd; tap kd reads gd = d0 + kd - KD / 2, in slot
    // (kd + rot) % KD with rot = (d0 - KD / 2 + 3) % KD
    // (R4: tap kd reads gd = d0 + kd - 1 in slot (gd + 4) & 3)
    constexpr int PL = PPOS * CI;
    const int rot = (d0 - KD / 2 + 3) % KD;
    int ab[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (R4) {
        const int kd = aoff[j] >= 2 * PL ? 2 : aoff[j] >= PL ? 1 : 0;
        ab[j] = aoff[j] + (((d0 + kd + 3) & 3) - kd) * PL;
      } else {
        ab[j] = aoff[j] + (aoff[j] >= (KD - rot) * PL ? (rot - KD) * PL : rot * PL);
      }
    }
    const unsigned short* Yc = Ys + (R4 ? ybuf * YB : 0);
    constexpr int KSU = NPL == 2 ? SPFF_WXUNROLL2 : SPFF_WXUNROLL;
#pragma unroll KSU
    for (int ks = 0; ks < WX_TH / 2; ++ks) {
      bf16x8 bq[NCB][NPL];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
          const unsigned short* yb = Yc + p * WX_TV * CO + 2 * ks * WX_TW * CO + boff[cb];
          bq[cb][p] = frag(tr_read(yb), tr_read(yb + 8 * CO));
        }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        bf16x8 aq[NPL];
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
          const unsigned short* xb = Xs + p * NPOSA * CI + 2 * ks * HWD * CI + ab[j];
          aq[p] = frag(tr_read(xb), tr_read(xb + 8 * CI));
        }
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          f32x4 c = acc[j][cb];
          if constexpr (NPL == 3) {
            c = mfma16x32<HF>(aq[1], bq[cb][1], c);
            c = mfma16x32<HF>(aq[0], bq[cb][2], c);
            c = mfma16x32<HF>(aq[2], bq[cb][0], c);
          }
          if constexpr (NPL >= 2) {
            c = mfma16x32<HF>(aq[0], bq[cb][1], c);
            c = mfma16x32<HF>(aq[1], bq[cb][0], c);
          }
          c = mfma16x32<HF>(aq[0], bq[cb][0], c);
          acc[j][cb] = c;
        }
      }
    }
  };

  const int tbeg = split * tps;
  const int tend = min(ntiles, tbeg + tps);
  // first tile of a column: its other planes d0 - KD / 2 .. d0 + KD / 2 - 1
  auto stage_column = [&](int tile, int d0) {
    const TileXY tx = tile_xy(tile);
#pragma unroll
    for (int hd = 0; hd < KD - 1; ++hd) {
      float4 r[NP];
      unsigned m;
      load_plane(tx, d0 + hd - KD / 2, r, m);
      store_plane(d0 + hd - KD / 2, r, m);
    }
  };
  if constexpr (R4) {
    // tile t computes from ring slots and dy buffer (t - tbeg) & 1, while tile t + 1's
    // plane / dy are fetched and stored to the slot / buffer it does not read; a new
    // column's two extra planes overwrite slots the tile before may read: one more barrier
    if (tbeg < tend) {
      fetch(tbeg);
      stage_column(tbeg, tbeg % D);
      stash(tbeg % D, false, 0);
    }
    for (int tile = tbeg; tile < tend; ++tile) {
      if (tile != tbeg) {
#pragma unroll
        for (int j = 0; j < NJMAX; ++j)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) acc[j][cb] = -acc[j][cb];
      }
      __syncthreads();  // this tile's plane / dy visible; every wave is past tile - 1
      const int d0 = tile % D;
      ybuf = (tile - tbeg) & 1;
      if (tile + 1 < tend) fetch(tile + 1);
      if (nj == NJMAX) compute(std::integral_constant<int, NJMAX>{}, d0);
      else if constexpr (NJMAX > 1) compute(std::integral_constant<int, NJMAX - 1>{}, d0);
      if (tile + 1 < tend) {
        const int d1 = (tile + 1) % D;
        if (d1 == 0) {
          __syncthreads();  // every wave is past this tile's reads of the ring
          stage_column(tile + 1, d1);
        }
        stash(d1, ((tile + 1 - tbeg) & 1) != 0, ybuf ^ 1);
      }
    }
  } else {
  if (tbeg < tend) fetch(tbeg);
  for (int tile = tbeg; tile < tend; ++tile) {
    // sign-alternating accumulation (conv3d_x.hip)
    if (tile != tbeg) {
#pragma unroll
      for (int j = 0; j < NJMAX; ++j)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc[j][cb] = -acc[j][cb];
    }
    __syncthreads();  // previous compute done reading LDS
    const int d0 = tile % D;
    if (KD > 1 && (tile == tbeg || d0 == 0)) stage_column(tile, d0);
    stash(d0, ((tile - tbeg) & 1) != 0, 0);
    __syncthreads();
    if (tile + 1 < tend) fetch(tile + 1);
    if (nj == NJMAX) compute(std::integral_constant<int, NJMAX>{}, d0);
    else if constexpr (NJMAX > 1) compute(std::integral_constant<int, NJMAX - 1>{}, d0);
  }
  }

  if (tend > tbeg && ((tend - 1 - tbeg) & 1)) {
#pragma unroll
    for (int j = 0; j < NJMAX; ++j)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[j][cb] = -acc[j][cb];
  }

  // partial slab [split][tap][kpad][npad]: output row 4 g + r of block blk = tap
  // (16 blk + row) / CI, channel (16 blk + row) % CI; col = co 16 cb + (lane & 15)
#pragma unroll
  for (int j = 0; j < NJMAX; ++j) {
    const int blk = wave + 4 * j;
    if (j >= nj || blk >= nblk) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * blk + 4 * g + r;
      const int t = row / CI;
      if (t >= T) continue;
      const int ci = ci_base + row % CI;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        part[(((int64_t)split * T + t) * kpad + ci) * npad + co0 + 16 * cb + (lane & 15)] =
            HF ? ldexpf(acc[j][cb][r], -(ex + ey)) : acc[j][cb][r];
    }
  }
}

// ------------------------------------------------------------------ host --
namespace {
// halo position offset of a tap inside the 1 x 8 x 16 tile's halo
int tap_pos(int t) {
  const int kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
  return (kd * (WX_TH + 2) + kh) * (WX_TW + 2) + kw;
}

WxTable make_table(int KD, int CI) {
  WxTable tb{};
  const int T = KD * 9;
  std::vector<int> taps;
  if (CI == 16) {
    // pair taps 2 per block, preferring halo offsets 4 apart (mod 8): the two
    // 16-lane groups of a half then cover disjoint 32-bank ranges
    std::vector<bool> used(T, false);
    for (int a = 0; a < T; ++a) {
      if (used[a]) continue;
      used[a] = true;
      int best = -1;
      for (int b = a + 1; b < T; ++b)
        if (!used[b] && (((tap_pos(b) - tap_pos(a)) % 8) + 8) % 8 == 4) { best = b; break; }
      if (best < 0)
        for (int b = a + 1; b < T; ++b)
          if (!used[b]) { best = b; break; }
      taps.push_back(a);
      taps.push_back(best);  // -1: half-empty block
      if (best >= 0) used[best] = true;
    }
    tb.nblk = (int)taps.size() / 2;
    for (int b = 0; b < tb.nblk; ++b)
      for (int c = 0; c < 8; ++c) {
        tb.tap[b][c] = (signed char)taps[2 * b + c / 4];
        tb.ci0[b][c] = (signed char)(4 * (c % 4));
      }
  } else {  // CI == 8: 4 taps per block
    tb.nblk = cdiv(T, 4);
    for (int b = 0; b < tb.nblk; ++b)
      for (int c = 0; c < 8; ++c) {
        const int t = 4 * b + c / 2;
        tb.tap[b][c] = (signed char)(t < T ? t : -1);
        tb.ci0[b][c] = (signed char)(4 * (c % 2));
      }
  }
  return tb;
}

struct WxPlan {
  int ci, co, kpad, npad, tilesH, tilesW, ntiles, nsplit, tps;
};
WxPlan wx_plan(Vol vol, int Cin, int Cout) {
  WxPlan p;
  p.ci = Cin <= 8 ? 8 : 16;
  p.co = (Cout <= 16 && SPFF_WX16) ? 16 : WX_CO;
  p.kpad = rup(Cin, p.ci);
  p.npad = rup(Cout, p.co);
  p.tilesH = cdiv(vol.H, WX_TH);
  p.tilesW = cdiv(vol.W, WX_TW);
  p.ntiles = vol.B * vol.D * p.tilesH * p.tilesW;
  const int nout = (p.kpad / p.ci) * (p.npad / p.co);
  // two workgroups per CU: aim at 2 rounds of 512, >= 4 tiles per workgroup
  int nsplit = std::max(1, cdiv(1024, nout));
  nsplit = std::min(nsplit, std::max(1, p.ntiles / 4));
  p.tps = cdiv(p.ntiles, nsplit);
  p.nsplit = cdiv(p.ntiles, p.tps);
  return p;
}
}  // namespace

// partial slabs, then (SPFF_MATH_F16X3) the two operand-scale slots [max |x|, max |dy|]
static size_t wx_main_bytes(Vol vol, int KD, int Cin, int Cout) {
  WxPlan p = wx_plan(vol, Cin, Cout);
  return ((size_t)p.nsplit * KD * 9 * p.kpad * p.npad * sizeof(float) + 255) & ~(size_t)255;
}
size_t conv3d_wgrad_x_ws_bytes(Vol vol, int KD, int Cin, int Cout) {
  return wx_main_bytes(vol, KD, Cin, Cout) + 256;
}

hipError_t conv3d_wgrad_x(const Src2& x, const float* dy, int lddy, float* dw, Vol vol, int KD,
                          int Cin, int Cout, int math, float* ws, hipStream_t s,
                          const unsigned* xmax, const unsigned* ymax) {
  if (lddy % 4) return hipErrorInvalidValue;
  WxPlan p = wx_plan(vol, Cin, Cout);
  const WxTable tb = make_table(KD, p.ci);
  dim3 grid(8 * cdiv(p.nsplit, 8) * (p.kpad / p.ci) * (p.npad / p.co));
#define SPFF_WX(KD_, CI_, NS_, NJ_)                                                            \
  hipLaunchKernelGGL((k_conv3d_wgrad_x<KD_, CI_, NS_, NJ_>), grid, dim3(256), 0, s, x, dy,     \
                     lddy, ws, vol, Cin, p.kpad, Cout, p.npad, p.tilesH, p.tilesW, p.ntiles,   \
                     p.tps, tb)
  const bool x3 = math == SPFF_MATH_BF16X3;
  const bool hf = math == SPFF_MATH_F16X3;
  unsigned* sl = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) +
                                             wx_main_bytes(vol, KD, Cin, Cout));
  if (hf) {  // operand maxima: the caller's precomputed slots, else computed here
    if (!SPFF_WX16) return hipErrorInvalidValue;
    if (!xmax || !ymax) {
      hipError_t e = spff::zero_async(sl, 2 * sizeof(unsigned), s);
      if (e != hipSuccess) return e;
    }
    if (!xmax) {
      hipError_t e = absmax_src(x, vol, Cin, true, sl, s);
      if (e != hipSuccess) return e;
      xmax = sl;
    }
    if (!ymax) {
      hipError_t e = absmax_src(src1(dy, lddy), vol, Cout, false, sl + 1, s);
      if (e != hipSuccess) return e;
      ymax = sl + 1;
    }
  }
  if (SPFF_WX16) {
    // 16-row blocks: nblk = ceil(T CI / 16); NJMAX = ceil(nblk / 4):
    // KD3/CI16 27 -> 7, KD3/CI8 14 -> 4, KD1/CI16 9 -> 3, KD1/CI8 5 -> 2
    const int nblk = cdiv(KD * 9 * p.ci, 16);
    // (the fused input activation only on 32-wide output tiles: conv3d_fuses_act's C = 32)
    if (x.al && p.co != 32) return hipErrorInvalidValue;
#define SPFF_WX16C(KD_, CI_, NS_, NJ_, HR_, CO_, ACT_)                                            \
  hipLaunchKernelGGL((k_conv3d_wgrad_x16<KD_, CI_, NS_, NJ_, HR_, CO_, ACT_>), grid, dim3(256),  \
                     0, s, x, dy, lddy, ws, vol, Cin, p.kpad, Cout, p.npad, p.tilesH, p.tilesW, \
                     p.ntiles, p.tps, nblk, xmax, ymax)
#define SPFF_WX16(KD_, CI_, NS_, NJ_)                                                          \
  do {                                                                                         \
    if (p.co == 16) {                                                                          \
      if (x.rows()) SPFF_WX16C(KD_, CI_, NS_, NJ_, true, 16, false);                           \
      else SPFF_WX16C(KD_, CI_, NS_, NJ_, false, 16, false);                                   \
    } else if (x.al) {                                                                         \
      if (x.rows()) SPFF_WX16C(KD_, CI_, NS_, NJ_, true, 32, true);                            \
      else SPFF_WX16C(KD_, CI_, NS_, NJ_, false, 32, true);                                    \
    } else {                                                                                   \
      if (x.rows()) SPFF_WX16C(KD_, CI_, NS_, NJ_, true, 32, false);                           \
      else SPFF_WX16C(KD_, CI_, NS_, NJ_, false, 32, false);                                   \
    }                                                                                          \
  } while (0)
    if (KD == 3) {
      if (p.ci == 16) {
        if (hf) SPFF_WX16(3, 16, NS_F16, 7);
        else if (x3) SPFF_WX16(3, 16, 2, 7);
        else SPFF_WX16(3, 16, 3, 7);
      } else {
        if (hf) SPFF_WX16(3, 8, NS_F16, 4);
        else if (x3) SPFF_WX16(3, 8, 2, 4);
        else SPFF_WX16(3, 8, 3, 4);
      }
    } else {
      if (p.ci == 16) {
        if (hf) SPFF_WX16(1, 16, NS_F16, 3);
        else if (x3) SPFF_WX16(1, 16, 2, 3);
        else SPFF_WX16(1, 16, 3, 3);
      } else {
        if (hf) SPFF_WX16(1, 8, NS_F16, 2);
        else if (x3) SPFF_WX16(1, 8, 2, 2);
        else SPFF_WX16(1, 8, 3, 2);
      }
    }
#undef SPFF_WX16
#undef SPFF_WX16C
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return conv3d_wgrad_reduce(ws, dw, p.nsplit, KD * 9, p.kpad, p.npad, Cin, Cout, s);
  }
  // NJMAX = ceil(nblk / 4): KD3/CI16 14 blocks -> 4, KD3/CI8 7 -> 2, KD1/CI16 5 -> 2, KD1/CI8 3 -> 1
  if (x.rows()) return hipErrorInvalidValue;  // (32x32x16 diagnostics kernel: no row halo)
  if (KD == 3) {
    if (p.ci == 16) { if (x3) SPFF_WX(3, 16, 2, 4); else SPFF_WX(3, 16, 3, 4); }
    else            { if (x3) SPFF_WX(3, 8, 2, 2);  else SPFF_WX(3, 8, 3, 2); }
  } else {
    if (p.ci == 16) { if (x3) SPFF_WX(1, 16, 2, 2); else SPFF_WX(1, 16, 3, 2); }
    else            { if (x3) SPFF_WX(1, 8, 2, 1);  else SPFF_WX(1, 8, 3, 1); }
  }
#undef SPFF_WX
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int T = KD * 9;
  return conv3d_wgrad_reduce(ws, dw, p.nsplit, T, p.kpad, p.npad, Cin, Cout, s);
}

}  // namespace spff
