// 3x3x3 convolution forward / input-gradient on the bf16 matrix cores with an
// fp32-faithful operand split ("bf16x6"), plus the layer-level dispatcher.
//
// Replaces nn.Conv3d(cin, cout, (ksd,3,3), padding=(ksd//2,1,1), bias=False)
// (reference models.py:616-618) forward and its input gradient, like
// k_conv3d_fwd in conv3d.hip, but at the bf16 MFMA rate (16x the f32 rate).
//
// Numerics.  Every fp32 operand is split exactly into three bf16 planes,
//   x = h + m + l (+ e),  h = bf16(x), m = bf16(x - h), l = bf16(x - h - m),
// |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, |e| <= 2^-25 |x|; both subtractions are exact
// in fp32.  The six products hh, hm, mh, hl, lh, mm are accumulated by the
// MFMA in fp32; the dropped terms ml + lm + ll + e are below 2^-24 |xy|, i.e.
// under half an fp32 ulp of each product -- the same accuracy class as the f32
// MFMA (an fp32 fma chain).  math = SPFF_MATH_BF16X3 keeps only h, l
// (x = h + l, |err| <= 2^-17) and hh, hl, lh: 2x faster, ~1e-5 relative.
//
// Structure (gfx950, 8 waves = 512 threads, one workgroup per CU):
//  * output tile 2 x 16 x 16 = 512 voxels x BN out channels; MFMA
//    v_mfma_f32_32x32x16_bf16, rows = voxels, cols = out channels,
//    k = (tap parity, 8 input channels): per input-channel chunk of 8 the 27
//    taps are walked as 14 tap pairs (lane half h takes tap 2j+h; tap 27 is a
//    zero weight row).
//  * LDS: halo [plane][pos][8ch] and weight slab [plane][tap][co][8ch], 16-byte
//    units read with ds_read_b128.  Lanes of one ds_read_b128 group must hit
//    distinct pos mod 16: a 32-row block covers two W-rows of 16 voxels and the
//    second row is rotated by 2 (tw = (r + 14) mod 16), which cancels the halo
//    row pitch 18 = 2 mod 16 -- conflict-free without padding.
//  * sign-alternating accumulation.  The bf16 MFMA adds products much smaller
//    than its fp32 accumulator (the hm / mh / hl / lh / mm terms) with a bias
//    toward -infinity of a few thousandths of an ulp per instruction (measured:
//    scripts/mfma_round4.hip, -0.75 ulp of rms(D) after 54 k-steps of 6 products;
//    the f32 MFMA's fma chain has none).  Small, but the same sign at every
//    output, so sums over voxels -- the InstanceNorm / gate reductions the
//    backward is made of -- keep it coherently.  Odd input-channel chunks carry
//    negated weights and the accumulator is negated at every chunk boundary, so
//    consecutive chunks' biases cancel.
//  * register-prefetch pipeline as in k_conv3d_fwd: chunk c+1's halo (fp32)
//    and weight slab (both fp32) are in flight during chunk c's MFMAs, and
//    are split into bf16 planes on their way into LDS.
#include "spff_internal.h"
#include "bf16split.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#ifndef SPFF_XDIAG
#define SPFF_XDIAG 0  // timing diagnostics only: 1 = no restaging, 2 = no MFMA loop,
                      // 3 = halo restaged but weights staged once, 4 = weights restaged,
                      // halo staged once (results wrong: kernel timing only)
#endif
#ifndef SPFF_XCDMAP
#define SPFF_XCDMAP 1  // 0: tile-fastest block order (A/B diagnostics)
#endif
#ifndef SPFF_XDFAST
#define SPFF_XDFAST 1  // 1: tiles depth-fastest (per batch sample), 0: W-fastest
#endif
#ifndef SPFF_X32T
// 1: 32-wide tiles are 4 x 16 x 16 voxels (MB 4), 0: 2 x 16 x 16 (MB 2).  Measured (with the
// depth-fastest order): 4-deep tiles -0.45 ms/step, but the 32-wide launches read 1.42 -> 2.35 GB
#define SPFF_X32T 0
#endif
#ifndef SPFF_X16
#define SPFF_X16 1  // 1: v_mfma_f32_16x16x32_bf16 tap-quad schedule, 0: 32x32x16 tap pairs
#endif
#ifndef SPFF_X32NW
// waves per 32-wide workgroup: 4 (default since round 3: a 2 x 8 x 16 tile in 78 KB of
// LDS, two workgroups per CU, so one's chunk-boundary staging overlaps the other's MFMAs
// -- the level-0 launches 6-8 % faster, -0.46 ms/step A/B) or 8 (one 2 x 16 x 16 tile,
// one workgroup per CU).  The 4-wave tiles change only the fused statistics' per-tile
// summation order; the round-2 sharded-test failure that held them back was a LeakyReLU
// input on its kink taking the other slope (an engine-vs-engine comparison without
// branch consistency), and both variants agree with the branch-consistent fp64 oracle
// (profiles/r02/ab_x32nw_branch_consistent.log; tests/test_gpu_sharded.py now judges that way)
#define SPFF_X32NW 4
#endif
#ifndef SPFF_X64NW
// waves per 64-wide f16x3 workgroup: 4 (a 2 x 8 x 16 tile in 80 KB of LDS -- two fp16 planes
// leave room for two workgroups per CU, as the 32-wide tiles) or 8 (one 2 x 16 x 16 tile)
#define SPFF_X64NW 4
#endif
#ifndef SPFF_X32D4
// 32-wide f16x3 tiles 4 x 8 x 16 voxels (4 waves x 8 row blocks, 75 KB, two workgroups per
// CU) instead of 2 x 8 x 16: 2.1 instead of 2.8 staged halo positions per output voxel
#define SPFF_X32D4 1
#endif
#ifndef SPFF_X32WG
// workgroups per CU the 16/32-wide f16x3 kernels are compiled for (their 52 KB image
// allows 3; 3 caps them at 168 VGPRs)
#define SPFF_X32WG 3
#endif
#ifndef SPFF_XSCALE_LATE
// f16x3 per-(tile, chunk) input scale: 1 = each wave publishes its max of the next chunk's
// halo late in the current chunk and the halo is split after the chunk-boundary barrier;
// 0 = a workgroup barrier in the middle of the chunk, the split beside the MFMAs
#define SPFF_XSCALE_LATE 0
#endif
#ifndef SPFF_XSCALEJ
// (SPFF_XSCALE_LATE 0) the k-step of the chunk at which the workgroup takes the next
// chunk's max and starts splitting its halo; -1 = the middle (NJ / 2)
#define SPFF_XSCALEJ -1
#endif
#ifndef SPFF_XIGLP
#define SPFF_XIGLP -1
#endif
#ifndef SPFF_XPRIO
#define SPFF_XPRIO 1
#endif
#ifndef SPFF_XFPIN
// 1: the next chunk's halo loads (and the fused activation's coefficients) are issued right
// after the chunk-boundary barrier, pinned there by a scheduling barrier.  Without it the
// compiler sank them to the last k-step before the mid-chunk scale barrier (ISA: the loads
// at MFMA 100-144 of the 144 before the vmcnt waits), so every wave waited out their whole
// latency at that barrier
#define SPFF_XFPIN 1
#endif
#ifndef SPFF_XPIPE
// 1: the 16/32-wide X16 k-loop is software-pipelined by one row block: the A fragments of
// row block rb + 1 (and, at the last row block, the next quad's B fragments and first A
// fragments) are read from LDS before row block rb's MFMAs, kept in that order by
// scheduling-group barriers.  Without it the compiler read each A fragment two MFMAs
// (32 cycles) before its use and waited lgkmcnt(0) there, i.e. most of the LDS latency
// exposed at every row block
#define SPFF_XPIPE 1
#endif
#ifndef SPFF_XPIPE64
#define SPFF_XPIPE64 1  // the XPIPE row-block pipeline in the 64-wide tiles too (A/B 35.53 -> 35.40; 0: 32-wide only)
#endif
#ifndef SPFF_XEARLYW
// 1: the first chunk's weight DMA is issued at the kernel start, before the first halo
// fetch, so its L2 latency overlaps the halo's HBM latency instead of following it at the
// first chunk-boundary barrier (in-kernel stamps: prologue 9-13 us per tile, of which
// 1-1.5 us that barrier and ~0.7 us the DMA issue)
#define SPFF_XEARLYW 1
#endif
#ifndef SPFF_XSTORE
// 1: the output tile goes through LDS (conflict-free [row][BN + 4] image in MFMA row order)
// and leaves as 16-byte row stores, instead of one 4-byte store per accumulator element
#define SPFF_XSTORE 1
#endif

#ifndef SPFF_XBSTAT
// 1: the input-gradient conv into da1 also forms the IN-backward sums of its output in the
// epilogue (BStat), replacing a RED_BWD_IN slab_reduce pass (0: that pass, A/B)
#define SPFF_XBSTAT 1
#endif

#ifndef SPFF_XSTAMP
// timing diagnostics only (variant builds): per workgroup of k_conv3d_fwd_x, s_memtime at
// kernel start, first MFMA, end of the k-loop and end, plus s_memrealtime at start / end
// and the CU it ran on, into g_xstamp; spff_debug_xstamps() copies them to the host
#define SPFF_XSTAMP 0
#endif

namespace spff {
#if SPFF_XSTAMP
constexpr int XSTAMP_N = 1 << 15, XSTAMP_W = 16;
__device__ unsigned long long g_xstamp[XSTAMP_N * XSTAMP_W];
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int rup(int a, int b) { return cdiv(a, b) * b; }

__device__ __forceinline__ unsigned short bfbits(__bf16 v) {
  return __builtin_bit_cast(unsigned short, v);
}
// exact split of x into NS bf16 planes (planes past NS-1 get the remainder)
template <int NS>
__device__ __forceinline__ void split_bf16(float x, unsigned short (&o)[NS]) {
  float r = x;
#pragma unroll
  for (int p = 0; p < NS; ++p) {
    const __bf16 b = (__bf16)r;
    o[p] = bfbits(b);
    r = r - (float)b;
  }
}

// 16x16x32 tap-quad schedule (X16): k = 4 lane groups x 8 channels, lane group g
// at its own tap.  A ds_read_b128 lane group mixes rows {0-3, 12-15} of k-group
// 0 (2) with rows 4-11 of k-group 1 (3): with the rows of a block mapped to the
// W-row's voxels as rows 4-11 -> even w, the rest -> odd w, every such group
// covers 16 distinct 16-byte bank quads as long as the two taps' halo offsets
// differ by an EVEN number of positions, i.e. have the same kw parity (offset
// = (kd HH + kh) HWD + kw with even HH, HWD).  Pairs are therefore formed within
// the even-kw and within the odd-kw taps; a leftover tap pairs with the zero
// padding row (weight index T), which reads its partner's position.
template <int KD>
struct XQuads {
  int nq = 0;
  signed char tap[32] = {};  // weight row per slot (T = the zero padding row)
  signed char src[32] = {};  // tap whose halo offset the slot reads
};
template <int KD>
__host__ __device__ constexpr XQuads<KD> x_quads() {
  XQuads<KD> q{};
  constexpr int T = KD * 9;
  int ev[27] = {}, od[27] = {}, ne = 0, no = 0;
  for (int t = 0; t < T; ++t) {
    if ((t % 3) % 2 == 0) ev[ne++] = t;
    else od[no++] = t;
  }
  int pa[32] = {}, pb[32] = {}, np = 0;
  for (int i = 0; i + 1 < ne; i += 2) { pa[np] = ev[i]; pb[np] = ev[i + 1]; ++np; }
  for (int i = 0; i + 1 < no; i += 2) { pa[np] = od[i]; pb[np] = od[i + 1]; ++np; }
  if (ne % 2) { pa[np] = ev[ne - 1]; pb[np] = -1; ++np; }
  if (no % 2) { pa[np] = od[no - 1]; pb[np] = -1; ++np; }
  if (np % 2) { pa[np] = -2; pb[np] = -2; ++np; }  // (pad, pad)
  q.nq = np / 2;
  for (int i = 0; i < np; ++i) {
    const int a = pa[i], b = pb[i];
    q.tap[2 * i] = (signed char)(a >= 0 ? a : T);
    q.src[2 * i] = (signed char)(a >= 0 ? a : 0);
    q.tap[2 * i + 1] = (signed char)(b >= 0 ? b : T);
    q.src[2 * i + 1] = (signed char)(b >= 0 ? b : (a >= 0 ? a : 0));
  }
  return q;
}
// ------------------------------------------------------------ weight pack --
// The weights are split into their NS bf16 planes once per launch, here, in the
// exact LDS image the conv kernel reads, so its weight staging is a plain
// global->LDS DMA copy: wp[nb][kc][plane][T2][BN] units of 8 bf16 (16 B), unit
// element e = gemm k = kc*8 + e, gemm n = nb*BN + co; fwd: k = ci, n = co;
// dgrad: k = co, n = ci with the tap flipped.  Taps >= T and padded k/n are zero.
// Odd chunks kc are stored NEGATED (sign-alternating accumulation, see below).
template <int NS>
__device__ __forceinline__ void pack_units(const float* __restrict__ w, uint4* __restrict__ wp,
                                           int Cout, int Cin, int T, int T2, int nkc, int npad,
                                           int BN, int dgrad, float sw, int64_t i0, int64_t step) {
  constexpr int NP = nplanes(NS);
  const int64_t total = (int64_t)(npad / BN) * nkc * T2 * BN;
  for (int64_t i = i0; i < total; i += step) {
    const int co = (int)(i % BN);
    const int tap = (int)((i / BN) % T2);
    const int kc = (int)((i / ((int64_t)BN * T2)) % nkc);
    const int nb = (int)(i / ((int64_t)BN * T2 * nkc));
    const int n = nb * BN + co;
    unsigned short s[8][NP];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = kc * 8 + e;
      float v = 0.f;
      if (tap < T) {
        if (!dgrad) {
          if (k < Cin && n < Cout) v = w[((int64_t)n * Cin + k) * T + tap];
        } else {
          if (k < Cout && n < Cin) v = w[((int64_t)k * Cin + n) * T + (T - 1 - tap)];
        }
      }
      v = (kc & 1) ? -v : v;
      if constexpr (NS == NS_F16) {
        unsigned pl[2];
        split_pair_f16(v * sw, 0.f, pl);
        s[e][0] = (unsigned short)pl[0];
        s[e][1] = (unsigned short)pl[1];
      } else {
        split_bf16<NS>(v, s[e]);
      }
    }
    const int64_t base = (((int64_t)nb * nkc + kc) * NP) * T2 * BN + (int64_t)tap * BN + co;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      uint4 u;
      u.x = (unsigned)s[0][p] | ((unsigned)s[1][p] << 16);
      u.y = (unsigned)s[2][p] | ((unsigned)s[3][p] << 16);
      u.z = (unsigned)s[4][p] | ((unsigned)s[5][p] << 16);
      u.w = (unsigned)s[6][p] | ((unsigned)s[7][p] << 16);
      wp[base + (int64_t)p * T2 * BN] = u;
    }
  }
}
template <int NS>
__global__ void k_conv_pack_x(const float* __restrict__ w, uint4* __restrict__ wp, int Cout,
                              int Cin, int T, int T2, int nkc, int npad, int BN, int dgrad,
                              const unsigned* __restrict__ wmx) {
  // NS_F16: the weights scaled by 2^e (*wmx: max |w|), fp16 planes
  const float sw = NS == NS_F16 ? exp2i(f16_scale_exp(*wmx)) : 1.f;
  pack_units<NS>(w, wp, Cout, Cin, T, T2, nkc, npad, BN, dgrad, sw,
                 blockIdx.x * (int64_t)blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}
// Every conv image of a plan in one launch (conv3d_pack_many): the job table travels as
// the kernel argument; job j owns blocks [blk0, blk0 + nblk).
template <int NS>
__global__ __launch_bounds__(256) void k_conv_pack_many(PackJobs J) {
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.j[j + 1].blk0) ++j;
  const PackJob& q = J.j[j];
  const float sw = NS == NS_F16 ? exp2i(f16_scale_exp(*q.wmx)) : 1.f;
  pack_units<NS>(q.w, q.wp, q.Cout, q.Cin, q.T, q.T2, q.nkc, q.npad, q.BN, q.dgrad, sw,
                 (int64_t)((int)blockIdx.x - q.blk0) * 256 + threadIdx.x, (int64_t)q.nblk * 256);
}

// ------------------------------------------------------------ fwd / dgrad --
namespace {
constexpr int XT_D = 2, XT_H = 16, XT_W = 16, XT_THREADS = 512;
// NW waves x MB 32-row blocks per wave: tile TD x TH x 16 voxels with TD TH = 2 NW MB
// (TD = 2 except the 32-wide 16x16x32 tiles, SPFF_X32T: 4 x 16 x 16)
template <int KD, int TD, int TH>
__host__ __device__ constexpr int xt_npos() {
  return (TD + KD - 1) * (TH + 2) * (XT_W + 2);
}
template <int KD>
__host__ __device__ constexpr int xt_t2() {
  return (KD * 9 + 1) & ~1;
}
template <int BN, int KD, int NS, int TD, int TH>
constexpr size_t xt_lds_bytes() {
  // operand images; the epilogue reuses the space for the output tile [TD TH 16][BN + 4]
  // fp32 plus the fused statistics' two [NW][BN] partial-sum tables
  const size_t ops = (size_t)nplanes(NS) * (xt_npos<KD, TD, TH>() + xt_t2<KD>() * BN) * 16;
  const size_t out = SPFF_XSTORE ? (size_t)TD * TH * 16 * (BN + 4) * 4 + 16 * BN * 4 : 0;
  return ops > out ? ops : out;
}
// tile depth of a BN-wide launch (host side: launches, fused-statistics layout)
constexpr bool xt_d4(int BN, int NS) {
  return BN == 32 && NS == NS_F16 && SPFF_X16 && SPFF_X32D4 && !SPFF_X32T;
}
constexpr int xt_td(int BN, int NS) {
  return ((BN == 32 && SPFF_X16 && SPFF_X32T) || xt_d4(BN, NS)) ? 4 : XT_D;
}
constexpr int xt_mb(int BN, int NS) {
  return ((BN == 32 && SPFF_X16 && SPFF_X32T) || xt_d4(BN, NS)) ? 4 : 2;
}
// waves of a BN-wide workgroup (4-wave 32-wide tiles: SPFF_X32NW, 2-deep tiles only)
// (16-wide tiles, Cout <= 16 -- the SwinUNETR's C = 12 convs: also 4 waves, 2 WGs / CU)
// (64-wide f16x3 tiles: SPFF_X64NW)
constexpr int xt_nw(int BN, int NS) {
  return (BN <= 32 && SPFF_X16 && !(BN == 32 && SPFF_X32T)) ? SPFF_X32NW
         : (BN == 64 && NS == NS_F16 && SPFF_X16)             ? SPFF_X64NW
                                                                : 8;
}
}  // namespace
// template plane count of a math mode
static int ns_of(int math) {
  return math == SPFF_MATH_F16X3 ? NS_F16 : math == SPFF_MATH_BF16X3 ? 2 : 3;
}

// MFMAs per multiply-add of an NP-plane operand pair (the split products)
__host__ __device__ constexpr int nprod(int np) { return np == 3 ? 6 : np == 2 ? 3 : 1; }

// MFMA row r (0..15) of a 16-row block -> w within the W-row (see x_quads)
__device__ __forceinline__ int x16_w(int r) {
  return (r >= 4 && r < 12) ? 2 * (r - 4) : (r < 4 ? 2 * r + 1 : 2 * r - 15);
}

// HR: height-sharded input -- stencil rows h = -1 / h = H read the neighbours' boundary
// rows (Src2::rlo / rhi; zero where null) instead of zero padding (hshard.hip).  A
// separate instantiation, so the unsharded kernels' register budget is unchanged.
template <int BN, int KD, int NS, int MB, int NW, bool X16, int TD, bool HR>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 1 : (BN <= 32 && NS == NS_F16 && TD == 2 ? SPFF_X32WG : 2)) void k_conv3d_fwd_x(
    Src2 x, const uint4* __restrict__ wp, Dst2 y, Vol vol, int Cin, int nkc, int Cout, int npad,
    int tilesD, int tilesH, int tilesW, float* __restrict__ part, int kps,
    float* __restrict__ stats, int ntiles, int td0, int tds, int th0, int ths,
    const unsigned* __restrict__ wmx, BStat bst) {
  constexpr int XT_THREADS = NW * 64;
#if SPFF_XSTAMP
  const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long st_r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st_t1 = 0, st_t2 = 0, st_pa = 0, st_pb = 0, st_pc = 0, st_c1a = 0,
                     st_c1b = 0, st_c1c = 0, st_c1d = 0;
#define XST(v) (v = __builtin_amdgcn_s_memtime())
#else
#define XST(v)
#endif
  // planes per operand; HF: two fp16 planes of the scaled operands (NS_F16, bf16split.h)
  constexpr int NP = nplanes(NS);
  constexpr bool HF = NS == NS_F16;
  constexpr int TH = X16 ? 2 * NW * MB / TD : NW * MB, TW = XT_W;
  static_assert(X16 || TD == 2, "32x32x16 schedule: 2-deep tiles");
  constexpr int HH = TH + 2, HWD = TW + 2;
  constexpr int NPOS = xt_npos<KD, TD, TH>();
  constexpr int T = KD * 9, T2 = xt_t2<KD>();
  // MFMA blocking: 32x32x16 -- MB 32-row blocks x BN/32 col blocks per wave, a k-step
  // per tap pair; 16x16x32 -- 2 MB 16-row blocks x BN/16, a k-step per tap quad
  constexpr int RB = X16 ? 2 * MB : MB, CB = X16 ? BN / 16 : BN / 32;
  constexpr int NCOL = X16 ? 16 : 32, NREG = X16 ? 4 : 16;
  constexpr XQuads<KD> QT = x_quads<KD>();
  constexpr int NJ = X16 ? QT.nq : T2 / 2;
  using AccT = typename std::conditional<X16, f32x4, f32x16>::type;
  constexpr int NHX = NPOS * 2;  // halo float4 per chunk (8 channels = 2 float4)
  constexpr int RH = (NHX + XT_THREADS - 1) / XT_THREADS;
  constexpr int NWU = NP * T2 * BN;  // pre-split weight units (16 B) per chunk
  static_assert(NWU % 64 == 0, "weight image must be whole 1 KiB DMA pieces");
  static_assert(!X16 || TD * TH == NW * RB, "X16: one W-row per 16-row block");
  // the epilogue's two fused-statistics tables [NW][CB][NCOL] (= NW BN floats each) live in
  // the 16 BN floats xt_lds_bytes reserves beside the output tile
  static_assert(NW <= 8, "fused-statistics tables: at most 8 waves");
  // the k-step from which the next chunk's halo is split (HF: after its block max), and the
  // halo float4 split per k-step from there on
  constexpr int J0 = (NS == NS_F16 && SPFF_XSCALEJ >= 0 && SPFF_XSCALEJ < NJ) ? SPFF_XSCALEJ : NJ / 2;
  constexpr int SPJ = (RH + (NJ - J0) - 1) / (NJ - J0);
  constexpr int NPC = NWU / 64;
  extern __shared__ uint4 lds4[];
  uint4* Xs = lds4;               // [NP][NPOS]
  uint4* Ws = lds4 + NP * NPOS;   // [NP][T2][BN]
  // HF: the packed weights are scaled by 2^ew (*wmx: max |w| of the tensor); the input by a
  // scale of its own per (tile, 8-channel chunk): 2^exc from the max |element| of exactly
  // the halo chunk this workgroup stages (block max below), so an element is flushed to
  // the fp16 subnormal floor only below 2^-39 of the largest element of its own tile's
  // halo chunk -- not of the whole tensor (f16_scale_exp, bf16split.h).  The accumulator
  // holds the products in units of 2^(exc + ew) and is rescaled (exact: a power of two)
  // when the next chunk's exponent differs.
  const int ew = HF ? f16_scale_exp(*wmx) : 0;
  int exc = 0;       // exponent of the chunk being accumulated
  int exn = 0;       // exponent of the chunk in the registers (the next one)
  float sx = 1.f;    // 2^exn: the scale the halo split applies
  __shared__ unsigned smx[2][NW];  // per-wave max |x| bits of a chunk (parity slots)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int khalf = lane >> 5, l32 = lane & 31, kg = lane >> 4, l16 = lane & 15;
  const int lcol = X16 ? l16 : l32;
  // XCD-aware order: blocks b and b + 8 share an XCD (and its L2), so XCD group
  // b % 8 walks a contiguous run of tiles, the npad / BN output-channel blocks of a
  // tile back to back -- neighbouring tiles' halos and a tile's input for its other
  // channel blocks are then L2 hits instead of HBM re-reads
  const int nnb = npad / BN;
  const int per = (ntiles + 7) >> 3;
  const int grp = blockIdx.x & 7, rk = blockIdx.x >> 3;
  const int tile = SPFF_XCDMAP ? grp * per + rk / nnb : (int)(blockIdx.x % (8 * per));
  const int nbk = SPFF_XCDMAP ? rk % nnb : (int)(blockIdx.x / (8 * per));
  if (tile >= ntiles) return;  // padding block (uniform: the whole workgroup)
  int t = tile;
  int twi, thi, tdi;
  if (SPFF_XDFAST) {
    // depth-fastest: the ~32 tiles an XCD runs at once are D-neighbours, whose halos
    // share KD - 1 planes -- those are L2 hits instead of a later HBM re-read
    tdi = t % tilesD; t /= tilesD;
    twi = t % tilesW; t /= tilesW;
    thi = t % tilesH; t /= tilesH;
  } else {
    twi = t % tilesW; t /= tilesW;
    thi = t % tilesH; t /= tilesH;
    tdi = t % tilesD; t /= tilesD;
  }
  const int b = t;
  tdi = td0 + tdi * tds;  // depth-tile subset (sharded halo overlap): td0 + k tds, k < tilesD
  if constexpr (HR) thi = th0 + thi * ths;  // H-tile subset (height-sharded overlap)
  const int d0 = tdi * TD, h0 = thi * TH, w0 = twi * TW;
  const int n0 = nbk * BN;
  const int D = vol.D, H = vol.H, W = vol.W;
  const uint4* wsrc = wp + (int64_t)nbk * nkc * NWU;

  // voxel of MFMA row r in row block q (q = wave*RB + rb)
  auto vrow = [](int q, int r, int& td, int& th, int& tw) {
    if constexpr (X16) {
      td = q / TH;
      th = q % TH;
      tw = x16_w(r);
    } else {
      td = q / (TH / 2);
      th = 2 * (q % (TH / 2)) + (r >> 4);
      tw = r < 16 ? r : ((r + 14) & 15);
    }
  };
  // output register r of this lane -> MFMA row
  auto orow = [&](int r) {
    return X16 ? 4 * kg + r : (r & 3) + 8 * (r >> 2) + 4 * khalf;
  };
  int hpos[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    int td, th, tw;
    vrow(wave * RB + rb, X16 ? l16 : l32, td, th, tw);
    hpos[rb] = (td * HH + th) * HWD + tw;
  }

  AccT acc[RB][CB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int r = 0; r < NREG; ++r) acc[rb][cb][r] = 0.f;

  // halo of the next chunk: fp32 loads in flight during this chunk's first
  // MFMAs, split into bf16 planes half-way through it (VALU beside the MFMAs),
  // stored to LDS right after the chunk boundary
  float4 hreg[RH];
  uint2 hs[RH][NP];
  unsigned hvalid = 0;  // bit k: hreg[k] is in bounds (else it is zeroed at the split)
  int fkc = 0;          // chunk of the registers in flight
  // PRE (16/32-wide tiles, no boundary rows): the chunk-invariant part of each halo float4's
  // address -- its voxel and spatial validity -- computed once, not per chunk (the position
  // decomposition and bounds are ~20 VALU per float4 beside MFMAs that now take half the
  // cycles with two fp16 planes); the 64-wide kernel has no registers to spare
  constexpr bool PRE = BN <= 32 && !HR;
  int pvox[PRE ? RH : 1];  // (voxel indices < 2^31: launch_fwd_xh checks)
  unsigned pok = 0;
  if constexpr (PRE) {
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      const int i = tid + XT_THREADS * k;
      const int pos = (i < NHX ? i : 0) >> 1;
      const int hw = pos % HWD, t2 = pos / HWD, hh = t2 % HH, hd = t2 / HH;
      const int gd = d0 + hd - KD / 2, gh = h0 + hh - 1, gw = w0 + hw - 1;
      const bool ok = i < NHX && (unsigned)(gd + vol.dh) < (unsigned)(D + 2 * vol.dh) &&
                      (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W &&
                      !((gd < 0 && x.zlo) || (gd >= D && x.zhi));
      pvox[k] = ok ? ((b * D + gd) * H + gh) * W + gw : 0;
      pok |= ok ? (1u << k) : 0u;
    }
  }
  // the chunk's 8 (al, de) pairs of the fused input activation, loaded once per chunk from
  // uniform addresses (scalar loads) and selected per lane: a thread's 4 channels are the
  // lower or upper half (XT_THREADS is even: q = tid & 1 for all k).  Loaded per halo float4
  // they became 9 dependent vector-memory round trips, each behind a vmcnt(0)
  auto act_coef_kc = [&](int kc, float (&a)[4], float (&e)[4]) {
    const int64_t o = __builtin_amdgcn_readfirstlane((int)((int64_t)b * x.ld0 + kc * 8));
    const float* ap = x.al + o;
    const float* dp = x.de + o;
    const bool hi = tid & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float alo = ap[j], ahi = ap[4 + j], elo = dp[j], ehi = dp[4 + j];
      a[j] = hi ? ahi : alo;
      e[j] = hi ? ehi : elo;
    }
  };
  // (SPFF_XFPIN, HF 32-wide tiles) every chunk's coefficients staged in LDS once per tile
  // (float4 q = the 4 channels 4q..4q+3): prep_max reads them there instead of issuing global
  // loads of its own (which the scale barrier then waited for, or -- preloaded into registers
  // with the halo -- which the register allocator waited for at the chunk start)
  constexpr int XCF = 32;  // float4s per table: channels < 128 (launch_fwd_x checks)
  __shared__ float4 scf[2][XCF];
  // live = false: a dummy fetch (every quad invalid, loads from clamped addresses) after the
  // last chunk, so that the fetch is unconditional: a conditional one left the registers'
  // old and new values to merge, and the compiler waited for the first loads at the merge
  auto fetch = [&](int kc, bool live = true) {
    hvalid = 0;
    fkc = kc;
    if constexpr (PRE) {
      // a thread's channel quad q = tid & 1 is the same for every k (XT_THREADS is even)
      const int cq = kc * 8 + 4 * (tid & 1);
      const bool cok = live && cq < Cin;
#pragma unroll
      for (int k = 0; k < RH; ++k) {
        const bool ok = ((pok >> k) & 1u) && cok;
        const int c = ok ? cq : 0;
        const bool s0 = c < x.split;
        const float* src = s0 ? x.p0 : x.p1;
        const int64_t ld = s0 ? x.ld0 : x.ld1;
        hreg[k] = *reinterpret_cast<const float4*>(src + (int64_t)(ok ? pvox[k] : 0) * ld +
                                                   (s0 ? c : c - x.split));
        hvalid |= ok ? (1u << k) : 0u;
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      const int i = tid + XT_THREADS * k;
      // unconditional load from a clamped address: no exec-masked branch and no
      // register copy of the result that would wait for it before the MFMAs
      const int q = i & 1, pos = (i < NHX ? i : 0) >> 1;
      const int hw = pos % HWD, t2 = pos / HWD, hh = t2 % HH, hd = t2 / HH;
      const int gd = d0 + hd - KD / 2, gh = h0 + hh - 1, gw = w0 + hw - 1;
      bool hin = (unsigned)gh < (unsigned)H;
      bool hrow = false;
      if constexpr (HR) {
        hrow = (gh < 0 && x.rlo) || (gh >= H && x.rhi);
        hin = hin || hrow;
      }
      const bool ok = live && i < NHX && (unsigned)(gd + vol.dh) < (unsigned)(D + 2 * vol.dh) &&
                      hin && (unsigned)gw < (unsigned)W &&
                      kc * 8 + 4 * q < Cin && !((gd < 0 && x.zlo) || (gd >= D && x.zhi));
      const int64_t vox = ok ? (((int64_t)b * D + gd) * H + gh) * W + gw : 0;
      // two-source select on the operands (v_cndmask), not on two address
      // expressions (which the compiler turns into divergent branches)
      const int c = ok ? kc * 8 + 4 * q : 0;
      const bool s0 = c < x.split;
      const float* src = s0 ? x.p0 : x.p1;
      const int64_t ld = s0 ? x.ld0 : x.ld1;
      int64_t off = vox * ld + (s0 ? c : c - x.split);
      if constexpr (HR) {
        if (hrow) {  // the neighbour's boundary row: [b][d][w][ldr], channel c
          src = gh < 0 ? x.rlo : x.rhi;
          off = (((int64_t)b * D + gd) * W + gw) * x.ldr + c;
        }
      }
      hreg[k] = *reinterpret_cast<const float4*>(src + off);
      hvalid |= ok ? (1u << k) : 0u;
    }
  };
  // HF: the fused input activation (32-wide tiles) and the zero padding applied to the
  // prefetched halo in place, and this thread's max |element| of it
  auto prep_max = [&]() {
    float m = 0.f;
    float ca[4] = {1.f, 1.f, 1.f, 1.f}, ce[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (BN == 32) if (x.al) {
      if constexpr (HF && SPFF_XFPIN) {
        const float4 fa = scf[0][2 * fkc + (tid & 1)], fe = scf[1][2 * fkc + (tid & 1)];
        ca[0] = fa.x; ca[1] = fa.y; ca[2] = fa.z; ca[3] = fa.w;
        ce[0] = fe.x; ce[1] = fe.y; ce[2] = fe.z; ce[3] = fe.w;
      } else {
        act_coef_kc(fkc, ca, ce);
      }
    }
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      const bool ok = (hvalid >> k) & 1u;
      float4 v = hreg[k];
      if constexpr (BN == 32) if (x.al) {
        float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = r[j] * ca[j] + ce[j];
          r[j] = fmaxf(t, 0.01f * t);
        }
        v = make_float4(r[0], r[1], r[2], r[3]);
      }
      if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
      hreg[k] = v;
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    return m;
  };
  // HF: the workgroup's max over the chunk (every thread's prep_max) -> its scale exponent.
  // Contains a workgroup barrier: call uniformly.
  auto wave_max_store = [&](float m, int slot) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) smx[slot][wave] = __float_as_uint(m);
  };
  auto read_scale = [&](int slot) {
    unsigned mb = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) mb = max(mb, smx[slot][w]);
    return f16_scale_exp(__builtin_amdgcn_readfirstlane(mb));
  };
  auto block_scale = [&](float m, int slot) {
    wave_max_store(m, slot);
    __syncthreads();
    return read_scale(slot);
  };
  auto split_one = [&](int k) {
    if constexpr (HF) {  // (prep_max has applied the activation and the padding)
      const float4 v = hreg[k];
      split4_pk<NS>(make_float4(v.x * sx, v.y * sx, v.z * sx, v.w * sx), hs[k]);
      return;
    }
    const bool ok = (hvalid >> k) & 1u;
    float4 v = hreg[k];
    // fused input activation (zero padding stays zero: applied to valid only).  Compiled
    // for the 32-wide tiles only: the level-0 convs (C = 32) carry 55 % of the fused
    // bytes, and in the 64-wide kernel the extra registers spill (256 VGPRs)
    if constexpr (BN == 32) if (x.al) {
      // the chunk's 8 (al, de) pairs are workgroup-uniform (scalar loads); a thread's 4
      // channels are the lower or upper half (XT_THREADS is even: q = tid & 1 for all k)
      const float* ap = x.al + (int64_t)b * x.ld0 + fkc * 8;
      const float* dp = x.de + (int64_t)b * x.ld0 + fkc * 8;
      const bool hi = tid & 1;
      float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = hi ? ap[4 + j] : ap[j], e = hi ? dp[4 + j] : dp[j];
        const float t = r[j] * a + e;
        r[j] = fmaxf(t, 0.01f * t);  // = lrelu(t, 0.01) (t > 0 ? t : 0.01 t) for finite t
      }
      v = make_float4(r[0], r[1], r[2], r[3]);
    }
    if constexpr (BN <= 32 || HF) {
      // packed pair split (bf16split.h): -0.5 to -3 % on the 16/32-wide launches; the
      // 64-wide kernel (255 VGPRs) measured +1 to +3 % with it and keeps the per-value form
      if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (HF) v = make_float4(v.x * sx, v.y * sx, v.z * sx, v.w * sx);
      split4_pk<NS>(v, hs[k]);
    } else {
      unsigned short s0[NS], s1[NS], s2[NS], s3[NS];
      split_bf16<NS>(ok ? v.x : 0.f, s0);
      split_bf16<NS>(ok ? v.y : 0.f, s1);
      split_bf16<NS>(ok ? v.z : 0.f, s2);
      split_bf16<NS>(ok ? v.w : 0.f, s3);
#pragma unroll
      for (int p = 0; p < NS; ++p) {
        hs[k][p].x = (unsigned)s0[p] | ((unsigned)s1[p] << 16);
        hs[k][p].y = (unsigned)s2[p] | ((unsigned)s3[p] << 16);
      }
    }
  };
  // store halo float4 k's planes (hs[k]) into the LDS image
  auto store_one = [&](int k) {
    const int i = tid + XT_THREADS * k;
    if (i < NHX) {
#pragma unroll
      for (int p = 0; p < NP; ++p)
        reinterpret_cast<uint2*>(Xs + p * NPOS + (i >> 1))[i & 1] = hs[k][p];
    }
  };
  auto stash = [&](int kc, bool first, bool halo = true, bool wts = true) {
#pragma unroll
    for (int k = 0; k < RH; ++k) {
      if (!halo) break;
      if (SPFF_XDIAG == 4 && !first) break;
      const int i = tid + XT_THREADS * k;
      if (i < NHX) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          reinterpret_cast<uint2*>(Xs + p * NPOS + (i >> 1))[i & 1] = hs[k][p];
      }
    }
    // weights: 1 KiB pieces global -> LDS, no registers (issued after the halo
    // stores: the compiler orders LDS stores behind an outstanding LDS-DMA)
    const uint4* src = wsrc + (int64_t)kc * NWU + lane;
#pragma unroll
    for (int k = 0; k < (NPC + NW - 1) / NW; ++k) {
      if (!wts) break;
      if (SPFF_XDIAG == 3 && !first) break;
      const int pc = wave + k * NW;
      if (k * NW + NW <= NPC || pc < NPC)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 64),
                                         (__attribute__((address_space(3))) void*)(Ws + pc * 64),
                                         16, 0, 0);
    }
  };
  auto toff_of = [](int tp) { return ((tp / 9) * HH + (tp / 3) % 3) * HWD + tp % 3; };

  // split-K (small volumes): this workgroup reduces chunks [kc0, kc1) only and
  // writes fp32 partial sums that k_splitk_reduce adds in a fixed order
  const int kc0 = part ? blockIdx.z * kps : 0;
  const int kc1 = part ? min(nkc, kc0 + kps) : nkc;
  // (SPFF_XEARLYW) the first chunk's weights first: the Ws image is free at the start
  if constexpr (SPFF_XEARLYW) stash(kc0, true, false, true);
  fetch(kc0);
  // (after the halo loads are in flight: these loads overlap them)
  if constexpr (BN == 32 && HF && SPFF_XFPIN) if (x.al) {
    for (int i = tid; i < 2 * XCF; i += XT_THREADS) {
      const int q = i % XCF, t = i / XCF;
      float4 v = make_float4(t ? 0.f : 1.f, t ? 0.f : 1.f, t ? 0.f : 1.f, t ? 0.f : 1.f);
      if (q < 2 * nkc) v = *reinterpret_cast<const float4*>((t ? x.de : x.al) + (int64_t)b * x.ld0 + 4 * q);
      scf[t][q] = v;
    }
    __syncthreads();
  }
  if constexpr (HF) {
    const float m0 = prep_max();
    XST(st_pa);
    exc = exn = block_scale(m0, kc0 & 1);
    XST(st_pb);
    sx = exp2i(exn);
  }
#pragma unroll
  for (int k = 0; k < RH; ++k) split_one(k);
  // the second-dispatched half of the workgroup loses every issue arbitration
  // on its SIMD: one static priority bump (MI355X_MICROARCH "two waves per SIMD")
  if (SPFF_XPRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  for (int kc = kc0; kc < kc1; ++kc) {
    constexpr bool LATE = HF && SPFF_XSCALE_LATE;
    if (LATE && kc != kc0) {
      // every wave is past chunk kc - 1's MFMAs and has published its max of chunk kc's
      // halo: the chunk's scale (capped 2^64 above the current one, so the rescaled
      // accumulator cannot overflow: |acc| < 2^40 in these units), then the split
      __syncthreads();
      exn = min(read_scale(kc & 1), exc + 64);
      sx = exp2i(exn);
#pragma unroll
      for (int k = 0; k < RH; ++k) {
        split_one(k);
        store_one(k);
      }
    }
    if (kc == kc0 + 1) XST(st_c1a);
    if (kc != kc0) {
      // sign-alternating accumulation: odd chunks carry negated weights, so the
      // accumulator holds (-1)^kc x the partial sum; flip it at every chunk boundary
      // (HF: and move it to the units of the next chunk's scale)
      const int dsc = exn - exc;
      if (HF && dsc != 0) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int r = 0; r < NREG; ++r) acc[rb][cb][r] = -ldexpf(acc[rb][cb][r], dsc);
      } else {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = -acc[rb][cb];
      }
      exc = exn;
      if (!LATE) __syncthreads();
    }
    if (kc == kc0 + 1) XST(st_c1b);
    if (SPFF_XDIAG != 1 || kc == kc0)
      stash(kc, kc == kc0, !(LATE && kc != kc0), !(SPFF_XEARLYW && kc == kc0));
    if (kc == kc0) XST(st_pc);
    if (kc == kc0 + 1) XST(st_c1c);
    __syncthreads();  // (vmcnt(0): the weight DMA has landed)
    if (kc == kc0 + 1) XST(st_c1d);
    fetch(kc + 1 < kc1 ? kc + 1 : kc, kc + 1 < kc1);
    // (SPFF_XFPIN) issue those loads here, a whole J0 k-steps before the scale barrier needs
    // them -- not where the scheduler would sink them, next to that barrier
    if constexpr (SPFF_XFPIN) __builtin_amdgcn_sched_barrier(0x7);  // (ALU may cross)
#if SPFF_XSTAMP
    if (kc == kc0) st_t1 = __builtin_amdgcn_s_memtime();
#endif
    // (XPIPE) the fragments of the current row block, carried across the unrolled k-loop
    constexpr bool XPIPE = X16 && SPFF_XPIPE && (BN <= 32 || SPFF_XPIPE64) && !HR;  // (HR: 249 -> 256 VGPRs, spills)
    const bool pg1 = kg & 1, pg2 = kg & 2;
    auto psel4 = [&](int c0, int c1, int c2, int c3) {
      const int lo = pg1 ? c1 : c0, hi = pg1 ? c3 : c2;
      return pg2 ? hi : lo;
    };
    auto ptoff = [&](int j) {
      return psel4(toff_of(QT.src[4 * j]), toff_of(QT.src[4 * j + 1]), toff_of(QT.src[4 * j + 2]),
                   toff_of(QT.src[4 * j + 3]));
    };
    auto pwtap = [&](int j) {
      return psel4(QT.tap[4 * j], QT.tap[4 * j + 1], QT.tap[4 * j + 2], QT.tap[4 * j + 3]);
    };
    auto loadA = [&](bf16x8 (&a)[NP], int j, int rb) {
      const int toff = ptoff(j);
#pragma unroll
      for (int p = 0; p < NP; ++p) a[p] = __builtin_bit_cast(bf16x8, Xs[p * NPOS + hpos[rb] + toff]);
    };
    auto loadB = [&](bf16x8 (&bb)[CB][NP], int j) {
      const int wtap = pwtap(j);
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          bb[cb][p] = __builtin_bit_cast(bf16x8, Ws[(p * T2 + wtap) * BN + cb * 16 + l16]);
    };
    bf16x8 pa[NP], pb[CB][NP];
    if constexpr (XPIPE) {
      if (SPFF_XDIAG != 2) {
        loadB(pb, 0);
        loadA(pa, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < (SPFF_XDIAG == 2 ? 0 : NJ); ++j) {
      if constexpr (SPFF_XIGLP >= 0) __builtin_amdgcn_iglp_opt(SPFF_XIGLP);
      // HF: the next chunk's scale before its halo is split (uniform: kc + 1 < kc1).
      // Capped at 2^64 above the current chunk's, so the rescaled accumulator cannot
      // overflow (|acc| < 2^40 in these units)
      if (HF && !LATE && j == J0 && kc + 1 < kc1) {
        exn = min(block_scale(prep_max(), (kc + 1) & 1), exc + 64);
        sx = exp2i(exn);
      }
      if (LATE && j == (NJ > 2 ? NJ - 2 : 0) && kc + 1 < kc1) {
        __builtin_amdgcn_sched_barrier(0x10C);
        wave_max_store(prep_max(), (kc + 1) & 1);
        __builtin_amdgcn_sched_barrier(0x10C);
      }
      // split one prefetched halo float4 per k-step from the middle of the
      // chunk on; the fences keep this VALU (and its vmcnt wait) in place
      // while MFMAs and LDS reads may still move across
      if (!LATE && j >= J0 && (j - J0) * SPJ < RH) {
        __builtin_amdgcn_sched_barrier(0x10C);
#pragma unroll
        for (int u = 0; u < SPJ; ++u)
          if ((j - J0) * SPJ + u < RH) split_one((j - J0) * SPJ + u);
        __builtin_amdgcn_sched_barrier(0x10C);
      }
      if constexpr (XPIPE) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          bf16x8 na[NP], nb[CB][NP];
          const bool last = rb + 1 == RB, more = j + 1 < NJ;
          // the next row block's reads, then this one's MFMAs: fenced so that neither DS
          // reads nor MFMAs cross (VALU / SALU may: the halo split still interleaves)
          __builtin_amdgcn_sched_barrier(0x6);
          if (!last) {
            loadA(na, j, rb + 1);
          } else if (more) {
            loadB(nb, j + 1);
            loadA(na, j + 1, 0);
          }
          __builtin_amdgcn_sched_barrier(0x6);
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            f32x4 c = acc[rb][cb];
            if constexpr (NP == 3) {
              c = mfma16x32<HF>(pa[1], pb[cb][1], c);
              c = mfma16x32<HF>(pa[0], pb[cb][2], c);
              c = mfma16x32<HF>(pa[2], pb[cb][0], c);
            }
            if constexpr (NP >= 2) {
              c = mfma16x32<HF>(pa[0], pb[cb][1], c);
              c = mfma16x32<HF>(pa[1], pb[cb][0], c);
            }
            c = mfma16x32<HF>(pa[0], pb[cb][0], c);
            acc[rb][cb] = c;
          }
          if (!last || more) {
#pragma unroll
            for (int p = 0; p < NP; ++p) pa[p] = na[p];
          }
          if (last && more) {
#pragma unroll
            for (int p = 0; p < NP; ++p)
#pragma unroll
              for (int cb = 0; cb < CB; ++cb) pb[cb][p] = nb[cb][p];
          }
        }
      } else if constexpr (X16) {
        // lane group kg takes slot 4j + kg of the quad schedule
        // (the four slots' table entries are indexed by the unrolled j only and selected per
        // lane group: a lane-varying index into the constexpr tables made the compiler load
        // them from memory at every k-step, each load followed by a vmcnt(0) that drained the
        // prefetched halo / weight DMA still in flight)
        const bool g1 = kg & 1, g2 = kg & 2;
        auto sel4 = [&](int c0, int c1, int c2, int c3) {
          const int lo = g1 ? c1 : c0, hi = g1 ? c3 : c2;
          return g2 ? hi : lo;
        };
        const int toff = sel4(toff_of(QT.src[4 * j]), toff_of(QT.src[4 * j + 1]),
                              toff_of(QT.src[4 * j + 2]), toff_of(QT.src[4 * j + 3]));
        const int wtap =
            sel4(QT.tap[4 * j], QT.tap[4 * j + 1], QT.tap[4 * j + 2], QT.tap[4 * j + 3]);
        // row blocks in groups of RBH (the 4 x 16 x 16 tiles' 8 row blocks: two groups,
        // so only half of the A fragments are live at a time)
        constexpr int RBH = RB > 4 ? 4 : RB;
        bf16x8 bm[CB][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
            bm[cb][p] = __builtin_bit_cast(bf16x8, Ws[(p * T2 + wtap) * BN + cb * 16 + l16]);
#pragma unroll
        for (int rg = 0; rg < RB; rg += RBH) {
        bf16x8 a[RBH][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int rh = 0; rh < RBH; ++rh)
            a[rh][p] = __builtin_bit_cast(bf16x8, Xs[p * NPOS + hpos[rg + rh] + toff]);
#pragma unroll
        for (int rh = 0; rh < RBH; ++rh)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            const int rb = rg + rh;
            f32x4 c = acc[rb][cb];
            if constexpr (NP == 3) {
              c = mfma16x32<HF>(a[rh][1], bm[cb][1], c);
              c = mfma16x32<HF>(a[rh][0], bm[cb][2], c);
              c = mfma16x32<HF>(a[rh][2], bm[cb][0], c);
            }
            if constexpr (NP >= 2) {
              c = mfma16x32<HF>(a[rh][0], bm[cb][1], c);
              c = mfma16x32<HF>(a[rh][1], bm[cb][0], c);
            }
            c = mfma16x32<HF>(a[rh][0], bm[cb][0], c);
            acc[rb][cb] = c;
          }
        }
      } else {
        // lane half h takes tap 2j+h; the padding tap (>= T) reads a valid
        // position against a zero weight row
        const int tp0 = 2 * j, tp1 = (2 * j + 1 < T) ? 2 * j + 1 : T - 1;
        const int toff = khalf ? toff_of(tp1) : toff_of(tp0);
        const int wtap = 2 * j + khalf;
        bf16x8 a[RB][NP], bm[CB][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
            a[rb][p] = __builtin_bit_cast(bf16x8, Xs[p * NPOS + hpos[rb] + toff]);
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
            bm[cb][p] = __builtin_bit_cast(bf16x8, Ws[(p * T2 + wtap) * BN + cb * 32 + l32]);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            f32x16 c = acc[rb][cb];
            if constexpr (NP == 3) {
              c = mfma32x16<HF>(a[rb][1], bm[cb][1], c);
              c = mfma32x16<HF>(a[rb][0], bm[cb][2], c);
              c = mfma32x16<HF>(a[rb][2], bm[cb][0], c);
            }
            if constexpr (NP >= 2) {
              c = mfma32x16<HF>(a[rb][0], bm[cb][1], c);
              c = mfma32x16<HF>(a[rb][1], bm[cb][0], c);
            }
            c = mfma32x16<HF>(a[rb][0], bm[cb][0], c);
            acc[rb][cb] = c;
          }
      }
    }
  }

#if SPFF_XSTAMP
  st_t2 = __builtin_amdgcn_s_memtime();
#endif
  if ((kc1 - 1) & 1) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = -acc[rb][cb];
  }
  if constexpr (HF) {  // undo the operand scales (exact: a power of two)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r = 0; r < NREG; ++r) acc[rb][cb][r] = ldexpf(acc[rb][cb][r], -(exc + ew));
  }

// ---- epilogue: C[i][j], row i = voxel (vrow mapping), col j = out channel ----
  constexpr int OP = BN + 4;  // output image pitch: 4 rows apart = 16 banks apart
  constexpr int NROW = TD * TH * TW;
  const bool vec = SPFF_XSTORE && !part && X16 && (Cout & 3) == 0 && (y.split & 3) == 0 &&
                   (y.ld0 & 3) == 0 && (y.ld1 & 3) == 0;
  // fused InstanceNorm statistics of this output (replaces two HBM passes): per (tile,
  // channel) the sum over the tile's valid voxels and the sum of squared deviations about
  // the tile mean; merged per (b, c) in a fixed order by k_in_stats_fin (Chan).
  // stats[(tile*npad + n)*2 + {0,1}], count[tile].  The column sums share the output
  // image's barriers: [NW][CB][NCOL] partial sums, then the squared deviations', after the
  // image when the epilogue staged it.
  float* sred = reinterpret_cast<float*>(lds4) + (vec ? NROW * OP : 0);
  float* sred2 = sred + NW * CB * NCOL;
  const int nd = min(D - d0, TD), nh = min(H - h0, TH), nwv = min(W - w0, TW);
  const float cnt = (float)(nd * nh * nwv);
  // lanes holding the same column: 32x32 -- l and l+32; 16x16 -- l, l+16, l+32, l+48
  auto colsum = [&](float v) {
    v += __shfl_xor(v, 32);
    if constexpr (X16) v += __shfl_xor(v, 16);
    return v;
  };
  auto okrow = [&](int rb, int r) {
    int td, th, tw;
    vrow(wave * RB + rb, orow(r), td, th, tw);
    return d0 + td < D && h0 + th < H && w0 + tw < W;
  };
  // (bst, input gradient with fused IN-backward sums): this thread's channel quad is fixed
  // in the row-major store loop below (XT_THREADS is a multiple of BN / 4); its y loads are
  // issued here, before the image barrier, so their latency overlaps it
  constexpr int Q4 = BN / 4;
  constexpr int NIT = NROW * Q4 / XT_THREADS;
  static_assert(XT_THREADS % Q4 == 0 && (NROW * Q4) % XT_THREADS == 0, "store loop shape");
  const bool bsm = SPFF_XBSTAT && !HR && vec && bst.y != nullptr;  // (uniform; unsharded only)
  float4 byv[NIT];
  if (bsm) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + it * XT_THREADS, row = i / Q4, q = i % Q4;
      int td, th, tw;
      vrow(row >> 4, row & 15, td, th, tw);
      const int gd = d0 + td, gh = h0 + th, gw = w0 + tw, n = n0 + 4 * q;
      const bool ok = gd < D && gh < H && gw < W && n < Cout;
      const int64_t vox = ok ? (((int64_t)b * D + gd) * H + gh) * W + gw : 0;
      byv[it] = *reinterpret_cast<const float4*>(bst.y + vox * bst.ld + (ok ? n : 0));
    }
  }
  // every wave is past its last operand read
  if (vec || stats) __syncthreads();
  if (vec) {
    // the image is in MFMA row order (row block q = wave RB + rb, row r), so a lane's 4
    // rows x 16 lanes hit 64 distinct banks
    float* ot = reinterpret_cast<float*>(lds4);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < NREG; ++r)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          ot[((wave * RB + rb) * 16 + orow(r)) * OP + cb * NCOL + lcol] = acc[rb][cb][r];
  }
  if (stats) {
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      float sacc = 0.f;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int r = 0; r < NREG; ++r) sacc += okrow(rb, r) ? acc[rb][cb][r] : 0.f;
      sacc = colsum(sacc);
      if (lane < NCOL) sred[(wave * CB + cb) * NCOL + lcol] = sacc;
    }
  }
  if (vec || stats) __syncthreads();
  if (bsm) {
    const float* ot = reinterpret_cast<const float*>(lds4);
    const int qf = tid % Q4, nf = n0 + 4 * qf;
    float ca[4], cd[4], cm[4], cr[4], s0[4], s1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t bc = (int64_t)b * bst.ld + (nf < Cout ? nf : 0) + j;
      ca[j] = bst.al[bc];
      cd[j] = bst.de[bc];
      cm[j] = bst.mean[bc];
      cr[j] = bst.rstd[bc];
      s0[j] = 0.f;
      s1[j] = 0.f;
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + it * XT_THREADS, row = i / Q4;
      int td, th, tw;
      vrow(row >> 4, row & 15, td, th, tw);
      const int gd = d0 + td, gh = h0 + th, gw = w0 + tw;
      if (gd >= D || gh >= H || gw >= W || nf >= Cout) continue;
      const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
      const float4 v = *reinterpret_cast<const float4*>(ot + row * OP + 4 * qf);
      float* pp = nf < y.split ? y.p0 + vox * y.ld0 + nf : y.p1 + vox * y.ld1 + (nf - y.split);
      *reinterpret_cast<float4*>(pp) = v;
      const float vv[4] = {v.x, v.y, v.z, v.w};
      const float yy[4] = {byv[it].x, byv[it].y, byv[it].z, byv[it].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // RED_BWD_IN's terms (norm.hip), without the gate A, Bc
        const float r = yy[j] * ca[j] + cd[j];
        const float dr = vv[j] * (r > 0.f ? 1.f : bst.neg);
        const float xh = (yy[j] - cm[j]) * cr[j];
        s0[j] += dr;
        s1[j] += dr * xh;
      }
    }
    // the lanes of a wave holding the same channel quad (lane mod Q4), then the waves in
    // order: a fixed reduction tree
#pragma unroll
    for (int o = Q4; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0[j] += __shfl_xor(s0[j], o);
        s1[j] += __shfl_xor(s1[j], o);
      }
    if (lane < Q4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sred[(wave * Q4 + lane) * 8 + j] = s0[j];
        sred[(wave * Q4 + lane) * 8 + 4 + j] = s1[j];
      }
    }
    __syncthreads();
    if (wave == 0 && lane < Q4 && n0 + 4 * lane < Cout) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = 0.f;
        for (int w = 0; w < NW; ++w) t += sred[(w * Q4 + lane) * 8 + j];
        bst.out[((int64_t)tile * npad + n0 + 4 * lane + (j & 3)) * 2 + (j >> 2)] = t;
      }
    }
  } else if (vec) {
    const float* ot = reinterpret_cast<const float*>(lds4);
    for (int i = tid; i < NROW * Q4; i += XT_THREADS) {
      const int row = i / Q4, q = i % Q4;
      int td, th, tw;
      vrow(row >> 4, row & 15, td, th, tw);
      const int gd = d0 + td, gh = h0 + th, gw = w0 + tw;
      const int n = n0 + 4 * q;
      if (gd >= D || gh >= H || gw >= W || n >= Cout) continue;
      const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
      const float4 v = *reinterpret_cast<const float4*>(ot + row * OP + 4 * q);
      float* pp = n < y.split ? y.p0 + vox * y.ld0 + n : y.p1 + vox * y.ld1 + (n - y.split);
      *reinterpret_cast<float4*>(pp) = v;
    }
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    if (vec) break;
#pragma unroll
    for (int r = 0; r < NREG; ++r) {
      int td, th, tw;
      vrow(wave * RB + rb, orow(r), td, th, tw);
      const int gd = d0 + td, gh = h0 + th, gw = w0 + tw;
      if (gd >= D || gh >= H || gw >= W) continue;
      const int64_t vox = (((int64_t)b * D + gd) * H + gh) * W + gw;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int n = n0 + cb * NCOL + lcol;
        if (n >= Cout) continue;
        if (part) {
          part[((int64_t)blockIdx.z * ((int64_t)vol.B * D * H * W) + vox) * npad + n] =
              acc[rb][cb][r];
          continue;
        }
        float* p = n < y.split ? y.p0 + vox * y.ld0 + n : y.p1 + vox * y.ld1 + (n - y.split);
        *p = acc[rb][cb][r];
      }
    }
  }
  if (stats) {
    float tsum[CB], mu[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      float t = 0.f;
      for (int w = 0; w < NW; ++w) t += sred[(w * CB + cb) * NCOL + lcol];
      tsum[cb] = t;
      mu[cb] = t / cnt;
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      float qacc = 0.f;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int r = 0; r < NREG; ++r) {
          const float dl = acc[rb][cb][r] - mu[cb];
          qacc += okrow(rb, r) ? dl * dl : 0.f;
        }
      qacc = colsum(qacc);
      if (lane < NCOL) sred2[(wave * CB + cb) * NCOL + lcol] = qacc;
    }
    __syncthreads();
    if (wave == 0 && lane < NCOL) {
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        float q = 0.f;
        for (int w = 0; w < NW; ++w) q += sred2[(w * CB + cb) * NCOL + lcol];
        const int n = n0 + cb * NCOL + lcol;
        if (n < Cout) {
          stats[((int64_t)tile * npad + n) * 2 + 0] = tsum[cb];
          stats[((int64_t)tile * npad + n) * 2 + 1] = q;
        }
      }
    }
    if (tid == 0 && nbk == 0)
      stats[(int64_t)ntiles * npad * 2 + tile] = cnt;
  }
#if SPFF_XSTAMP
  __syncthreads();
  if (tid == 0 && blockIdx.x < (unsigned)XSTAMP_N && blockIdx.z == 0) {
    unsigned long long* o = g_xstamp + (size_t)blockIdx.x * XSTAMP_W;
    o[0] = st_t0; o[1] = st_t1; o[2] = st_t2; o[3] = __builtin_amdgcn_s_memtime();
    o[4] = st_r0; o[5] = __builtin_amdgcn_s_memrealtime();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    o[6] = hw; o[7] = xcc;
    o[8] = st_pa; o[9] = st_pb; o[10] = st_pc;
    o[11] = st_c1a; o[12] = st_c1b; o[13] = st_c1c; o[14] = st_c1d;
  }
#endif
}

// InstanceNorm3d statistics from the conv's per-tile partials (see the fused
// epilogue above).  One workgroup per (b, c): in fp64, the sample mean from the
// tile sums, then M2 = sum_t [M2_t + n_t (mean_t - mean)^2] (the exact
// decomposition of the squared deviations), each a strided per-thread sum plus
// a fixed-order LDS tree -> mean, rstd = 1/sqrt(var + eps), al = gamma*rstd,
// de = beta - mean*al (the outputs of slab_reduce + in_mean + in_rstd).
__global__ __launch_bounds__(256) void k_in_stats_fin(const float* __restrict__ stats, int ntiles,
                                                      int tpb, int npad, int C,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      float* __restrict__ mean,
                                                      float* __restrict__ rstd,
                                                      float* __restrict__ al,
                                                      float* __restrict__ de) {
  __shared__ double r0[256], r1[256];
  const int bc = blockIdx.x, b = bc / C, c = bc % C, tid = threadIdx.x;
  const float* cnt = stats + (int64_t)ntiles * npad * 2;
  double s = 0.0, n = 0.0;
  const int tend = (b + 1) * tpb;
  // (8 tiles' loads issued before any is added -- the same summation order as one at a
  //  time, which waited out a load latency per tile)
  for (int t0 = b * tpb + tid; t0 < tend; t0 += 256 * 8) {
    float sv[8], nv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + 256 * u;
      const bool ok = t < tend;
      sv[u] = ok ? stats[((int64_t)t * npad + c) * 2] : 0.f;
      nv[u] = ok ? cnt[t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (t0 + 256 * u < tend) {
        s += sv[u];
        n += nv[u];
      }
    }
  }
  r0[tid] = s;
  r1[tid] = n;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
      r0[tid] += r0[tid + st];
      r1[tid] += r1[tid + st];
    }
    __syncthreads();
  }
  const double N = r1[0], mu = r0[0] / N;
  __syncthreads();
  double q = 0.0;
  for (int t0 = b * tpb + tid; t0 < tend; t0 += 256 * 8) {
    float sv[8], qv[8], nv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + 256 * u;
      const bool ok = t < tend;
      const float2 v = ok ? *reinterpret_cast<const float2*>(stats + ((int64_t)t * npad + c) * 2)
                          : make_float2(0.f, 0.f);
      sv[u] = v.x;
      qv[u] = v.y;
      nv[u] = ok ? cnt[t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double nt = nv[u];
      if (t0 + 256 * u >= tend || nt <= 0.0) continue;
      const double dl = sv[u] / nt - mu;
      q += qv[u] + nt * dl * dl;
    }
  }
  r0[tid] = q;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) r0[tid] += r0[tid + st];
    __syncthreads();
  }
  if (tid == 0) {
    const float rs = (float)(1.0 / sqrt(r0[0] / N + 1e-5));
    const float m = (float)mu;
    mean[bc] = m;
    rstd[bc] = rs;
    const float a = gamma[c] * rs;
    al[bc] = a;
    de[bc] = beta[c] - m * a;
  }
}

// y[v][n] = sum over the nsplit partial slabs part[z][v][n], z in order
__global__ void k_splitk_reduce(const float* __restrict__ part, int nsplit, int64_t V, int npad,
                                int N, Dst2 y) {
  const int64_t total = V * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    const int64_t v = i / N;
    float acc = 0.f;
    for (int z = 0; z < nsplit; ++z) acc += part[((int64_t)z * V + v) * npad + n];
    float* p = n < y.split ? y.p0 + v * y.ld0 + n : y.p1 + v * y.ld1 + (n - y.split);
    *p = acc;
  }
}

// 2-deep 32-wide tiles where the 4-deep ones waste more depth planes: D mod 4 = 1 or 2
// (the registry's D = 5 computes 6 planes instead of 8).  Every host-side tile count
// (xt_ntiles: fused statistics, split-K, depth / height splits) takes the same choice.
#ifndef SPFF_X32SHALLOW
#define SPFF_X32SHALLOW 1
#endif
static bool xt_shallow(Vol vol, int BN, int ns) {
  return SPFF_X32SHALLOW && xt_d4(BN, ns) && (vol.D % 4 == 1 || vol.D % 4 == 2);
}
static int xt_td_v(Vol vol, int BN, int ns) { return xt_shallow(vol, BN, ns) ? XT_D : xt_td(BN, ns); }
static int xt_mb_v(Vol vol, int BN, int ns) { return xt_shallow(vol, BN, ns) ? 2 : xt_mb(BN, ns); }

template <int BN, int KD, int NS, bool HR, int MB = xt_mb(BN, NS), int NW = xt_nw(BN, NS),
          int TD = xt_td(BN, NS)>
static hipError_t launch_fwd_xh(const Src2& x, const uint4* wx, const Dst2& y, Vol vol, int K,
                                int nkc, int N, int npad, hipStream_t s, float* part, int nsplit,
                                int kps, float* stats, int dpart, const unsigned* wmx,
                                const BStat& bst) {
  constexpr int TH = SPFF_X16 ? 2 * NW * MB / TD : NW * MB;
  static_assert(NW == 8 || TD == XT_D || xt_d4(BN, NS), "xt_ntiles: tile shape");
  constexpr size_t shm = xt_lds_bytes<BN, KD, NS, TD, TH>();
  // (+ the kernel's static tables: the fused activation's scf[2][32] float4 and the per-wave
  // scale slots smx[2][NW])
  static_assert(shm + 2 * 32 * 16 + 2 * NW * 4 <= (NW == 8 ? 160 : 80) * 1024, "LDS budget");
  if (x.al && BN != 32) return hipErrorInvalidValue;  // fused activation: 32-wide tiles only
  if (x.al && nkc > 16) return hipErrorInvalidValue;  // the kernel's LDS coefficient table
  // the 16/32-wide kernels hold halo voxel indices in 32 bits (with the halo slices)
  if (BN <= 32 && (int64_t)vol.B * (vol.D + 2 * vol.dh) * vol.H * vol.W >= (int64_t(1) << 31))
    return hipErrorInvalidValue;
  auto kern = k_conv3d_fwd_x<BN, KD, NS, MB, NW, SPFF_X16 != 0, TD, HR>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int thn = cdiv(vol.H, TH), tilesW = cdiv(vol.W, XT_W);
  // dpart 1: the interior depth tiles 1 .. n-2 (no halo slice read), 2: the first and last;
  // 3 / 4: the same for the H tiles (height-sharded: no boundary row read / the others)
  const int tdn = cdiv(vol.D, TD);
  if ((dpart == 1 || dpart == 2) && (tdn < 3 || part || stats)) return hipErrorInvalidValue;
  if ((dpart == 3 || dpart == 4) && (thn < 3 || part || stats || !HR)) return hipErrorInvalidValue;
  const int tilesD = dpart == 1 ? tdn - 2 : dpart == 2 ? 2 : tdn;
  const int td0 = dpart == 1 ? 1 : 0, tds = dpart == 2 ? tdn - 1 : 1;
  const int tilesH = dpart == 3 ? thn - 2 : dpart == 4 ? 2 : thn;
  const int th0 = dpart == 3 ? 1 : 0, ths = dpart == 4 ? thn - 1 : 1;
  const int ntiles = vol.B * tilesD * tilesH * tilesW;
  dim3 grid(8 * cdiv(ntiles, 8) * (npad / BN), 1, part ? nsplit : 1);
  hipLaunchKernelGGL(kern, grid, dim3(NW * 64), shm, s, x, wx, y, vol, K, nkc, N, npad, tilesD,
                     tilesH, tilesW, part, part ? kps : nkc, part ? nullptr : stats, ntiles, td0,
                     tds, th0, ths, wmx, bst);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !part) return e;
  const int64_t total = nvox(vol) * N;
  hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 8192)),
                     dim3(256), 0, s, part, nsplit, nvox(vol), npad, N, y);
  return hipGetLastError();
}
template <int BN, int KD, int NS>
static hipError_t launch_fwd_x(const Src2& x, const uint4* wx, const Dst2& y, Vol vol, int K,
                               int nkc, int N, int npad, hipStream_t s, float* part, int nsplit,
                               int kps, float* stats, int dpart, const unsigned* wmx,
                               const BStat& bst) {
  if constexpr (xt_d4(BN, NS)) {
    constexpr int NW = xt_nw(BN, NS);
    if (xt_shallow(vol, BN, NS))
      return x.rows() ? launch_fwd_xh<BN, KD, NS, true, 2, NW, XT_D>(
                            x, wx, y, vol, K, nkc, N, npad, s, part, nsplit, kps, stats, dpart, wmx,
                            bst)
                      : launch_fwd_xh<BN, KD, NS, false, 2, NW, XT_D>(
                            x, wx, y, vol, K, nkc, N, npad, s, part, nsplit, kps, stats, dpart, wmx,
                            bst);
  }
  return x.rows() ? launch_fwd_xh<BN, KD, NS, true>(x, wx, y, vol, K, nkc, N, npad, s, part,
                                                    nsplit, kps, stats, dpart, wmx, bst)
                  : launch_fwd_xh<BN, KD, NS, false>(x, wx, y, vol, K, nkc, N, npad, s, part,
                                                     nsplit, kps, stats, dpart, wmx, bst);
}

namespace {
struct XDims {
  int K, N, BN, nkc, npad, T, T2;
};
XDims xdims(int KD, int Cin_w, int Cout_w, bool dgrad) {
  XDims d;
  d.K = dgrad ? Cout_w : Cin_w;
  d.N = dgrad ? Cin_w : Cout_w;
  // 16-wide tiles for narrow outputs (N <= 16, 3x3x3): the SwinUNETR's C = 12 convs
  // ran their 12 columns in 32-wide tiles (62 % of the MFMA columns padding)
  d.BN = d.N >= 64 ? 64 : (d.N <= 16 && KD == 3 && SPFF_X16) ? 16 : 32;
  d.nkc = cdiv(d.K, 8);
  d.npad = rup(d.N, d.BN);
  d.T = KD * 9;
  d.T2 = (d.T + 1) & ~1;
  return d;
}
// SPFF_DEBUG_SPLIT (diagnostics only): a comma list of the directions that take
// the split path, e.g. "fwd,wgrad"; the others run the f32 MFMA kernels.  Unset:
// all three.  Bits: 1 fwd, 2 dgrad, 4 wgrad.
int debug_split_dir() {
  static int v = [] {
    const char* e = getenv("SPFF_DEBUG_SPLIT");
    if (!e) return 7;
    int m = 0;
    if (strstr(e, "fwd")) m |= 1;
    if (strstr(e, "dgrad")) m |= 2;
    if (strstr(e, "wgrad")) m |= 4;
    return m;
  }();
  return v;
}
bool use_split(Vol vol, int math, bool dgrad) {
  if (!(debug_split_dir() & (dgrad ? 2 : 1))) return false;
  return math != SPFF_MATH_F32;
}
}  // namespace
bool debug_split_wgrad() { return (debug_split_dir() & 4) != 0; }
bool conv3d_fuses_act(int math, int C) {
  return math != SPFF_MATH_F32 && debug_split_dir() == 7 && C == 32;
}
// tiles of a BN-wide launch (the fused IN statistics are per (tile, out channel))
static int64_t xt_ntiles(Vol vol, int BN, int ns) {
  const int nw = xt_nw(BN, ns);
  const int td = xt_td_v(vol, BN, ns), mb = xt_mb_v(vol, BN, ns);
  const int th = SPFF_X16 ? 2 * nw * mb / td : nw * mb;
  return (int64_t)vol.B * cdiv(vol.D, td) * cdiv(vol.H, th) * cdiv(vol.W, XT_W);
}
namespace {
// split-K for launches that would not fill the chip (the deep levels of the
// 3DUNet: 2 x 12 x 12 and 1 x 6 x 6 voxels with 256-512 channels): the input
// channel chunks are divided over grid.z so that >= ~512 workgroups run
struct SplitK {
  int nsplit = 1, kps = 0;
};
SplitK splitk_plan(Vol vol, const XDims& d, int nsp) {
  SplitK k;
  k.kps = d.nkc;
  const int64_t wgs = xt_ntiles(vol, d.BN, nsp) * (d.npad / d.BN);
  if (wgs >= 256 || d.nkc < 4) return k;
  int ns = (int)std::min<int64_t>(d.nkc / 2, (512 + wgs - 1) / wgs);
  ns = std::max(1, ns);
  k.kps = cdiv(d.nkc, ns);
  k.nsplit = cdiv(d.nkc, k.kps);
  return k;
}
}  // namespace

// ----------------------------------------------------------- dispatcher --
// ---- SPFF_MATH_F16X3 operand scales ----
// The largest |element| of each operand, as float bits (a non-negative float orders like
// its bits), by integer atomicMax -- order-independent, so deterministic -- into two
// slots after the packed weight image: [0] max |w| (conv3d_pack zeroes both and fills
// it), [1] max |x| (conv3d_run, over exactly what the launch reads).
__global__ __launch_bounds__(256) void k_absmax_f32(const float* __restrict__ p, int64_t n,
                                                    unsigned* __restrict__ slot) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(p[i]));
  block_amax(m, slot);
}
// |elements| of channels [c, c + 4) of one voxel's row (4-aligned, one source), input
// activation applied; channels >= C (row padding) ignored
__device__ __forceinline__ float amax4(const float* row, const Src2& x, int b, int c, int C) {
  const float4 v = *reinterpret_cast<const float4*>(row);
  float r[4] = {v.x, v.y, v.z, v.w};
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float t = r[j];
    if (x.al) {
      t = t * x.al[(int64_t)b * x.ld0 + c + j] + x.de[(int64_t)b * x.ld0 + c + j];
      t = t > 0.f ? t : 0.01f * t;
    }
    m = c + j < C ? fmaxf(m, fabsf(t)) : m;
  }
  return m;
}
// max |x| over what a conv launch reads: depth planes [dlo, dhi) of [B][D][H][W] (the
// halo slices of a depth-sharded input when included), and the height-sharded boundary
// rows rlo / rhi ([B][D][W][ldr]) when withrows
__global__ __launch_bounds__(256) void k_absmax_src(Src2 x, Vol vol, int C, int dlo, int dhi,
                                                    int withrows, unsigned* __restrict__ slot,
                                                    const unsigned* __restrict__ also) {
  const int C4 = (C + 3) >> 2, H = vol.H, W = vol.W, nd = dhi - dlo;
  const int64_t total = (int64_t)vol.B * nd * H * W * C4;
  float m = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = 4 * (int)(i % C4);
    int64_t t = i / C4;
    const int gw = (int)(t % W); t /= W;
    const int gh = (int)(t % H); t /= H;
    const int gd = dlo + (int)(t % nd);
    const int b = (int)(t / nd);
    const int64_t vox = (((int64_t)b * vol.D + gd) * H + gh) * W + gw;
    const float* row = c < x.split ? x.p0 + vox * x.ld0 + c : x.p1 + vox * x.ld1 + (c - x.split);
    m = fmaxf(m, amax4(row, x, b, c, C));
  }
  if (withrows) {
    const int64_t nr = (int64_t)vol.B * vol.D * W * C4;
    for (int side = 0; side < 2; ++side) {
      const float* rp = side ? x.rhi : x.rlo;
      if (!rp) continue;
      for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nr; i += (int64_t)gridDim.x * 256) {
        const int c = 4 * (int)(i % C4);
        const int64_t bdw = i / C4;
        const int b = (int)(bdw / ((int64_t)vol.D * W));
        m = fmaxf(m, amax4(rp + bdw * x.ldr + c, x, b, c, C));
      }
    }
  }
  if (also && blockIdx.x == 0) m = fmaxf(m, __uint_as_float(*also));
  block_amax(m, slot);
}
// a dense [n4] float4 array (one source, no padding channels, no activation, no halo):
// pure streaming, 4 loads in flight per thread
__global__ __launch_bounds__(256) void k_absmax_dense(const float4* __restrict__ p, int64_t n4,
                                                      unsigned* __restrict__ slot,
                                                      const unsigned* __restrict__ also) {
  float m = 0.f;
  const int64_t st = (int64_t)gridDim.x * 256;
  int64_t i = blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n4; i += 4 * st) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[i + u * st];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
  }
  for (; i < n4; i += st) {
    const float4 v = p[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  if (also && blockIdx.x == 0) m = fmaxf(m, __uint_as_float(*also));
  block_amax(m, slot);
}
static unsigned absmax_grid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 2047) / 2048, 1024));
}
hipError_t absmax_src(const Src2& x, Vol vol, int C, bool halo, unsigned* slot, hipStream_t s,
                      const unsigned* also) {
  if ((x.ld0 & 3) || (x.ld1 & 3) || (x.split & 3) || (x.rows() && (x.ldr & 3)))
    return hipErrorInvalidValue;
  const int dlo = halo && vol.dh && !x.zlo ? -vol.dh : 0;
  const int dhi = vol.D + (halo && vol.dh && !x.zhi ? vol.dh : 0);
  const int64_t n = (int64_t)vol.B * (dhi - dlo) * vol.H * vol.W * ((C + 3) / 4);
  if (!x.al && dlo == 0 && dhi == vol.D && !(halo && x.rows()) && x.split >= C && x.ld0 == C) {
    hipLaunchKernelGGL(k_absmax_dense, dim3(absmax_grid(n)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(x.p0), n, slot, also);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_absmax_src, dim3(absmax_grid(n)), dim3(256), 0, s, x, vol, C, dlo, dhi,
                     halo && x.rows() ? 1 : 0, slot, also);
  return hipGetLastError();
}
hipError_t absmax_f32(const float* p, int64_t n, unsigned* slot, hipStream_t s) {
  hipLaunchKernelGGL(k_absmax_f32, dim3(absmax_grid(n)), dim3(256), 0, s, p, n, slot);
  return hipGetLastError();
}

static size_t pack_main_bytes(int KD, int Cin, int Cout) {
  size_t f32 = 0, x = 0;
  for (int dg = 0; dg < 2; ++dg) {
    const XDims d = xdims(KD, Cin, Cout, dg != 0);
    f32 = std::max(f32, (size_t)d.T * rup(d.K, 8) * rup(d.N, conv3d_bn(d.N)) * sizeof(float));
    x = std::max(x, (size_t)d.T2 * d.nkc * d.npad * 16 * 3);  // 3 bf16 planes of 8 k
  }
  return (std::max(f32, x) + 255) & ~(size_t)255;
}
size_t conv3d_pack_bytes(int KD, int Cin, int Cout) {
  return pack_main_bytes(KD, Cin, Cout) + 256;  // + the F16X3 scale slots
}
static unsigned* f16_slots(const void* wpack, int KD, int Cin_w, int Cout_w) {
  return reinterpret_cast<unsigned*>(static_cast<char*>(const_cast<void*>(wpack)) +
                                     pack_main_bytes(KD, Cin_w, Cout_w));
}

hipError_t conv3d_pack(const float* w, void* wpack, Vol vol, int KD, int Cin_w, int Cout_w,
                       bool dgrad, int math, hipStream_t s, const unsigned* wmax) {
  const XDims d = xdims(KD, Cin_w, Cout_w, dgrad);
  if (use_split(vol, math, dgrad)) {
    const int64_t total = (int64_t)d.nkc * d.T2 * d.npad;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
    uint4* wp = static_cast<uint4*>(wpack);
    unsigned* sl = f16_slots(wpack, KD, Cin_w, Cout_w);
    if (math == SPFF_MATH_F16X3) {
      if (!wmax) {  // max |w| into the image's slot 0 (else the caller's precomputed slot)
        hipError_t e = spff::zero_async(sl, sizeof(unsigned), s);
        if (e != hipSuccess) return e;
        e = absmax_f32(w, (int64_t)Cout_w * Cin_w * d.T, sl, s);
        if (e != hipSuccess) return e;
        wmax = sl;
      }
      hipLaunchKernelGGL(k_conv_pack_x<NS_F16>, dim3(grid), dim3(256), 0, s, w, wp, Cout_w, Cin_w,
                         d.T, d.T2, d.nkc, d.npad, d.BN, dgrad ? 1 : 0, wmax);
    } else if (math == SPFF_MATH_BF16X3) {
      hipLaunchKernelGGL(k_conv_pack_x<2>, dim3(grid), dim3(256), 0, s, w, wp, Cout_w, Cin_w, d.T,
                         d.T2, d.nkc, d.npad, d.BN, dgrad ? 1 : 0, (const unsigned*)nullptr);
    } else {
      hipLaunchKernelGGL(k_conv_pack_x<3>, dim3(grid), dim3(256), 0, s, w, wp, Cout_w, Cin_w, d.T,
                         d.T2, d.nkc, d.npad, d.BN, dgrad ? 1 : 0, (const unsigned*)nullptr);
    }
    return hipGetLastError();
  }
  return conv_pack_weights(w, static_cast<float*>(wpack), Cout_w, Cin_w, KD, rup(d.K, 8),
                           rup(d.N, conv3d_bn(d.N)), dgrad, s);
}

// ------------------------------------------------- batched weight preparation --
// job j of the table owns blocks [blk0, blk0 + nblk); kinds: 0 max |a| over n elements
// (integer atomicMax into the zeroed slot, like k_absmax_f32), 1 act_bound's parameter
// bound 2 (max|gamma| sq + max|beta|) + 1e-30 (k_act_bound's value; max is exact in any order)
__global__ __launch_bounds__(256) void k_prep_many(PrepJobs J) {
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.j[j + 1].blk0) ++j;
  const PrepJob& q = J.j[j];
  if (q.kind == 0) {
    float m = 0.f;
    const int64_t st = (int64_t)q.nblk * 256;
    for (int64_t i = (int64_t)((int)blockIdx.x - q.blk0) * 256 + threadIdx.x; i < q.n; i += st)
      m = fmaxf(m, fabsf(q.a[i]));
    block_amax(m, q.slot);
    return;
  }
  __shared__ float wg[4], wb[4];
  float mg = 0.f, mb = 0.f;
  for (int c = threadIdx.x; c < (int)q.n; c += 256) {
    mg = fmaxf(mg, fabsf(q.a[c]));
    mb = fmaxf(mb, fabsf(q.b[c]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o));
    mb = fmaxf(mb, __shfl_xor(mb, o));
  }
  if ((threadIdx.x & 63) == 0) {
    wg[threadIdx.x >> 6] = mg;
    wb[threadIdx.x >> 6] = mb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mg = fmaxf(fmaxf(wg[0], wg[1]), fmaxf(wg[2], wg[3]));
    mb = fmaxf(fmaxf(wb[0], wb[1]), fmaxf(wb[2], wb[3]));
    *q.slot = __float_as_uint(2.f * (mg * q.sq + mb) + 1e-30f);
  }
}
// (SPFF_PACK_BATCH=0, diagnostics / A/B only: one max + one pack launch per conv again)
bool conv3d_packs_batched(int math) {
  static const bool off = [] {
    const char* e = getenv("SPFF_PACK_BATCH");
    return e && e[0] == '0';
  }();
  return !off && use_split(Vol{}, math, false) && use_split(Vol{}, math, true);
}
// Blocks per job: the largest weights (the 3DUNet's 320 x 320 x 27) set the launch's time,
// so a job's cap is several blocks per CU, not the 64 (a quarter of the CUs) of round 4.
#ifndef SPFF_PREP_NB
#define SPFF_PREP_NB 256
#endif
#ifndef SPFF_PACK_NB
#define SPFF_PACK_NB 512
#endif
bool prep_absmax(PrepJobs* J, const float* p, int64_t n, unsigned* slot) {
  if (J->n == 32 || n <= 0) return false;
  const int nb = (int)std::min<int64_t>(SPFF_PREP_NB, std::max<int64_t>(1, (n + 4095) / 4096));
  J->j[J->n++] = PrepJob{p, nullptr, slot, n, 0.f, 0, J->nblk, nb};
  J->nblk += nb;
  return true;
}
bool prep_act_bound(PrepJobs* J, const float* gamma, const float* beta, int C, double N,
                    unsigned* slot) {
  if (J->n == 32 || C <= 0) return false;
  const float sq = (float)std::sqrt(std::max(N - 1.0, 1.0));
  J->j[J->n++] = PrepJob{gamma, beta, slot, C, sq, 1, J->nblk, 1};
  J->nblk += 1;
  return true;
}
hipError_t prep_run(const PrepJobs& J, hipStream_t s) {
  if (J.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prep_many, dim3(J.nblk), dim3(256), 0, s, J);
  return hipGetLastError();
}
bool conv3d_pack_job(PackJobs* J, const float* w, void* wpack, int KD, int Cin_w, int Cout_w,
                     bool dgrad, const unsigned* wmax) {
  if (J->n == 40) return false;
  const XDims d = xdims(KD, Cin_w, Cout_w, dgrad);
  const int64_t total = (int64_t)d.nkc * d.T2 * d.npad;
  const int nb = (int)std::min<int64_t>(SPFF_PACK_NB, (total + 255) / 256);
  J->j[J->n++] = PackJob{w, static_cast<uint4*>(wpack), wmax, Cout_w, Cin_w, d.T, d.T2, d.nkc,
                         d.npad, d.BN, dgrad ? 1 : 0, J->nblk, nb};
  J->nblk += nb;
  return true;
}
hipError_t conv3d_pack_many(const PackJobs& J, int math, hipStream_t s) {
  if (!conv3d_packs_batched(math)) return hipErrorInvalidValue;
  if (J.n == 0) return hipSuccess;
  if (math == SPFF_MATH_F16X3) {
    for (int i = 0; i < J.n; ++i)
      if (!J.j[i].wmx) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_conv_pack_many<NS_F16>, dim3(J.nblk), dim3(256), 0, s, J);
  } else if (math == SPFF_MATH_BF16X3) {
    hipLaunchKernelGGL(k_conv_pack_many<2>, dim3(J.nblk), dim3(256), 0, s, J);
  } else {
    hipLaunchKernelGGL(k_conv_pack_many<3>, dim3(J.nblk), dim3(256), 0, s, J);
  }
  return hipGetLastError();
}

template <int NS>
static hipError_t run_x(const Src2& x, const uint4* wu, const Dst2& y, Vol vol, int KD,
                        const XDims& d, hipStream_t s, float* ws, float* stats, int dpart,
                        const unsigned* wmx, const BStat& bst) {
  // (32x32x16, MB = 4, 2 x 32 x 16 tiles for Cout <= 32: fits LDS but spills 91 VGPRs)
  // (32x32x16 schedule, NW = 4 waves, 2 x 8 x 16 tiles: measured 6 % slower; the 16x16x32
  // schedule takes NW = 4 for BN 32 by default, SPFF_X32NW)
  SplitK k = ws ? splitk_plan(vol, d, NS) : SplitK{1, d.nkc};
  float* part = k.nsplit > 1 ? ws : nullptr;
  if (d.BN == 64)
    return KD == 3
               ? launch_fwd_x<64, 3, NS>(x, wu, y, vol, d.K, d.nkc, d.N, d.npad, s, part,
                                                k.nsplit, k.kps, stats, dpart, wmx, bst)
               : launch_fwd_x<64, 1, NS>(x, wu, y, vol, d.K, d.nkc, d.N, d.npad, s, part,
                                                k.nsplit, k.kps, stats, dpart, wmx, bst);
  if (d.BN == 16)
    return launch_fwd_x<16, 3, NS>(x, wu, y, vol, d.K, d.nkc, d.N, d.npad, s, part, k.nsplit,
                                   k.kps, stats, dpart, wmx, bst);
  return KD == 3 ? launch_fwd_x<32, 3, NS>(x, wu, y, vol, d.K, d.nkc, d.N, d.npad, s,
                                                  part, k.nsplit, k.kps, stats, dpart, wmx, bst)
                 : launch_fwd_x<32, 1, NS>(x, wu, y, vol, d.K, d.nkc, d.N, d.npad, s,
                                                  part, k.nsplit, k.kps, stats, dpart, wmx, bst);
}


size_t conv3d_splitk_bytes(Vol vol, int KD, int Cin, int Cout) {
  size_t b = 0;
  for (int dg = 0; dg < 2; ++dg) {
    const XDims d = xdims(KD, Cin, Cout, dg != 0);
    for (int ns : {3, NS_F16}) {  // (the tile counts of every arithmetic)
      const SplitK k = splitk_plan(vol, d, ns);
      if (k.nsplit > 1) b = std::max(b, (size_t)k.nsplit * nvox(vol) * d.npad * sizeof(float));
    }
  }
  return b;
}

bool conv3d_splits_depth(Vol vol, int KD, int Cin_w, int Cout_w, bool dgrad, int math) {
  const XDims d = xdims(KD, Cin_w, Cout_w, dgrad);
  return KD == 3 && use_split(vol, math, dgrad) && splitk_plan(vol, d, ns_of(math)).nsplit == 1 &&
         cdiv(vol.D, xt_td_v(vol, d.BN, ns_of(math))) >= 3;
}
bool conv3d_splits_height(Vol vol, int KD, int Cin_w, int Cout_w, bool dgrad, int math) {
  const XDims d = xdims(KD, Cin_w, Cout_w, dgrad);
  const int nw = xt_nw(d.BN, ns_of(math));
  const int ns = ns_of(math);
  const int th = SPFF_X16 ? 2 * nw * xt_mb_v(vol, d.BN, ns) / xt_td_v(vol, d.BN, ns)
                          : nw * xt_mb_v(vol, d.BN, ns);
  return use_split(vol, math, dgrad) && splitk_plan(vol, d, ns_of(math)).nsplit == 1 &&
         cdiv(vol.H, th) >= 3;
}
size_t conv3d_stats_bytes(Vol vol, int KD, int Cin, int Cout) {
  const XDims d = xdims(KD, Cin, Cout, false);
  const int64_t nt = std::max(xt_ntiles(vol, d.BN, 3), xt_ntiles(vol, d.BN, NS_F16));
  return (size_t)nt * (2 * d.npad + 1) * sizeof(float);
}
// the input gradient's epilogue with the IN-backward sums (BStat): the split kernel, one
// launch (no split-K, unsharded), 16-B row stores (the X16 LDS-staged epilogue)
bool conv3d_fuses_bwd_stats(Vol vol, int KD, int Cin_w, int Cout_w, int math) {
  const XDims d = xdims(KD, Cin_w, Cout_w, true);
  return SPFF_XBSTAT && SPFF_X16 && SPFF_XSTORE && use_split(vol, math, true) && vol.dh == 0 &&
         (d.N & 3) == 0 && splitk_plan(vol, d, ns_of(math)).nsplit == 1;
}
// per (b, c): sum dr, sum dr xhat over the sample's tiles in a fixed order (fp64) -> k1, k2
// (/ N) and dgamma, dbeta (summed over b) -- k_in_bwd_stats' outputs
__global__ __launch_bounds__(256) void k_in_bwd_stats_tiles(const float* __restrict__ part,
                                                            int tpb, int npad, int B, int C,
                                                            double N, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta,
                                                            float* __restrict__ k1,
                                                            float* __restrict__ k2) {
  __shared__ double r0[256], r1[256];
  const int c = blockIdx.x, tid = threadIdx.x;
  double tg = 0.0, tb = 0.0;
  for (int b = 0; b < B; ++b) {
    double s0 = 0.0, s1 = 0.0;
    const int tend = (b + 1) * tpb;
    for (int t0 = b * tpb + tid; t0 < tend; t0 += 256 * 8) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = t0 + 256 * u;
        v[u] = t < tend ? *reinterpret_cast<const float2*>(part + ((int64_t)t * npad + c) * 2)
                        : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s0 += v[u].x;
        s1 += v[u].y;
      }
    }
    r0[tid] = s0;
    r1[tid] = s1;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (tid < st) {
        r0[tid] += r0[tid + st];
        r1[tid] += r1[tid + st];
      }
      __syncthreads();
    }
    if (tid == 0) {
      k1[b * C + c] = (float)(r0[0] / N);
      k2[b * C + c] = (float)(r1[0] / N);
    }
    tb += r0[0];
    tg += r1[0];
    __syncthreads();
  }
  if (tid == 0) {
    if (dgamma) dgamma[c] = (float)tg;
    if (dbeta) dbeta[c] = (float)tb;
  }
}
hipError_t conv3d_in_bwd_stats_fin(const float* part, Vol vol, int KD, int Cin_w, int Cout_w,
                                   int math, float* dgamma, float* dbeta, float* k1, float* k2,
                                   hipStream_t s) {
  const XDims d = xdims(KD, Cin_w, Cout_w, true);
  const int64_t nt = xt_ntiles(vol, d.BN, ns_of(math));
  hipLaunchKernelGGL(k_in_bwd_stats_tiles, dim3(d.N), dim3(256), 0, s, part, (int)(nt / vol.B),
                     d.npad, vol.B, d.N, (double)vol.D * vol.H * vol.W, dgamma, dbeta, k1, k2);
  return hipGetLastError();
}
bool conv3d_fuses_stats(Vol vol, int KD, int Cin, int Cout, int math) {
  const XDims d = xdims(KD, Cin, Cout, false);
  return use_split(vol, math, false) && vol.dh == 0 && splitk_plan(vol, d, ns_of(math)).nsplit == 1;
}
hipError_t conv3d_in_stats_fin(const float* stats, Vol vol, int KD, int Cin, int Cout, int math,
                               const float* gamma, const float* beta, float* mean, float* rstd,
                               float* al, float* de, hipStream_t s) {
  const XDims d = xdims(KD, Cin, Cout, false);
  const int64_t nt = xt_ntiles(vol, d.BN, ns_of(math));
  hipLaunchKernelGGL(k_in_stats_fin, dim3(vol.B * Cout), dim3(256), 0, s, stats, (int)nt,
                     (int)(nt / vol.B), d.npad, Cout, gamma, beta, mean, rstd, al, de);
  return hipGetLastError();
}

namespace {
struct CProfRec {
  hipEvent_t a = nullptr, b = nullptr;
  int cls = 0;
  double flops = 0.0;
};
std::vector<CProfRec> g_cprof;
size_t g_cprof_n = 0;
bool g_cprof_on = false;
}  // namespace
CProf::CProf(int cls, double flops, hipStream_t s) {
  if (!g_cprof_on) return;
  if (g_cprof_n == g_cprof.size()) {
    CProfRec r;
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return;
    g_cprof.push_back(r);
  }
  CProfRec& r = g_cprof[g_cprof_n];
  r.cls = cls;
  r.flops = flops;
  if (hipEventRecord(r.a, s) != hipSuccess) return;
  rec = (int)g_cprof_n++;
}
void CProf::end(hipStream_t s) {
  if (rec >= 0) (void)hipEventRecord(g_cprof[rec].b, s);
  rec = -1;
}
void conv_prof_enable(bool on) {
  g_cprof_on = on;
  g_cprof_n = 0;
}
hipError_t conv_prof_collect(double* out, int nclass) {
  for (int i = 0; i < 4 * nclass; ++i) out[i] = 0.0;
  for (size_t i = 0; i < g_cprof_n; ++i) {
    CProfRec& r = g_cprof[i];
    hipError_t e = hipEventSynchronize(r.b);
    if (e != hipSuccess) return e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess) return e;
    if (r.cls < nclass) {
      out[4 * r.cls + 0] += ms;
      out[4 * r.cls + 1] += r.flops;
      out[4 * r.cls + 2] += 1.0;
    }
  }
  g_cprof_n = 0;
  return hipSuccess;
}

static hipError_t conv3d_run_(const Src2& x, const void* wpack, const Dst2& y, Vol vol, int KD,
                              int Cin_w, int Cout_w, bool dgrad, int math, hipStream_t s,
                              float* ws, float* stats, int dpart, const unsigned* wmax,
                              const BStat* bst);
hipError_t conv3d_run(const Src2& x, const void* wpack, const Dst2& y, Vol vol, int KD,
                      int Cin_w, int Cout_w, bool dgrad, int math, hipStream_t s, float* ws,
                      float* stats, int dpart, const unsigned* wmax, const BStat* bst) {
  CProf pr(dgrad ? 1 : 0, 2.0 * (double)nvox(vol) * Cin_w * Cout_w * 9 * KD, s);
  const hipError_t e = conv3d_run_(x, wpack, y, vol, KD, Cin_w, Cout_w, dgrad, math, s, ws,
                                   stats, dpart, wmax, bst);
  pr.end(s);
  return e;
}
static hipError_t conv3d_run_(const Src2& x, const void* wpack, const Dst2& y, Vol vol, int KD,
                              int Cin_w, int Cout_w, bool dgrad, int math, hipStream_t s,
                              float* ws, float* stats, int dpart, const unsigned* wmax,
                              const BStat* bst) {
  const XDims d = xdims(KD, Cin_w, Cout_w, dgrad);
  if (bst && (dpart != 0 || x.rows() || !conv3d_fuses_bwd_stats(vol, KD, Cin_w, Cout_w, math) ||
              (y.split & 3) || (y.ld0 & 3) || (y.ld1 & 3) || (bst->ld & 3) || !bst->y ||
              !bst->out))
    return hipErrorInvalidValue;
  const BStat bs = bst ? *bst : BStat{};
  if (stats && (dgrad || !conv3d_fuses_stats(vol, KD, Cin_w, Cout_w, math)))
    return hipErrorInvalidValue;
  if ((dpart == 1 || dpart == 2) && !conv3d_splits_depth(vol, KD, Cin_w, Cout_w, dgrad, math))
    return hipErrorInvalidValue;
  if ((dpart == 3 || dpart == 4) &&
      (!x.rows() || !conv3d_splits_height(vol, KD, Cin_w, Cout_w, dgrad, math)))
    return hipErrorInvalidValue;
  if (use_split(vol, math, dgrad)) {
    const uint4* wu = static_cast<const uint4*>(wpack);
    if (math == SPFF_MATH_F16X3) {
      // the input's scale is taken per (tile, chunk) inside the kernel; the weights' from
      // the caller's precomputed max |w| or the one conv3d_pack left in the image's slot 0
      unsigned* sl = f16_slots(wpack, KD, Cin_w, Cout_w);
      return run_x<NS_F16>(x, wu, y, vol, KD, d, s, ws, stats, dpart, wmax ? wmax : sl, bs);
    }
    return math == SPFF_MATH_BF16X3
               ? run_x<2>(x, wu, y, vol, KD, d, s, ws, stats, dpart, nullptr, bs)
               : run_x<3>(x, wu, y, vol, KD, d, s, ws, stats, dpart, nullptr, bs);
  }
  return conv3d_fwd(x, static_cast<const float*>(wpack), y, vol, KD, d.K, rup(d.K, 8), d.N,
                    rup(d.N, conv3d_bn(d.N)), s);
}

#if SPFF_XSTAMP
}  // namespace spff
extern "C" int spff_debug_xstamps_reset() {
  void* p = nullptr;
  hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(spff::g_xstamp));
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(p, 0, sizeof(spff::g_xstamp));
}
extern "C" int spff_debug_xstamps(unsigned long long* host, int n) {
  if (n > spff::XSTAMP_N) n = spff::XSTAMP_N;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(spff::g_xstamp),
                                  sizeof(unsigned long long) * spff::XSTAMP_W * n, 0,
                                  hipMemcpyDeviceToHost);
}
namespace spff {
#endif
}  // namespace spff
