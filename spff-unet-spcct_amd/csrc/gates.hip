// Gate algebra of the SPFF block tail at (b, c, d) granularity.
//
// Reference ops (models.py): EnergyFiLM3D 1479-1512, FourierGate3D 1515-1544,
// _SpectralSE 611-614, _SEChannelLite 600-609.  Every one of them is a per-(c,d)
// affine, a per-d scalar or a per-c scalar applied to the same tensor, so with
//   a2 = lrelu(IN(y2)),  z = a2*(1+t[c,d]) + bt[c,d],
//   Sa[b,c,d] = sum_hw a2   ->   Z[b,c,d] = sum_hw z = (1+t)*Sa + bt*HW
// all means the gates need are (b,c,d)-level algebra on Z (DESIGN.md derives
// it), and the block output is  out = a2 * P[b,c,d] + Q[b,c,d].
// The FourierGate's rfft -> real mask -> irfft(n=D) is a real circulant
// operator w = A s1 with A[d,d'] = (1/D) sum_k c_k M_k cos(2 pi k (d-d') / D)
// (c_0 = 1, c_{D/2} = 1 for even D, else 2); it is evaluated as an explicit
// double-precision DFT from an LDS twiddle table (D <= 512, negligible work).
//
// One 1024-thread workgroup per sample; every sum is a fixed-order
// (thread-slice partials in LDS, then an ordered combine) -> deterministic.
#include "spff_internal.h"
#include <math.h>

#include <algorithm>

namespace spff {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ double ck_coef(int k, int D) {
  return (k == 0 || (D % 2 == 0 && k == D / 2)) ? 1.0 : 2.0;
}

// FourierGate3D(learn_phase=True) multiplies the spectrum by M_k + 0.01 i (models.py:1538-1539).
// irfft keeps only the real part of the DC and Nyquist bins, so the extra term of w[d] is
//   (1/D) sum_k c'_k Re(0.01 i S_k e^{i theta}) = -(0.01/D) sum_k c'_k (Sre sin + Sim cos),
// theta = 2 pi k d / D, c'_k = c_k except 0 at DC / Nyquist: a real circulant H with
// H[d, d'] = -(1/D) sum_k c'_k sin(2 pi k (d - d') / D), independent of M (so the mask and
// mag_scale gradients are unchanged).  Its transpose on the backward (T = the dw spectrum,
// Tre = sum dw cos, Tim = sum dw sin): -(0.01/D) sum_k c'_k (Tim cos - Tre sin).
__device__ __forceinline__ double phase_c(int k, int D) {
  return (k == 0 || (D % 2 == 0 && k == D / 2)) ? 0.0 : 2.0;
}
__device__ __forceinline__ double phase_term(int on, int k, int D, double Sre, double Sim,
                                             double c, double sn) {
  return on ? -0.01 * phase_c(k, D) * (Sre * sn + Sim * c) : 0.0;
}
__device__ __forceinline__ double phase_term_t(int on, int k, int D, double Tre, double Tim,
                                               double c, double sn) {
  return on ? -0.01 * phase_c(k, D) * (Tim * c - Tre * sn) : 0.0;
}

int se_hidden(int C) { return C / 16 > 4 ? C / 16 : 4; }

constexpr int GT = 1024;  // threads per gate workgroup
#ifndef SPFF_GSPLIT_MIN
// C x D from which the gate algebra runs as the channel-split kernels (grid C / 8 x B)
// instead of one workgroup per sample
#define SPFF_GSPLIT_MIN 8192
#endif
constexpr size_t GATE_LDS_MAX = 160 * 1024;

// twiddles: twc[m] = cos(2 pi m / D), tws[m] = sin(2 pi m / D)
__device__ void make_twiddles(double* twc, double* tws, int D) {
  for (int m = threadIdx.x; m < D; m += blockDim.x) {
    double s, c;
    sincos(6.283185307179586476925286766559 * (double)m / (double)D, &s, &c);
    twc[m] = c;
    tws[m] = s;
  }
}

// out[i] = scale * sum_{j<NJ} f(i, j) for i < NI, computed by slices of threads
// (partials in `part`, combined in slice order).  Ends with __syncthreads().
template <class Fn>
__device__ void rowsum(int NI, int NJ, Fn f, double* part, double scale, double* out) {
  const int t = threadIdx.x;
  if (NI >= (int)blockDim.x) {  // one thread per row
    for (int i = t; i < NI; i += blockDim.x) {
      double s = 0.0;
      for (int j = 0; j < NJ; ++j) s += f(i, j);
      out[i] = s * scale;
    }
    __syncthreads();
    return;
  }
  const int S = (int)blockDim.x / NI;
  double acc = 0.0;
  if (t < NI * S) {
    const int i = t / S, sl = t % S;
    for (int j = sl; j < NJ; j += S) acc += f(i, j);
  }
  __syncthreads();
  if (t < NI * S) part[t] = acc;
  __syncthreads();
  for (int i = t; i < NI; i += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q < S; ++q) s += part[i * S + q];
    out[i] = s * scale;
  }
  __syncthreads();
}

// N row sums over the same (NI, NJ) index space in one pass (f(i, j, v) fills v[0..N-1]);
// part holds N x blockDim.x doubles.  Same slice partition and combine order as rowsum.
template <int N, class Fn>
__device__ void rowsum_n(int NI, int NJ, Fn f, double* part, double scale, double* const* out) {
  const int t = threadIdx.x, nt = (int)blockDim.x;
  const int S = NI >= nt ? 1 : nt / NI;
  double acc[N];
#pragma unroll
  for (int q = 0; q < N; ++q) acc[q] = 0.0;
  if (NI >= nt) {
    for (int i = t; i < NI; i += nt) {
#pragma unroll
      for (int q = 0; q < N; ++q) acc[q] = 0.0;
      for (int j = 0; j < NJ; ++j) {
        double v[N];
        f(i, j, v);
#pragma unroll
        for (int q = 0; q < N; ++q) acc[q] += v[q];
      }
#pragma unroll
      for (int q = 0; q < N; ++q) out[q][i] = acc[q] * scale;
    }
    __syncthreads();
    return;
  }
  if (t < NI * S) {
    const int i = t / S, sl = t % S;
    for (int j = sl; j < NJ; j += S) {
      double v[N];
      f(i, j, v);
#pragma unroll
      for (int q = 0; q < N; ++q) acc[q] += v[q];
    }
  }
  __syncthreads();
  if (t < NI * S)
#pragma unroll
    for (int q = 0; q < N; ++q) part[q * nt + t] = acc[q];
  __syncthreads();
  for (int i = t; i < NI; i += nt)
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double sum = 0.0;
      for (int k = 0; k < S; ++k) sum += part[q * nt + i * S + k];
      out[q][i] = sum * scale;
    }
  __syncthreads();
}

// ------------------------------------------------------------- EFiLM fwd --
// hid[j][d] = fw0[j] . pe[:,d] + fb0[j]; gb[o][d] = fw2[o] . relu(hid[:,d]) + fb2[o]
// (H hidden units, P code rows: EnergyFiLM3D(hidden, pe_dims), 32 and 16 by default)
// one workgroup = 32 of the 2C FiLM outputs of one block (the hidden layer recomputed per
// workgroup: H x P x D MACs)
__device__ __forceinline__ void efilm_fwd_body(const float* __restrict__ pe,
                                               const float* __restrict__ fw0,
                                               const float* __restrict__ fb0,
                                               const float* __restrict__ fw2,
                                               const float* __restrict__ fb2, float* __restrict__ t,
                                               float* __restrict__ bt, float* __restrict__ hid,
                                               int C, int D, int pitch, int wg, int H, int P) {
  extern __shared__ float hs[];  // [H][D] hidden, then pe [P][D] and fw0 [H][P] staged
  float* pes = hs + H * D;
  float* w0s = pes + P * D;
  for (int i = threadIdx.x; i < P * D; i += blockDim.x) pes[i] = pe[(i / D) * pitch + i % D];
  for (int i = threadIdx.x; i < H * P; i += blockDim.x) w0s[i] = fw0[i];
  __syncthreads();
  for (int i = threadIdx.x; i < H * D; i += blockDim.x) {
    const int j = i / D, d = i % D;
    float s = 0.f;
    for (int q = 0; q < P; ++q) s += w0s[j * P + q] * pes[q * D + d];
    s += fb0[j];
    hs[i] = s;
    if (wg == 0) hid[i] = s;
  }
  __syncthreads();
  const int o0 = wg * 32;
  for (int i = threadIdx.x; i < 32 * D; i += blockDim.x) {
    const int o = o0 + i / D, d = i % D;
    if (o >= 2 * C) continue;
    float s = 0.f;
    for (int j = 0; j < H; ++j) s += fw2[o * H + j] * fmaxf(hs[j * D + d], 0.f);
    s += fb2[o];
    if (o < C) t[o * D + d] = tanhf(s);
    else bt[(o - C) * D + d] = s;
  }
}
__global__ void k_efilm_fwd(const float* __restrict__ pe, const float* __restrict__ fw0,
                            const float* __restrict__ fb0, const float* __restrict__ fw2,
                            const float* __restrict__ fb2, float* __restrict__ t,
                            float* __restrict__ bt, float* __restrict__ hid, int C, int D,
                            int pitch, int H, int P) {
  efilm_fwd_body(pe, fw0, fb0, fw2, fb2, t, bt, hid, C, D, pitch, blockIdx.x, H, P);
}
// all blocks' coefficients in one launch: grid.y = job (block), grid.x = 32-output groups
__global__ void k_efilm_fwd_all(const float* __restrict__ pe, EfilmJobs jobs, int D, int pitch) {
  const EfilmJob& J = jobs.j[blockIdx.y];
  if ((int)blockIdx.x * 32 >= 2 * J.C) return;  // (uniform: the whole workgroup)
  efilm_fwd_body(pe, J.fw0, J.fb0, J.fw2, J.fb2, J.t, J.bt, J.hid, J.C, D, pitch, blockIdx.x,
                 jobs.H, jobs.P);
}

size_t efilm_fwd_lds(int H, int P, int D) {
  return ((size_t)(H + P) * D + (size_t)H * P) * sizeof(float);
}

hipError_t efilm_fwd_all(const float* pe, int pe_pitch, const EfilmJobs& jobs, int D,
                         hipStream_t s) {
  if (jobs.n <= 0) return hipSuccess;
  if (jobs.n > 8 || jobs.H < 1 || jobs.H > EFH_MAX || jobs.P < 1 || jobs.P > EFP_MAX)
    return hipErrorInvalidValue;
  const size_t shm = efilm_fwd_lds(jobs.H, jobs.P, D);
  if (shm > 64 * 1024) {
    if (shm > GATE_LDS_MAX) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_efilm_fwd_all),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
  }
  int gx = 1;
  for (int i = 0; i < jobs.n; ++i) gx = std::max(gx, cdiv(2 * jobs.j[i].C, 32));
  hipLaunchKernelGGL(k_efilm_fwd_all, dim3(gx, jobs.n), dim3(256), shm, s, pe, jobs, D, pe_pitch);
  return hipGetLastError();
}

static hipError_t efilm_fwd(const GateParams& gp, const GateSaved& sv, int C, int D,
                            hipStream_t s) {
  const size_t shm = efilm_fwd_lds(gp.efh, gp.efp, D);
  if (shm > 64 * 1024) {
    if (shm > GATE_LDS_MAX) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_efilm_fwd),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_efilm_fwd, dim3(cdiv(2 * C, 32)), dim3(256), shm, s, gp.pe + gp.d_off,
                     gp.fw0, gp.fb0, gp.fw2, gp.fb2, sv.t, sv.bt, sv.hid, C, D, gp.pe_pitch,
                     gp.efh, gp.efp);
  return hipGetLastError();
}

// ------------------------------------------------------------- gates fwd --
struct GFShm {
  double *twc, *tws, *Sre, *Sim, *part, *tmp;
  float *s1, *g1, *sg2, *p, *h, *e, *zc;
};
__device__ GFShm gf_carve(void* base, int C, int D, int Hse) {
  const int L = D / 2 + 1;
  GFShm m;
  double* dp = reinterpret_cast<double*>(base);
  m.twc = dp; dp += D;
  m.tws = dp; dp += D;
  m.Sre = dp; dp += L;
  m.Sim = dp; dp += L;
  m.part = dp; dp += GT;
  m.tmp = dp; dp += (C > D ? C : D) + 1;
  float* fp = reinterpret_cast<float*>(dp);
  m.s1 = fp; fp += D;
  m.g1 = fp; fp += D;
  m.sg2 = fp; fp += D;
  m.p = fp; fp += C;
  m.h = fp; fp += Hse;
  m.e = fp; fp += C;
  m.zc = fp;  // [C][D] (cached kernels only)
  return m;
}
// cached: Z[c][d] staged in LDS once (one parallel pass over the inputs) so the
// serial chain of row sums reads LDS, not HBM/L2 -- these one-workgroup-per-
// sample kernels are latency-bound
static size_t gates_fwd_shmem(int C, int D, int Hse, bool cached) {
  const int L = D / 2 + 1;
  return (2 * (size_t)D + 2 * L + GT + (C > D ? C : D) + 1) * sizeof(double) +
         (3 * (size_t)D + 2 * C + Hse + (cached ? (size_t)C * D : 0)) * sizeof(float);
}

template <bool CACHED>
__global__ __launch_bounds__(GT) void k_gates_fwd(GateParams gp, const float* __restrict__ Sa,
                                                  GateSaved sv, Vol vol, int C, int Hse,
                                                  int efilm) {
  const int b = blockIdx.x;
  const int D = vol.D, HW = vol.H * vol.W, L = D / 2 + 1;
  extern __shared__ double shd[];
  GFShm m = gf_carve(shd, C, D, Hse);
  const float* Sab = Sa + (int64_t)b * C * D;
  auto Zg = [&](int c, int d) -> float {
    const float sa = Sab[c * D + d];
    return efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
  };
  auto Z = [&](int c, int d) -> float { return CACHED ? m.zc[c * D + d] : Zg(c, d); };
  if (CACHED) {
    for (int i = threadIdx.x; i < C * D; i += blockDim.x) m.zc[i] = Zg(i / D, i % D);
    __syncthreads();
  }
  make_twiddles(m.twc, m.tws, D);
  // s1[d] = mean_{c,hw} z
  rowsum(D, C, [&](int d, int c) { return (double)Z(c, d); }, m.part, 1.0 / ((double)C * HW),
         m.tmp);
  for (int d = threadIdx.x; d < D; d += blockDim.x) m.s1[d] = (float)m.tmp[d];
  __syncthreads();
  if (gp.mask) {
    rowsum(L, D, [&](int k, int d) { return (double)m.s1[d] * m.twc[(k * d) % D]; }, m.part, 1.0,
           m.Sre);
    rowsum(L, D, [&](int k, int d) { return -(double)m.s1[d] * m.tws[(k * d) % D]; }, m.part, 1.0,
           m.Sim);
    rowsum(D, L, [&](int d, int k) {
      const int q = (k * d) % D;
      const double Mk = (double)(gp.mask[k] * gp.mag[0]);
      return ck_coef(k, D) * Mk * (m.Sre[k] * m.twc[q] - m.Sim[k] * m.tws[q]) +
             phase_term(gp.fphase, k, D, m.Sre[k], m.Sim[k], m.twc[q], m.tws[q]);
    }, m.part, 1.0 / D, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = sigm((float)m.tmp[d]);
  } else {
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = 1.f;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    m.sg2[d] = gp.specse ? sigm(m.g1[d] * m.s1[d]) : 1.f;
  __syncthreads();
  if (gp.sw0) {
    rowsum(C, D, [&](int c, int d) { return (double)(m.g1[d] * m.sg2[d]) * (double)Z(c, d); },
           m.part, 1.0 / ((double)D * HW), m.tmp);
    for (int c = threadIdx.x; c < C; c += blockDim.x) m.p[c] = (float)m.tmp[c];
    __syncthreads();
    for (int j = threadIdx.x; j < Hse; j += blockDim.x) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += gp.sw0[j * C + c] * m.p[c];
      m.h[j] = s + gp.sb0[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < Hse; ++j) s += gp.sw2[c * Hse + j] * fmaxf(m.h[j], 0.f);
      m.e[c] = sigm(s + gp.sb2[c]);
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) m.e[c] = 1.f;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    sv.s1[b * D + d] = m.s1[d];
    sv.g1[b * D + d] = m.g1[d];
    sv.sg2[b * D + d] = m.sg2[d];
  }
  if (gp.sw0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) { sv.p[b * C + c] = m.p[c]; sv.e[b * C + c] = m.e[c]; }
    for (int j = threadIdx.x; j < Hse; j += blockDim.x) sv.h[b * Hse + j] = m.h[j];
  }
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    const int c = i / D, d = i % D;
    const float G = m.g1[d] * m.sg2[d] * m.e[c];
    const float onept = efilm ? (1.f + sv.t[i]) : 1.f;
    const float btv = efilm ? sv.bt[i] : 0.f;
    sv.P[(int64_t)b * C * D + i] = onept * G;
    sv.Q[(int64_t)b * C * D + i] = btv * G;
    if (sv.PT) {  // [B][D][C] copies for the GEMM loaders (ActRows)
      sv.PT[((int64_t)b * D + d) * C + c] = onept * G;
      sv.QT[((int64_t)b * D + d) * C + c] = btv * G;
    }
  }
}

// ------------------------------------------------------------- gates bwd --
// scratch layout (floats): dt[B][C][D], dbt[B][C][D], sw2p[B][C][Hse], sb2p[B][C],
// sw0p[B][Hse][C], sb0p[B][Hse], dMr[B][L], dgb[2C][D], dh[EFiLM hidden][D]
struct GScr {
  float *dt, *dbt, *sw2p, *sb2p, *sw0p, *sb0p, *dMr, *dgb, *dh;
};
static GScr gscr(float* base, int B, int C, int D, int Hse) {
  const int L = D / 2 + 1;
  GScr g;
  g.dt = base;
  g.dbt = g.dt + (size_t)B * C * D;
  g.sw2p = g.dbt + (size_t)B * C * D;
  g.sb2p = g.sw2p + (size_t)B * C * Hse;
  g.sw0p = g.sb2p + (size_t)B * C;
  g.sb0p = g.sw0p + (size_t)B * Hse * C;
  g.dMr = g.sb0p + (size_t)B * Hse;
  g.dgb = g.dMr + (size_t)B * L;
  g.dh = g.dgb + (size_t)2 * C * D;
  return g;
}
static size_t gates_base_bytes(Vol vol, int C) {
  const int B = vol.B, D = vol.D, Hse = se_hidden(C), L = D / 2 + 1;
  size_t n = 2 * (size_t)B * C * D + (size_t)B * C * Hse + (size_t)B * C + (size_t)B * Hse * C +
             (size_t)B * Hse + (size_t)B * L + 2 * (size_t)C * D + EFH_MAX * (size_t)D;
  return (n * sizeof(float) + 256 + 255) / 256 * 256;
}
// (channel-split kernels, below) partial column sums [B][C/8][D] (double, twice), the SE
// channel sums u and c0 [B][C], and the FourierGate / spectral-SE depth terms [B][D] (twice)
static size_t gates_split_bytes(Vol vol, int C) {
  const size_t B = vol.B, D = vol.D, nch = (C + 7) / 8;
  return 2 * B * nch * D * sizeof(double) + 2 * B * C * sizeof(float) + 2 * B * D * sizeof(float) +
         256;
}
size_t gates_scratch_bytes(Vol vol, int C) {
  return gates_base_bytes(vol, C) + gates_split_bytes(vol, C);
}

struct GBShm {
  double *twc, *tws, *Sre, *Sim, *Tre, *Tim, *part, *tmp;
  float *e, *c0, *dq, *dh, *g1, *sg2, *ds2, *dw, *ds1, *zc, *rc;
};
__device__ GBShm gb_carve(void* base, int C, int D, int Hse) {
  const int L = D / 2 + 1;
  GBShm m;
  double* dp = reinterpret_cast<double*>(base);
  m.twc = dp; dp += D;
  m.tws = dp; dp += D;
  m.Sre = dp; dp += L;
  m.Sim = dp; dp += L;
  m.Tre = dp; dp += L;
  m.Tim = dp; dp += L;
  m.part = dp; dp += GT;
  m.tmp = dp; dp += (C > D ? C : D) + 1;
  float* fp = reinterpret_cast<float*>(dp);
  m.e = fp; fp += C;
  m.c0 = fp; fp += C;
  m.dq = fp; fp += C;
  m.dh = fp; fp += Hse;
  m.g1 = fp; fp += D;
  m.sg2 = fp; fp += D;
  m.ds2 = fp; fp += D;
  m.dw = fp; fp += D;
  m.ds1 = fp; fp += D;
  m.rc = fp; fp += (size_t)C * D;  // [C][D] R1, then Z (cached kernels only)
  m.zc = fp;
  return m;
}
// ncache: how many of the [C][D] inputs R1, Z are staged in LDS (2, 1 = R1 only, 0)
static size_t gates_bwd_shmem(int C, int D, int Hse, int ncache) {
  const int L = D / 2 + 1;
  return (2 * (size_t)D + 4 * L + GT + (C > D ? C : D) + 1) * sizeof(double) +
         (3 * (size_t)C + Hse + 5 * (size_t)D + (size_t)ncache * C * D) * sizeof(float);
}

template <int NCACHE>
__global__ __launch_bounds__(GT) void k_gates_bwd(GateParams gp, GateSaved sv,
                                                  const float* __restrict__ Sa,
                                                  const float* __restrict__ Sg, GScr gs,
                                                  float* __restrict__ Aout,
                                                  float* __restrict__ Bout, Vol vol, int C,
                                                  int Hse, int efilm) {
  const int b = blockIdx.x;
  const int D = vol.D, HW = vol.H * vol.W, L = D / 2 + 1;
  extern __shared__ double shd[];
  GBShm m = gb_carve(shd, C, D, Hse);
  const int64_t bo = (int64_t)b * C * D;
  auto Zg = [&](int c, int d) -> float {
    const float sa = Sa[bo + c * D + d];
    return efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
  };
  auto R1g = [&](int c, int d) -> float {  // sum_hw dout * z
    const float sgd = Sg[(bo + c * D + d) * 2 + 0], sda = Sg[(bo + c * D + d) * 2 + 1];
    return efilm ? (1.f + sv.t[c * D + d]) * sda + sv.bt[c * D + d] * sgd : sda;
  };
  auto Zf = [&](int c, int d) -> float { return NCACHE >= 2 ? m.zc[c * D + d] : Zg(c, d); };
  auto R1 = [&](int c, int d) -> float { return NCACHE >= 1 ? m.rc[c * D + d] : R1g(c, d); };
  for (int i = threadIdx.x; NCACHE >= 1 && i < C * D; i += blockDim.x) {
    m.rc[i] = R1g(i / D, i % D);
    if (NCACHE >= 2) m.zc[i] = Zg(i / D, i % D);
  }
  make_twiddles(m.twc, m.tws, D);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.g1[d] = sv.g1[b * D + d];
    m.sg2[d] = sv.sg2[b * D + d];
  }
  __syncthreads();
  // ---- channel SE: out = v * e[c] ----
  if (gp.sw0) {
    rowsum(C, D, [&](int c, int d) { return (double)(m.g1[d] * m.sg2[d]) * (double)R1(c, d); },
           m.part, 1.0, m.tmp);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float ev = sv.e[b * C + c];
      m.e[c] = ev;
      m.dq[c] = (float)m.tmp[c] * ev * (1.f - ev);
      gs.sb2p[b * C + c] = m.dq[c];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C * Hse; i += blockDim.x) {
      const int c = i / Hse, j = i % Hse;
      gs.sw2p[(int64_t)b * C * Hse + i] = m.dq[c] * fmaxf(sv.h[b * Hse + j], 0.f);
    }
    for (int j = threadIdx.x; j < Hse; j += blockDim.x) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += gp.sw2[c * Hse + j] * m.dq[c];
      const float dhv = sv.h[b * Hse + j] > 0.f ? s : 0.f;
      m.dh[j] = dhv;
      gs.sb0p[b * Hse + j] = dhv;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < Hse * C; i += blockDim.x) {
      const int j = i / C, c = i % C;
      gs.sw0p[(int64_t)b * Hse * C + i] = m.dh[j] * sv.p[b * C + c];
    }
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < Hse; ++j) s += gp.sw0[j * C + c] * m.dh[j];
      m.c0[c] = s / ((float)D * (float)HW);
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) { m.e[c] = 1.f; m.c0[c] = 0.f; }
  }
  __syncthreads();
  // ---- spectral SE: v = u * sg2[d] ----
  // T[d] = sum_c (e[c] R1(c,d) + c0[c] Z(c,d)) serves both gates: the spectral SE's
  // gradient, and the FourierGate's sum_c (a R1 + bb Z) with a = e[c] sg2[d],
  // bb = c0[c] sg2[d] + ds2[d] / (C HW), which is sg2[d] T[d] + ds2[d] s1[d] because
  // sum_c Z(c,d) = C HW s1[d] (the forward's mean over (c, hw)) -- one pass over the
  // [C][D] inputs instead of two
  if (gp.specse || gp.mask) {
    rowsum(D, C, [&](int d, int c) {
      return (double)m.e[c] * R1(c, d) + (double)m.c0[c] * Zf(c, d);
    }, m.part, 1.0, m.tmp);
  }
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    m.ds2[d] = gp.specse ? m.sg2[d] * (1.f - m.sg2[d]) * m.g1[d] * (float)m.tmp[d] : 0.f;
  __syncthreads();
  const float invCHW = 1.f / ((float)C * (float)HW);
  // du = dout*a + bb, a = e[c]*sg2[d], bb = c0[c]*sg2[d] + ds2[d]/(C*HW)
  // ---- FourierGate: u = z * g1[d] ----
  if (gp.mask) {
    const float* s1f = sv.s1 + b * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const double t = (double)m.sg2[d] * m.tmp[d] + (double)m.ds2[d] * s1f[d];
      m.dw[d] = (float)t * m.g1[d] * (1.f - m.g1[d]);
    }
    __syncthreads();
    const float* s1 = sv.s1 + b * D;
    rowsum(L, D, [&](int k, int d) { return (double)s1[d] * m.twc[(k * d) % D]; }, m.part, 1.0, m.Sre);
    rowsum(L, D, [&](int k, int d) { return -(double)s1[d] * m.tws[(k * d) % D]; }, m.part, 1.0, m.Sim);
    rowsum(L, D, [&](int k, int d) { return (double)m.dw[d] * m.twc[(k * d) % D]; }, m.part, 1.0, m.Tre);
    rowsum(L, D, [&](int k, int d) { return (double)m.dw[d] * m.tws[(k * d) % D]; }, m.part, 1.0, m.Tim);
    for (int k = threadIdx.x; k < L; k += blockDim.x)
      gs.dMr[b * L + k] =
          (float)(ck_coef(k, D) / D * (m.Sre[k] * m.Tre[k] - m.Sim[k] * m.Tim[k]));
    rowsum(D, L, [&](int d, int k) {
      const int q = (k * d) % D;
      const double Mk = (double)(gp.mask[k] * gp.mag[0]);
      return ck_coef(k, D) * Mk * (m.twc[q] * m.Tre[k] + m.tws[q] * m.Tim[k]) +
             phase_term_t(gp.fphase, k, D, m.Tre[k], m.Tim[k], m.twc[q], m.tws[q]);
    }, m.part, 1.0 / D, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.ds1[d] = (float)m.tmp[d];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    const int c = i / D, d = i % D;
    float al = m.e[c] * m.sg2[d];
    float be = m.c0[c] * m.sg2[d] + m.ds2[d] * invCHW;
    if (gp.mask) {
      al = al * m.g1[d];
      be = be * m.g1[d] + m.ds1[d] * invCHW;
    }
    if (efilm) {
      const float sgd = Sg[(bo + i) * 2 + 0], sda = Sg[(bo + i) * 2 + 1];
      gs.dt[bo + i] = al * sda + be * Sa[bo + i];
      gs.dbt[bo + i] = al * sgd + be * (float)HW;
      const float onept = 1.f + sv.t[i];
      al *= onept;
      be *= onept;
    }
    Aout[bo + i] = al;
    Bout[bo + i] = be;
  }
}

// sums over b of the per-b partials -> SE and FourierGate grads
__global__ void k_gates_bwd_final(GateParams gp, GateGrads gg, GScr gs, int B, int C, int D,
                                  int Hse) {
  const int L = D / 2 + 1;
  const int n1 = C * Hse, n2 = C, n3 = Hse * C, n4 = Hse, n5 = L;
  const int tot = (gp.sw0 ? n1 + n2 + n3 + n4 : 0) + (gp.mask ? n5 : 0);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
    int k = i;
    if (gp.sw0) {
      if (k < n1) { float s = 0.f; for (int b = 0; b < B; ++b) s += gs.sw2p[(int64_t)b * n1 + k]; gg.sw2[k] = s; continue; }
      k -= n1;
      if (k < n2) { float s = 0.f; for (int b = 0; b < B; ++b) s += gs.sb2p[(int64_t)b * n2 + k]; gg.sb2[k] = s; continue; }
      k -= n2;
      if (k < n3) { float s = 0.f; for (int b = 0; b < B; ++b) s += gs.sw0p[(int64_t)b * n3 + k]; gg.sw0[k] = s; continue; }
      k -= n3;
      if (k < n4) { float s = 0.f; for (int b = 0; b < B; ++b) s += gs.sb0p[(int64_t)b * n4 + k]; gg.sb0[k] = s; continue; }
      k -= n4;
    }
    // FourierGate: M = mask * mag
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += gs.dMr[b * L + k];
    gg.mask[k] = s * gp.mag[0];
  }
  // d mag = sum_k mask_k sum_b dMr[b][k]: one wave, lanes over k, a fixed shuffle tree
  // (a single thread walking the L x B terms took most of this kernel's 15 us)
  if (gp.mask && blockIdx.x == 0 && threadIdx.x < 64) {
    float t = 0.f;
    for (int k = threadIdx.x; k < L; k += 64) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += gs.dMr[b * L + k];
      t += s * gp.mask[k];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) gg.mag[0] = t;
  }
}

// EFiLM MLP backward: dgb[o][d] (o<C: dt*(1-t^2), o>=C: dbt), then
// dfw2 = dgb . relu(hid)^T, dfb2 = sum_d dgb, dh = (fw2^T dgb) * (hid>0),
// dfw0 = dh . pe^T, dfb0 = sum_d dh.
__global__ void k_efilm_bwd1(GScr gs, const float* __restrict__ t, int B, int C, int D) {
  const int n = 2 * C * D;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int o = i / D, d = i % D;
    float s = 0.f;
    if (o < C) {
      for (int b = 0; b < B; ++b) s += gs.dt[(int64_t)b * C * D + o * D + d];
      const float tv = t[o * D + d];
      s *= (1.f - tv * tv);
    } else {
      for (int b = 0; b < B; ++b) s += gs.dbt[(int64_t)b * C * D + (o - C) * D + d];
    }
    gs.dgb[i] = s;
  }
}
// one wave per output: lanes take strided slices of the reduction, then a fixed
// shuffle tree (deterministic; 64x shorter dependent chains than a thread per
// output -- these tiny kernels are latency-bound)
__device__ __forceinline__ float gate_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__global__ __launch_bounds__(256) void k_efilm_bwd2(GateParams gp, GateGrads gg, GScr gs,
                                                    const float* __restrict__ hid, int C, int D) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int H = gp.efh, H1 = H + 1;
  if (i >= 2 * C * H1 + H * D) return;
  float s = 0.f;
  if (i < 2 * C * H1) {
    const int o = i / H1, j = i % H1;
    if (j < H) {
      for (int d = lane; d < D; d += 64) s += gs.dgb[o * D + d] * fmaxf(hid[j * D + d], 0.f);
      s = gate_wave_sum(s);
      if (lane == 0) gg.fw2[o * H + j] = s;
    } else {
      for (int d = lane; d < D; d += 64) s += gs.dgb[o * D + d];
      s = gate_wave_sum(s);
      if (lane == 0) gg.fb2[o] = s;
    }
  } else {
    const int k = i - 2 * C * H1;
    const int j = k / D, d = k % D;
    for (int o = lane; o < 2 * C; o += 64) s += gp.fw2[o * H + j] * gs.dgb[o * D + d];
    s = gate_wave_sum(s);
    if (lane == 0) gs.dh[k] = hid[k] > 0.f ? s : 0.f;
  }
}
__global__ __launch_bounds__(256) void k_efilm_bwd3(GateParams gp, GateGrads gg, GScr gs,
                                                    int D) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int P = gp.efp, P1 = P + 1;
  if (i >= gp.efh * P1) return;
  const int j = i / P1, q = i % P1;
  float s = 0.f;
  if (q < P) {
    const float* pe = gp.pe + q * gp.pe_pitch + gp.d_off;
    for (int d = lane; d < D; d += 64) s += gs.dh[j * D + d] * pe[d];
    s = gate_wave_sum(s);
    if (lane == 0) gg.fw0[j * P + q] = s;
  } else {
    for (int d = lane; d < D; d += 64) s += gs.dh[j * D + d];
    s = gate_wave_sum(s);
    if (lane == 0) gg.fb0[j] = s;
  }
}

// SE / FourierGate parameter grads (sums over b) and the EFiLM MLP backward.
// Lf = the spectrum length of the FULL depth (sharded plans: D_glob / 2 + 1).
static hipError_t gates_bwd_tail(const GateParams& gp, const GateSaved& sv, GateGrads& gg,
                                 const GScr& g, int B, int C, int D, int Dfull, int Hse,
                                 hipStream_t s) {
  hipError_t e;
  if (gp.sw0 || gp.mask) {
    hipLaunchKernelGGL(k_gates_bwd_final, dim3(64), dim3(256), 0, s, gp, gg, g, B, C, Dfull, Hse);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (gp.fw0) {
    hipLaunchKernelGGL(k_efilm_bwd1, dim3(std::min(cdiv(2 * C * D, 256), 1024)), dim3(256), 0, s,
                       g, sv.t, B, C, D);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (gp.efh < 1 || gp.efh > EFH_MAX || gp.efp < 1 || gp.efp > EFP_MAX)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_efilm_bwd2, dim3(cdiv(2 * C * (gp.efh + 1) + gp.efh * D, 4)), dim3(256),
                       0, s, gp, gg, g, sv.hid, C, D);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_efilm_bwd3, dim3(cdiv(gp.efh * (gp.efp + 1), 4)), dim3(256), 0, s, gp, gg,
                       g, D);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

// ================================================ channel-split kernels ==
// The one-workgroup-per-sample kernels above keep two CUs busy; at the deeper levels
// (C x D up to 256 x 128 per sample) their [C][D] passes dominate (k_gates_bwd: 148 us for
// the bottleneck block).  Here every [C][D] pass runs over 8-channel chunks, grid
// (C / 8, B) -- column sums as fixed-order partials per chunk, row sums one wave per
// channel -- and only the serial D-length chain (spectra, DFT, sigmoids) stays on one
// workgroup per sample.  Same algebra as k_gates_fwd / k_gates_bwd.
namespace {
constexpr int GCH = 8;      // channels per chunk
constexpr int GST = 256;    // threads of the chunk kernels
struct GSplit {
  double *ps1, *Tp;        // [B][nch][D]
  float *u, *c0;           // [B][C]
  float *ds2, *ds1;        // [B][D]
};
GSplit gsplit(float* scratch, Vol vol, int C) {
  char* p = reinterpret_cast<char*>(scratch) + gates_base_bytes(vol, C);
  const size_t B = vol.B, D = vol.D, nch = (C + GCH - 1) / GCH;
  GSplit g;
  g.ps1 = reinterpret_cast<double*>(p); p += B * nch * D * sizeof(double);
  g.Tp = reinterpret_cast<double*>(p); p += B * nch * D * sizeof(double);
  g.u = reinterpret_cast<float*>(p); p += B * C * sizeof(float);
  g.c0 = reinterpret_cast<float*>(p); p += B * C * sizeof(float);
  g.ds2 = reinterpret_cast<float*>(p); p += B * D * sizeof(float);
  g.ds1 = reinterpret_cast<float*>(p);
  return g;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
}  // namespace

// split path for C x D >= SPFF_GSPLIT_MIN (C a multiple of 8, at most 1024 channels; the
// chain kernels' LDS -- twiddles, spectra and the 2 / 4 x GT partials of the merged row
// sums, no [C][D] caches -- fits for D <= 1024)
static bool gates_split(int C, int D) {
  return (int64_t)C * D >= SPFF_GSPLIT_MIN && C % GCH == 0 && C <= 1024 && D <= 1024;
}

// fwd 1: partial s1 numerators of one 8-channel chunk, ps1[b][ch][d] = sum_{c in ch} Z(c, d)
__global__ __launch_bounds__(GST) void k_gfs_colsum(const float* __restrict__ Sa, GateSaved sv,
                                                   Vol vol, int C, int efilm, GSplit sp) {
  const int ch = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  const int D = vol.D, HW = vol.H * vol.W;
  const float* Sab = Sa + (int64_t)b * C * D;
  const int c1 = min(C, (ch + 1) * GCH);
  for (int d = threadIdx.x; d < D; d += GST) {
    double acc = 0.0;
    for (int c = ch * GCH; c < c1; ++c) {
      const float sa = Sab[c * D + d];
      acc += (double)(efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa);
    }
    sp.ps1[((int64_t)b * nch + ch) * D + d] = acc;
  }
}

// fwd 2 (one workgroup per sample): s1 from the chunk partials (fixed order), the
// FourierGate's DFT chain -> g1, the spectral SE -> sg2
__global__ __launch_bounds__(GT) void k_gfs_chain(GateParams gp, GateSaved sv, Vol vol, int C,
                                                  int nch, GSplit sp, int part_off) {
  const int b = blockIdx.x;
  const int D = vol.D, HW = vol.H * vol.W, L = D / 2 + 1;
  extern __shared__ double shd[];
  GFShm m = gf_carve(shd, C, D, 0);
  double* part4 = shd + part_off;  // 2 x GT doubles after the carve
  make_twiddles(m.twc, m.tws, D);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    double acc = 0.0;
    for (int ch = 0; ch < nch; ++ch) acc += sp.ps1[((int64_t)b * nch + ch) * D + d];
    m.s1[d] = (float)(acc / ((double)C * HW));
  }
  __syncthreads();
  if (gp.mask) {
    double* outs[2] = {m.Sre, m.Sim};
    rowsum_n<2>(L, D, [&](int k, int d, double* v) {
      const int q = (k * d) % D;
      v[0] = (double)m.s1[d] * m.twc[q];
      v[1] = -(double)m.s1[d] * m.tws[q];
    }, part4, 1.0, outs);
    rowsum(D, L, [&](int d, int k) {
      const int q = (k * d) % D;
      const double Mk = (double)(gp.mask[k] * gp.mag[0]);
      return ck_coef(k, D) * Mk * (m.Sre[k] * m.twc[q] - m.Sim[k] * m.tws[q]) +
             phase_term(gp.fphase, k, D, m.Sre[k], m.Sim[k], m.twc[q], m.tws[q]);
    }, m.part, 1.0 / D, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = sigm((float)m.tmp[d]);
  } else {
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = 1.f;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float sg = gp.specse ? sigm(m.g1[d] * m.s1[d]) : 1.f;
    sv.s1[b * D + d] = m.s1[d];
    sv.g1[b * D + d] = m.g1[d];
    sv.sg2[b * D + d] = sg;
  }
}

// fwd 3 (SE): p[b][c] = sum_d g1 sg2 Z(c, d) / (D HW), one wave per channel
__global__ __launch_bounds__(GST) void k_gfs_pool(const float* __restrict__ Sa, GateSaved sv,
                                                 Vol vol, int C, int efilm) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int c = blockIdx.x * (GST / 64) + (threadIdx.x >> 6);
  if (c >= C) return;  // (whole wave)
  const int D = vol.D, HW = vol.H * vol.W;
  const float* Sab = Sa + (int64_t)b * C * D;
  double acc = 0.0;
  for (int d = lane; d < D; d += 64) {
    const float sa = Sab[c * D + d];
    const float z = efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
    acc += (double)(sv.g1[b * D + d] * sv.sg2[b * D + d]) * (double)z;
  }
  acc = wave_sum_d(acc);
  if (lane == 0) sv.p[b * C + c] = (float)(acc / ((double)D * HW));
}

// fwd 4: the SE MLP (each chunk recomputes the Hse hidden units from p, a C x Hse dot),
// e of this chunk's channels, then P / Q (and the [B][D][C] copies) of its channels
__global__ __launch_bounds__(GST) void k_gfs_apply(GateParams gp, GateSaved sv, Vol vol, int C,
                                                  int Hse, int efilm) {
  const int ch = blockIdx.x, b = blockIdx.y;
  const int D = vol.D, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float hs[64], es[GCH];
  const int c0 = ch * GCH, c1 = min(C, c0 + GCH);
  if (gp.sw0) {
    for (int j = wave; j < Hse; j += GST / 64) {
      float acc = 0.f;
      for (int c = lane; c < C; c += 64) acc += gp.sw0[j * C + c] * sv.p[b * C + c];
      acc = gate_wave_sum(acc);
      if (lane == 0) hs[j] = acc + gp.sb0[j];
    }
    __syncthreads();
    if (ch == 0)
      for (int j = threadIdx.x; j < Hse; j += GST) sv.h[b * Hse + j] = hs[j];
    for (int c = c0 + (int)threadIdx.x; c < c1; c += GST) {
      float acc = 0.f;
      for (int j = 0; j < Hse; ++j) acc += gp.sw2[c * Hse + j] * fmaxf(hs[j], 0.f);
      const float ev = sigm(acc + gp.sb2[c]);
      es[c - c0] = ev;
      sv.e[b * C + c] = ev;
    }
  } else {
    for (int c = c0 + (int)threadIdx.x; c < c1; c += GST) es[c - c0] = 1.f;
  }
  __syncthreads();
  const int n = (c1 - c0) * D;
  for (int i = threadIdx.x; i < n; i += GST) {
    const int c = c0 + i / D, d = i % D;
    const int cd = c * D + d;
    const float G = sv.g1[b * D + d] * sv.sg2[b * D + d] * es[c - c0];
    const float onept = efilm ? (1.f + sv.t[cd]) : 1.f;
    const float btv = efilm ? sv.bt[cd] : 0.f;
    sv.P[(int64_t)b * C * D + cd] = onept * G;
    sv.Q[(int64_t)b * C * D + cd] = btv * G;
    if (sv.PT) {
      sv.PT[((int64_t)b * D + d) * C + c] = onept * G;
      sv.QT[((int64_t)b * D + d) * C + c] = btv * G;
    }
  }
}

// bwd 1 (SE): u[b][c] = sum_d g1 sg2 R1(c, d), one wave per channel
__global__ __launch_bounds__(GST) void k_gbs_rowsum(const float* __restrict__ Sg, GateSaved sv,
                                                   Vol vol, int C, int efilm, GSplit sp) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int c = blockIdx.x * (GST / 64) + (threadIdx.x >> 6);
  if (c >= C) return;
  const int D = vol.D;
  const int64_t bo = (int64_t)b * C * D;
  double acc = 0.0;
  for (int d = lane; d < D; d += 64) {
    const int64_t i = bo + c * D + d;
    const float sgd = Sg[i * 2 + 0], sda = Sg[i * 2 + 1];
    const float r1 = efilm ? (1.f + sv.t[c * D + d]) * sda + sv.bt[c * D + d] * sgd : sda;
    acc += (double)(sv.g1[b * D + d] * sv.sg2[b * D + d]) * (double)r1;
  }
  acc = wave_sum_d(acc);
  if (lane == 0) sp.u[b * C + c] = (float)acc;
}

// bwd 2: the SE backward (each chunk recomputes dh from all channels' dq, a C x Hse dot;
// writes its channels' SE gradient partials, chunk 0 the hidden ones), c0 of its channels,
// and the partial T[d] = sum_{c in chunk} (e R1 + c0 Z) for the spectral SE / FourierGate
__global__ __launch_bounds__(GST) void k_gbs_colsum(GateParams gp, GateSaved sv,
                                                   const float* __restrict__ Sa,
                                                   const float* __restrict__ Sg, GScr gs, Vol vol,
                                                   int C, int Hse, int efilm, GSplit sp) {
  const int ch = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  const int D = vol.D, HW = vol.H * vol.W, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float dq[1024], dh[64], ec[GCH], cc[GCH];
  const int c0 = ch * GCH, c1 = min(C, c0 + GCH);
  const int64_t bo = (int64_t)b * C * D;
  if (gp.sw0) {
    for (int c = threadIdx.x; c < C; c += GST) {
      const float ev = sv.e[b * C + c];
      dq[c] = sp.u[b * C + c] * ev * (1.f - ev);
    }
    __syncthreads();
    for (int j = wave; j < Hse; j += GST / 64) {
      float acc = 0.f;
      for (int c = lane; c < C; c += 64) acc += gp.sw2[c * Hse + j] * dq[c];
      acc = gate_wave_sum(acc);
      if (lane == 0) dh[j] = sv.h[b * Hse + j] > 0.f ? acc : 0.f;
    }
    __syncthreads();
    if (ch == 0)
      for (int j = threadIdx.x; j < Hse; j += GST) gs.sb0p[b * Hse + j] = dh[j];
    for (int c = c0 + (int)threadIdx.x; c < c1; c += GST) {
      gs.sb2p[b * C + c] = dq[c];
      float acc = 0.f;
      for (int j = 0; j < Hse; ++j) acc += gp.sw0[j * C + c] * dh[j];
      const float c0v = acc / ((float)D * (float)HW);
      cc[c - c0] = c0v;
      ec[c - c0] = sv.e[b * C + c];
      sp.c0[b * C + c] = c0v;
    }
    for (int i = threadIdx.x; i < (c1 - c0) * Hse; i += GST) {
      const int c = c0 + i / Hse, j = i % Hse;
      gs.sw2p[(int64_t)b * C * Hse + c * Hse + j] = dq[c] * fmaxf(sv.h[b * Hse + j], 0.f);
    }
    for (int i = threadIdx.x; i < Hse * (c1 - c0); i += GST) {
      const int j = i / (c1 - c0), c = c0 + i % (c1 - c0);
      gs.sw0p[(int64_t)b * Hse * C + j * C + c] = dh[j] * sv.p[b * C + c];
    }
  } else {
    for (int c = c0 + (int)threadIdx.x; c < c1; c += GST) {
      cc[c - c0] = 0.f;
      ec[c - c0] = 1.f;
      sp.c0[b * C + c] = 0.f;
    }
  }
  if (!(gp.specse || gp.mask)) return;
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += GST) {
    double acc = 0.0;
    for (int c = c0; c < c1; ++c) {
      const int64_t i = bo + c * D + d;
      const float sgd = Sg[i * 2 + 0], sda = Sg[i * 2 + 1];
      const float tt = efilm ? sv.t[c * D + d] : 0.f;
      const float r1 = efilm ? (1.f + tt) * sda + sv.bt[c * D + d] * sgd : sda;
      const float sa = Sa[i];
      const float z = efilm ? (1.f + tt) * sa + sv.bt[c * D + d] * (float)HW : sa;
      acc += (double)ec[c - c0] * r1 + (double)cc[c - c0] * z;
    }
    sp.Tp[((int64_t)b * nch + ch) * D + d] = acc;
  }
}

// bwd 3 (one workgroup per sample): T from the chunk partials, the spectral SE's ds2 and the
// FourierGate's spectra / mask gradient partials / ds1
__global__ __launch_bounds__(GT) void k_gbs_chain(GateParams gp, GateSaved sv, GScr gs, Vol vol,
                                                  int C, int nch, GSplit sp, int part_off) {
  const int b = blockIdx.x;
  const int D = vol.D, L = D / 2 + 1;
  extern __shared__ double shd[];
  GBShm m = gb_carve(shd, C, D, 0);
  make_twiddles(m.twc, m.tws, D);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    double acc = 0.0;
    if (gp.specse || gp.mask)
      for (int ch = 0; ch < nch; ++ch) acc += sp.Tp[((int64_t)b * nch + ch) * D + d];
    m.tmp[d] = acc;
    const float g1 = sv.g1[b * D + d], sg2 = sv.sg2[b * D + d];
    m.g1[d] = g1;
    m.sg2[d] = sg2;
    const float ds2 = gp.specse ? sg2 * (1.f - sg2) * g1 * (float)acc : 0.f;
    m.ds2[d] = ds2;
    sp.ds2[b * D + d] = ds2;
    if (!gp.mask) sp.ds1[b * D + d] = 0.f;
  }
  __syncthreads();
  if (!gp.mask) return;
  const float* s1 = sv.s1 + b * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const double t = (double)m.sg2[d] * m.tmp[d] + (double)m.ds2[d] * s1[d];
    m.dw[d] = (float)t * m.g1[d] * (1.f - m.g1[d]);
  }
  __syncthreads();
  {
    double* part4 = shd + part_off;  // 4 x GT doubles after the carve
    double* outs[4] = {m.Sre, m.Sim, m.Tre, m.Tim};
    rowsum_n<4>(L, D, [&](int k, int d, double* v) {
      const int q = (k * d) % D;
      const double c = m.twc[q], sn = m.tws[q];
      v[0] = (double)s1[d] * c;
      v[1] = -(double)s1[d] * sn;
      v[2] = (double)m.dw[d] * c;
      v[3] = (double)m.dw[d] * sn;
    }, part4, 1.0, outs);
  }
  for (int k = threadIdx.x; k < L; k += blockDim.x)
    gs.dMr[b * L + k] = (float)(ck_coef(k, D) / D * (m.Sre[k] * m.Tre[k] - m.Sim[k] * m.Tim[k]));
  rowsum(D, L, [&](int d, int k) {
    const int q = (k * d) % D;
    const double Mk = (double)(gp.mask[k] * gp.mag[0]);
    return ck_coef(k, D) * Mk * (m.twc[q] * m.Tre[k] + m.tws[q] * m.Tim[k]) +
           phase_term_t(gp.fphase, k, D, m.Tre[k], m.Tim[k], m.twc[q], m.tws[q]);
  }, m.part, 1.0 / D, m.tmp);
  for (int d = threadIdx.x; d < D; d += blockDim.x) sp.ds1[b * D + d] = (float)m.tmp[d];
}

// bwd 4: A / B (and the EnergyFiLM partials dt, dbt) of this chunk's channels
__global__ __launch_bounds__(GST) void k_gbs_apply(GateParams gp, GateSaved sv,
                                                  const float* __restrict__ Sa,
                                                  const float* __restrict__ Sg, GScr gs,
                                                  float* __restrict__ Aout,
                                                  float* __restrict__ Bout, Vol vol, int C,
                                                  int efilm, GSplit sp) {
  const int ch = blockIdx.x, b = blockIdx.y;
  const int D = vol.D, HW = vol.H * vol.W;
  const int c0 = ch * GCH, c1 = min(C, c0 + GCH);
  const int64_t bo = (int64_t)b * C * D;
  const float invCHW = 1.f / ((float)C * (float)HW);
  const int n = (c1 - c0) * D;
  for (int i = threadIdx.x; i < n; i += GST) {
    const int c = c0 + i / D, d = i % D;
    const int cd = c * D + d;
    const float e = gp.sw0 ? sv.e[b * C + c] : 1.f;
    const float sg2 = sv.sg2[b * D + d], g1 = sv.g1[b * D + d];
    float al = e * sg2;
    float be = sp.c0[b * C + c] * sg2 + sp.ds2[b * D + d] * invCHW;
    if (gp.mask) {
      al = al * g1;
      be = be * g1 + sp.ds1[b * D + d] * invCHW;
    }
    if (efilm) {
      const float sgd = Sg[(bo + cd) * 2 + 0], sda = Sg[(bo + cd) * 2 + 1];
      gs.dt[bo + cd] = al * sda + be * Sa[bo + cd];
      gs.dbt[bo + cd] = al * sgd + be * (float)HW;
      const float onept = 1.f + sv.t[cd];
      al *= onept;
      be *= onept;
    }
    Aout[bo + cd] = al;
    Bout[bo + cd] = be;
  }
}

hipError_t gates_fwd(const GateParams& gp, const float* Sa, GateSaved& sv, Vol vol, int C,
                     float* scratch, hipStream_t s) {
  const int D = vol.D, Hse = se_hidden(C);
  const int efilm = gp.fw0 != nullptr;
  if (efilm && !gp.efilm_ready) {
    hipError_t e = efilm_fwd(gp, sv, C, D, s);
    if (e != hipSuccess) return e;
  }
  if (gates_split(C, D)) {
    const GSplit sp = gsplit(scratch, vol, C);
    const int nch = C / GCH;
    hipLaunchKernelGGL(k_gfs_colsum, dim3(nch, vol.B), dim3(GST), 0, s, Sa, sv, vol, C, efilm, sp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int off = (int)((gates_fwd_shmem(C, D, 0, false) + 15) / 16 * 2);  // (doubles)
    const size_t shm = (off + 2 * GT) * sizeof(double);
    if (shm > 64 * 1024 &&
        (e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gfs_chain),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(k_gfs_chain, dim3(vol.B), dim3(GT), shm, s, gp, sv, vol, C, nch, sp, off);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (gp.sw0) {
      hipLaunchKernelGGL(k_gfs_pool, dim3(cdiv(C, GST / 64), vol.B), dim3(GST), 0, s, Sa, sv, vol, C,
                         efilm);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_gfs_apply, dim3(nch, vol.B), dim3(GST), 0, s, gp, sv, vol, C, Hse, efilm);
    return hipGetLastError();
  }
  const size_t shc = gates_fwd_shmem(C, D, Hse, true);
  if (shc <= GATE_LDS_MAX) {
    hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gates_fwd<true>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shc);
    if (e0 != hipSuccess) return e0;
    hipLaunchKernelGGL(k_gates_fwd<true>, dim3(vol.B), dim3(GT), shc, s, gp, Sa, sv, vol, C, Hse,
                       efilm);
  } else {
    hipLaunchKernelGGL(k_gates_fwd<false>, dim3(vol.B), dim3(GT),
                       gates_fwd_shmem(C, D, Hse, false), s, gp, Sa, sv, vol, C, Hse, efilm);
  }
  return hipGetLastError();
}

hipError_t gates_bwd(const GateParams& gp, const GateSaved& sv, const float* Sa, const float* Sg,
                     GateGrads& gg, float* A, float* Bc, Vol vol, int C, float* scratch,
                     hipStream_t s) {
  const int D = vol.D, B = vol.B, Hse = se_hidden(C);
  const int efilm = gp.fw0 != nullptr;
  GScr g = gscr(scratch, B, C, D, Hse);
  if (gates_split(C, D)) {
    const GSplit sp = gsplit(scratch, vol, C);
    const int nch = C / GCH;
    hipError_t e;
    if (gp.sw0) {
      hipLaunchKernelGGL(k_gbs_rowsum, dim3(cdiv(C, GST / 64), B), dim3(GST), 0, s, Sg, sv, vol, C,
                         efilm, sp);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_gbs_colsum, dim3(nch, B), dim3(GST), 0, s, gp, sv, Sa, Sg, g, vol, C, Hse,
                       efilm, sp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int off = (int)((gates_bwd_shmem(C, D, 0, 0) + 15) / 16 * 2);  // (doubles)
    const size_t shm = (off + 4 * GT) * sizeof(double);
    if (shm > 64 * 1024) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gbs_chain),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_gbs_chain, dim3(B), dim3(GT), shm, s, gp, sv, g, vol, C, nch, sp, off);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_gbs_apply, dim3(nch, B), dim3(GST), 0, s, gp, sv, Sa, Sg, g, A, Bc, vol, C,
                       efilm, sp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return gates_bwd_tail(gp, sv, gg, g, B, C, D, D, Hse, s);
  }
  int nc = 2;
  while (nc > 0 && gates_bwd_shmem(C, D, Hse, nc) > GATE_LDS_MAX) --nc;
  const size_t shm = gates_bwd_shmem(C, D, Hse, nc);
  auto kern = nc == 2 ? k_gates_bwd<2> : nc == 1 ? k_gates_bwd<1> : k_gates_bwd<0>;
  if (shm > 64 * 1024) {
    hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e0 != hipSuccess) return e0;
  }
  hipLaunchKernelGGL(kern, dim3(B), dim3(GT), shm, s, gp, sv, Sa, Sg, g, A, Bc, vol, C, Hse,
                     efilm);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return gates_bwd_tail(gp, sv, gg, g, B, C, D, D, Hse, s);
}

// ====================================================== depth-sharded path ==
// The slab holds depths [d_off, d_off + D) of Dg.  s1, g1, sg2, P, Q and the
// EFiLM coefficients are per depth (local).  The FourierGate needs the
// spectrum of the FULL s1: each slab adds its depths' terms (at their global
// indices) and the partial spectra are all-reduced -- likewise the SE pool p[c]
// and, backward, sum_d g1 sg2 R1 and the spectrum of dw.  Gradients of the SE
// and FourierGate parameters are functions of those replicated totals: rank 0
// writes them, the others write zeros, so the flat gradient all-reduce counts
// them once.  EFiLM gradients are sums over the local depths (partials).
namespace {
struct ShScr {
  double *ppart, *depart, *Tpart;
  float *dw, *ds2, *c0, *dMr;
};
size_t sh_base(Vol vol, int C) { return (gates_scratch_bytes(vol, C) + 255) / 256 * 256; }
ShScr shscr(float* base, Vol vol, int C, int Dg) {
  char* p = reinterpret_cast<char*>(base) + sh_base(vol, C);
  const int B = vol.B, L = Dg / 2 + 1, D = vol.D;
  ShScr r;
  r.ppart = reinterpret_cast<double*>(p); p += (size_t)B * C * 8;
  r.depart = reinterpret_cast<double*>(p); p += (size_t)B * C * 8;
  r.Tpart = reinterpret_cast<double*>(p); p += (size_t)B * L * 16;
  r.dw = reinterpret_cast<float*>(p); p += (size_t)B * D * 4;
  r.ds2 = reinterpret_cast<float*>(p); p += (size_t)B * D * 4;
  r.c0 = reinterpret_cast<float*>(p); p += (size_t)B * C * 4;
  r.dMr = reinterpret_cast<float*>(p);
  return r;
}
struct ShShm {
  double *twc, *tws, *part, *tmp, *Sre, *Sim, *Tre, *Tim;
  float *s1, *g1, *sg2, *e, *c0, *ds2, *dw, *ds1;
};
__device__ ShShm sh_carve(void* base, int C, int D, int Dg) {
  const int L = Dg / 2 + 1, M = (C > D ? C : D) > L ? (C > D ? C : D) : L;
  ShShm m;
  double* dp = reinterpret_cast<double*>(base);
  m.twc = dp; dp += Dg;
  m.tws = dp; dp += Dg;
  m.part = dp; dp += GT;
  m.tmp = dp; dp += M + 1;
  m.Sre = dp; dp += L;
  m.Sim = dp; dp += L;
  m.Tre = dp; dp += L;
  m.Tim = dp; dp += L;
  float* fp = reinterpret_cast<float*>(dp);
  m.s1 = fp; fp += D;
  m.g1 = fp; fp += D;
  m.sg2 = fp; fp += D;
  m.ds2 = fp; fp += D;
  m.dw = fp; fp += D;
  m.ds1 = fp; fp += D;
  m.e = fp; fp += C;
  m.c0 = fp;
  return m;
}
size_t sh_shmem(int C, int D, int Dg) {
  const int L = Dg / 2 + 1, M = std::max(std::max(C, D), L);
  return (2 * (size_t)Dg + GT + M + 1 + 4 * (size_t)L) * sizeof(double) +
         (6 * (size_t)D + 2 * (size_t)C) * sizeof(float);
}
}  // namespace

size_t gates_sh_scratch_bytes(Vol vol, int C, int Dg) {
  const int B = vol.B, L = Dg / 2 + 1;
  return sh_base(vol, C) + (size_t)B * C * 16 + (size_t)B * L * 16 + (size_t)B * vol.D * 8 +
         (size_t)B * C * 4 + (size_t)B * L * 4 + 256;
}

// fwd A: s1 (local depths) and its partial spectrum -> sv.spec
__global__ __launch_bounds__(GT) void k_gsh_fwd_a(GateParams gp, const float* __restrict__ Sa,
                                                  GateSaved sv, Vol vol, int C, int efilm,
                                                  int d_off, int Dg) {
  const int b = blockIdx.x, D = vol.D, HW = vol.H * vol.W, L = Dg / 2 + 1;
  extern __shared__ double shd[];
  ShShm m = sh_carve(shd, C, D, Dg);
  const float* Sab = Sa + (int64_t)b * C * D;
  auto Z = [&](int c, int d) -> float {
    const float sa = Sab[c * D + d];
    return efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
  };
  make_twiddles(m.twc, m.tws, Dg);
  rowsum(D, C, [&](int d, int c) { return (double)Z(c, d); }, m.part, 1.0 / ((double)C * HW),
         m.tmp);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.s1[d] = (float)m.tmp[d];
    sv.s1[b * D + d] = m.s1[d];
  }
  __syncthreads();
  if (gp.mask) {
    rowsum(L, D, [&](int k, int d) { return (double)m.s1[d] * m.twc[(k * (d_off + d)) % Dg]; },
           m.part, 1.0, m.Sre);
    rowsum(L, D, [&](int k, int d) { return -(double)m.s1[d] * m.tws[(k * (d_off + d)) % Dg]; },
           m.part, 1.0, m.Sim);
    for (int k = threadIdx.x; k < L; k += blockDim.x) {
      sv.spec[((int64_t)b * L + k) * 2 + 0] = m.Sre[k];
      sv.spec[((int64_t)b * L + k) * 2 + 1] = m.Sim[k];
    }
  }
}

// fwd B: gates from the full spectrum; SE pool partial -> ppart
__global__ __launch_bounds__(GT) void k_gsh_fwd_b(GateParams gp, const float* __restrict__ Sa,
                                                  GateSaved sv, Vol vol, int C, int efilm,
                                                  int d_off, int Dg, ShScr sc) {
  const int b = blockIdx.x, D = vol.D, HW = vol.H * vol.W, L = Dg / 2 + 1;
  extern __shared__ double shd[];
  ShShm m = sh_carve(shd, C, D, Dg);
  const float* Sab = Sa + (int64_t)b * C * D;
  auto Z = [&](int c, int d) -> float {
    const float sa = Sab[c * D + d];
    return efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
  };
  make_twiddles(m.twc, m.tws, Dg);
  for (int d = threadIdx.x; d < D; d += blockDim.x) m.s1[d] = sv.s1[b * D + d];
  if (gp.mask)
    for (int k = threadIdx.x; k < L; k += blockDim.x) {
      m.Sre[k] = sv.spec[((int64_t)b * L + k) * 2 + 0];
      m.Sim[k] = sv.spec[((int64_t)b * L + k) * 2 + 1];
    }
  __syncthreads();
  if (gp.mask) {
    rowsum(D, L, [&](int d, int k) {
      const int q = (k * (d_off + d)) % Dg;
      const double Mk = (double)(gp.mask[k] * gp.mag[0]);
      return ck_coef(k, Dg) * Mk * (m.Sre[k] * m.twc[q] - m.Sim[k] * m.tws[q]) +
             phase_term(gp.fphase, k, Dg, m.Sre[k], m.Sim[k], m.twc[q], m.tws[q]);
    }, m.part, 1.0 / Dg, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = sigm((float)m.tmp[d]);
  } else {
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.g1[d] = 1.f;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.sg2[d] = gp.specse ? sigm(m.g1[d] * m.s1[d]) : 1.f;
    sv.g1[b * D + d] = m.g1[d];
    sv.sg2[b * D + d] = m.sg2[d];
  }
  __syncthreads();
  if (gp.sw0) {
    rowsum(C, D, [&](int c, int d) { return (double)(m.g1[d] * m.sg2[d]) * (double)Z(c, d); },
           m.part, 1.0 / ((double)Dg * HW), m.tmp);
    for (int c = threadIdx.x; c < C; c += blockDim.x) sc.ppart[(int64_t)b * C + c] = m.tmp[c];
  }
}

// fwd C: SE MLP on the all-reduced pool; apply coefficients P, Q
__global__ __launch_bounds__(GT) void k_gsh_fwd_c(GateParams gp, GateSaved sv, Vol vol, int C,
                                                  int Hse, int efilm, ShScr sc) {
  const int b = blockIdx.x, D = vol.D;
  __shared__ float pp[1024], hh[64], ee[1024];
  if (gp.sw0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      pp[c] = (float)sc.ppart[(int64_t)b * C + c];
      sv.p[b * C + c] = pp[c];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < Hse; j += blockDim.x) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += gp.sw0[j * C + c] * pp[c];
      hh[j] = s + gp.sb0[j];
      sv.h[b * Hse + j] = hh[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < Hse; ++j) s += gp.sw2[c * Hse + j] * fmaxf(hh[j], 0.f);
      ee[c] = sigm(s + gp.sb2[c]);
      sv.e[b * C + c] = ee[c];
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) ee[c] = 1.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    const int c = i / D, d = i % D;
    const float G = sv.g1[b * D + d] * sv.sg2[b * D + d] * ee[c];
    const float onept = efilm ? (1.f + sv.t[i]) : 1.f;
    const float btv = efilm ? sv.bt[i] : 0.f;
    sv.P[(int64_t)b * C * D + i] = onept * G;
    sv.Q[(int64_t)b * C * D + i] = btv * G;
    if (sv.PT) {  // [B][D][C] copies for the GEMM loaders (ActRows)
      sv.PT[((int64_t)b * D + d) * C + c] = onept * G;
      sv.QT[((int64_t)b * D + d) * C + c] = btv * G;
    }
  }
}

hipError_t gates_fwd_sh(const GateParams& gp, const float* Sa, GateSaved& sv, Vol vol, int C,
                        float* scratch, const Coll& co, hipStream_t s) {
  const int D = vol.D, B = vol.B, Hse = se_hidden(C), Dg = co.D_glob, L = Dg / 2 + 1;
  const int efilm = gp.fw0 != nullptr;
  if (C > 1024 || Hse > 64) return hipErrorInvalidValue;
  hipError_t e;
  if (efilm && !gp.efilm_ready) {
    if ((e = efilm_fwd(gp, sv, C, D, s)) != hipSuccess) return e;
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  ShScr sc = shscr(scratch, vol, C, Dg);
  const size_t shm = sh_shmem(C, D, Dg);
  hipLaunchKernelGGL(k_gsh_fwd_a, dim3(B), dim3(GT), shm, s, gp, Sa, sv, vol, C, efilm, co.d_off,
                     Dg);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (gp.mask && (e = co.sum_f64(sv.spec, (int64_t)B * L * 2, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_gsh_fwd_b, dim3(B), dim3(GT), shm, s, gp, Sa, sv, vol, C, efilm, co.d_off,
                     Dg, sc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (gp.sw0 && (e = co.sum_f64(sc.ppart, (int64_t)B * C, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_gsh_fwd_c, dim3(B), dim3(GT), 0, s, gp, sv, vol, C, Hse, efilm, sc);
  return hipGetLastError();
}

// bwd A: de[c] partial = sum_{local d} g1 sg2 R1
__global__ __launch_bounds__(GT) void k_gsh_bwd_a(GateParams gp, GateSaved sv,
                                                  const float* __restrict__ Sa,
                                                  const float* __restrict__ Sg, Vol vol, int C,
                                                  int efilm, int Dg, ShScr sc) {
  const int b = blockIdx.x, D = vol.D;
  extern __shared__ double shd[];
  ShShm m = sh_carve(shd, C, D, Dg);
  const int64_t bo = (int64_t)b * C * D;
  auto R1 = [&](int c, int d) -> float {
    const float sgd = Sg[(bo + c * D + d) * 2 + 0], sda = Sg[(bo + c * D + d) * 2 + 1];
    return efilm ? (1.f + sv.t[c * D + d]) * sda + sv.bt[c * D + d] * sgd : sda;
  };
  (void)Sa;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.g1[d] = sv.g1[b * D + d];
    m.sg2[d] = sv.sg2[b * D + d];
  }
  __syncthreads();
  rowsum(C, D, [&](int c, int d) { return (double)(m.g1[d] * m.sg2[d]) * (double)R1(c, d); },
         m.part, 1.0, m.tmp);
  for (int c = threadIdx.x; c < C; c += blockDim.x) sc.depart[(int64_t)b * C + c] = m.tmp[c];
}

// bwd B: SE grads (owner), c0, ds2, dw (local) and the partial spectrum of dw
__global__ __launch_bounds__(GT) void k_gsh_bwd_b(GateParams gp, GateSaved sv,
                                                  const float* __restrict__ Sa,
                                                  const float* __restrict__ Sg, GScr gs, Vol vol,
                                                  int C, int Hse, int efilm, int d_off, int Dg,
                                                  int owner, ShScr sc) {
  const int b = blockIdx.x, D = vol.D, HW = vol.H * vol.W, L = Dg / 2 + 1;
  extern __shared__ double shd[];
  ShShm m = sh_carve(shd, C, D, Dg);
  __shared__ float dq[1024], dh[64];
  const int64_t bo = (int64_t)b * C * D;
  auto Zf = [&](int c, int d) -> float {
    const float sa = Sa[bo + c * D + d];
    return efilm ? (1.f + sv.t[c * D + d]) * sa + sv.bt[c * D + d] * (float)HW : sa;
  };
  auto R1 = [&](int c, int d) -> float {
    const float sgd = Sg[(bo + c * D + d) * 2 + 0], sda = Sg[(bo + c * D + d) * 2 + 1];
    return efilm ? (1.f + sv.t[c * D + d]) * sda + sv.bt[c * D + d] * sgd : sda;
  };
  make_twiddles(m.twc, m.tws, Dg);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.g1[d] = sv.g1[b * D + d];
    m.sg2[d] = sv.sg2[b * D + d];
  }
  __syncthreads();
  if (gp.sw0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float ev = sv.e[b * C + c];
      m.e[c] = ev;
      dq[c] = (float)sc.depart[(int64_t)b * C + c] * ev * (1.f - ev);
      gs.sb2p[b * C + c] = owner ? dq[c] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C * Hse; i += blockDim.x) {
      const int c = i / Hse, j = i % Hse;
      gs.sw2p[(int64_t)b * C * Hse + i] = owner ? dq[c] * fmaxf(sv.h[b * Hse + j], 0.f) : 0.f;
    }
    for (int j = threadIdx.x; j < Hse; j += blockDim.x) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += gp.sw2[c * Hse + j] * dq[c];
      const float dhv = sv.h[b * Hse + j] > 0.f ? s : 0.f;
      dh[j] = dhv;
      gs.sb0p[b * Hse + j] = owner ? dhv : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < Hse * C; i += blockDim.x) {
      const int j = i / C, c = i % C;
      gs.sw0p[(int64_t)b * Hse * C + i] = owner ? dh[j] * sv.p[b * C + c] : 0.f;
    }
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < Hse; ++j) s += gp.sw0[j * C + c] * dh[j];
      m.c0[c] = s / ((float)Dg * (float)HW);
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) { m.e[c] = 1.f; m.c0[c] = 0.f; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) sc.c0[(int64_t)b * C + c] = m.c0[c];
  if (gp.specse) {
    rowsum(D, C, [&](int d, int c) {
      return (double)m.e[c] * R1(c, d) + (double)m.c0[c] * Zf(c, d);
    }, m.part, 1.0, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      m.ds2[d] = m.sg2[d] * (1.f - m.sg2[d]) * m.g1[d] * (float)m.tmp[d];
  } else {
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.ds2[d] = 0.f;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) sc.ds2[b * D + d] = m.ds2[d];
  const float invCHW = 1.f / ((float)C * (float)HW);
  if (gp.mask) {
    rowsum(D, C, [&](int d, int c) {
      const float a = m.e[c] * m.sg2[d];
      const float bb = m.c0[c] * m.sg2[d] + m.ds2[d] * invCHW;
      return (double)a * R1(c, d) + (double)bb * Zf(c, d);
    }, m.part, 1.0, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      m.dw[d] = (float)m.tmp[d] * m.g1[d] * (1.f - m.g1[d]);
      sc.dw[b * D + d] = m.dw[d];
    }
    __syncthreads();
    rowsum(L, D, [&](int k, int d) { return (double)m.dw[d] * m.twc[(k * (d_off + d)) % Dg]; },
           m.part, 1.0, m.Tre);
    rowsum(L, D, [&](int k, int d) { return (double)m.dw[d] * m.tws[(k * (d_off + d)) % Dg]; },
           m.part, 1.0, m.Tim);
    for (int k = threadIdx.x; k < L; k += blockDim.x) {
      sc.Tpart[((int64_t)b * L + k) * 2 + 0] = m.Tre[k];
      sc.Tpart[((int64_t)b * L + k) * 2 + 1] = m.Tim[k];
    }
  }
}

// bwd C: FourierGate mask grads (owner), ds1 and the per-(c,d) A / Bc outputs
__global__ __launch_bounds__(GT) void k_gsh_bwd_c(GateParams gp, GateSaved sv,
                                                  const float* __restrict__ Sa,
                                                  const float* __restrict__ Sg, GScr gs,
                                                  float* __restrict__ Aout,
                                                  float* __restrict__ Bout, Vol vol, int C,
                                                  int efilm, int d_off, int Dg, int owner,
                                                  ShScr sc) {
  const int b = blockIdx.x, D = vol.D, HW = vol.H * vol.W, L = Dg / 2 + 1;
  extern __shared__ double shd[];
  ShShm m = sh_carve(shd, C, D, Dg);
  const int64_t bo = (int64_t)b * C * D;
  make_twiddles(m.twc, m.tws, Dg);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    m.g1[d] = sv.g1[b * D + d];
    m.sg2[d] = sv.sg2[b * D + d];
    m.ds2[d] = sc.ds2[b * D + d];
    m.ds1[d] = 0.f;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    m.e[c] = gp.sw0 ? sv.e[b * C + c] : 1.f;
    m.c0[c] = sc.c0[(int64_t)b * C + c];
  }
  if (gp.mask)
    for (int k = threadIdx.x; k < L; k += blockDim.x) {
      m.Sre[k] = sv.spec[((int64_t)b * L + k) * 2 + 0];
      m.Sim[k] = sv.spec[((int64_t)b * L + k) * 2 + 1];
      m.Tre[k] = sc.Tpart[((int64_t)b * L + k) * 2 + 0];
      m.Tim[k] = sc.Tpart[((int64_t)b * L + k) * 2 + 1];
    }
  __syncthreads();
  if (gp.mask) {
    for (int k = threadIdx.x; k < L; k += blockDim.x)
      gs.dMr[b * L + k] =
          owner ? (float)(ck_coef(k, Dg) / Dg * (m.Sre[k] * m.Tre[k] - m.Sim[k] * m.Tim[k]))
                : 0.f;
    rowsum(D, L, [&](int d, int k) {
      const int q = (k * (d_off + d)) % Dg;
      const double Mk = (double)(gp.mask[k] * gp.mag[0]);
      return ck_coef(k, Dg) * Mk * (m.twc[q] * m.Tre[k] + m.tws[q] * m.Tim[k]) +
             phase_term_t(gp.fphase, k, Dg, m.Tre[k], m.Tim[k], m.twc[q], m.tws[q]);
    }, m.part, 1.0 / Dg, m.tmp);
    for (int d = threadIdx.x; d < D; d += blockDim.x) m.ds1[d] = (float)m.tmp[d];
    __syncthreads();
  }
  const float invCHW = 1.f / ((float)C * (float)HW);
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    const int c = i / D, d = i % D;
    float al = m.e[c] * m.sg2[d];
    float be = m.c0[c] * m.sg2[d] + m.ds2[d] * invCHW;
    if (gp.mask) {
      al = al * m.g1[d];
      be = be * m.g1[d] + m.ds1[d] * invCHW;
    }
    if (efilm) {
      const float sgd = Sg[(bo + i) * 2 + 0], sda = Sg[(bo + i) * 2 + 1];
      gs.dt[bo + i] = al * sda + be * Sa[bo + i];
      gs.dbt[bo + i] = al * sgd + be * (float)HW;
      const float onept = 1.f + sv.t[i];
      al *= onept;
      be *= onept;
    }
    Aout[bo + i] = al;
    Bout[bo + i] = be;
  }
}

hipError_t gates_bwd_sh(const GateParams& gp, const GateSaved& sv, const float* Sa,
                        const float* Sg, GateGrads& gg, float* A, float* Bc, Vol vol, int C,
                        float* scratch, const Coll& co, hipStream_t s) {
  const int D = vol.D, B = vol.B, Hse = se_hidden(C), Dg = co.D_glob, L = Dg / 2 + 1;
  const int efilm = gp.fw0 != nullptr, owner = co.rank == 0;
  if (C > 1024 || Hse > 64) return hipErrorInvalidValue;
  GScr g = gscr(scratch, B, C, D, Hse);
  ShScr sc = shscr(scratch, vol, C, Dg);
  g.dMr = sc.dMr;  // [B][L] of the full depth
  const size_t shm = sh_shmem(C, D, Dg);
  hipError_t e;
  if (gp.sw0) {
    hipLaunchKernelGGL(k_gsh_bwd_a, dim3(B), dim3(GT), shm, s, gp, sv, Sa, Sg, vol, C, efilm, Dg,
                       sc);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = co.sum_f64(sc.depart, (int64_t)B * C, s)) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_gsh_bwd_b, dim3(B), dim3(GT), shm, s, gp, sv, Sa, Sg, g, vol, C, Hse, efilm,
                     co.d_off, Dg, owner, sc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (gp.mask && (e = co.sum_f64(sc.Tpart, (int64_t)B * L * 2, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_gsh_bwd_c, dim3(B), dim3(GT), shm, s, gp, sv, Sa, Sg, g, A, Bc, vol, C,
                     efilm, co.d_off, Dg, owner, sc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return gates_bwd_tail(gp, sv, gg, g, B, C, D, Dg, Hse, s);
}

}  // namespace spff
