// Exact split of fp32 operands into NS bf16 planes, x = h + m + l (+ remainder), in the
// packed form the MFMA operand images hold: two values per dword, the first in the low half.
//
// Per pair of values a plane costs one v_cvt_pk_bf16_f32 (both values, round to nearest
// even, the same conversion a scalar (__bf16) cast emits), the bf16 -> fp32 widening is a
// shift / mask of the packed dword, and the remainder is one exact v_sub_f32 per value.
// The subtraction is an asm helper: a plain -O3 build SLP-packs the adjacent pair into
// v_pk_add_f32, which beside MFMAs costs more issue cycles than two single subtractions
// (MI355X_MICROARCH.md, "price of one filler beside MFMAs").  Round 2's per-value split
// (one conversion per value, then shifts / ors to pack) took ~70 VALU instructions per
// float4 in the conv kernels' k-loops; this takes 26.  Results are bitwise identical.
#pragma once

#include <hip/hip_runtime.h>

namespace spff {

typedef float spff_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 spff_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((spff_f32x2){a, b}, spff_bf16x2));
}
__device__ __forceinline__ float vsub_f32(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (a, b) -> NS packed planes o[p] = bf16(a_p) | bf16(b_p) << 16
template <int NS>
__device__ __forceinline__ void split_pair(float a, float b, unsigned (&o)[NS]) {
#pragma unroll
  for (int p = 0; p < NS; ++p) {
    const unsigned h = cvt_pk_bf16(a, b);
    o[p] = h;
    if (p + 1 < NS) {
      a = vsub_f32(a, __uint_as_float(h << 16));
      b = vsub_f32(b, __uint_as_float(h & 0xffff0000u));
    }
  }
}
// ---- scaled fp16 planes (SPFF_MATH_F16X3) ----
// The split kernels' template parameter NS is the plane count, or NS_F16 for two fp16
// planes of a power-of-two-scaled operand: x s = h + l, h = f16(x s), l = f16(x s - h)
// (round to nearest even; the subtraction is exact), |x s - h - l| <= 2^-22 |x s|.  The
// scale s = 2^e puts max|x s| below 2^14 (f16 max 65504), so no element overflows and the
// f16 subnormal floor (2^-25 absolute) is 2^-39 of the operand's largest element.  The
// products hh, hl, lh (3 MFMAs) drop l l <= 2^-22 |xy|.
constexpr int NS_F16 = 12;
__host__ __device__ constexpr int nplanes(int ns) { return ns == NS_F16 ? 2 : ns; }

typedef _Float16 spff_f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt_pk_f16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((spff_f32x2){a, b}, spff_f16x2));
}
// (a, b) -> 2 packed fp16 planes (values already scaled)
__device__ __forceinline__ void split_pair_f16(float a, float b, unsigned (&o)[2]) {
  const unsigned h = cvt_pk_f16(a, b);
  const spff_f16x2 hv = __builtin_bit_cast(spff_f16x2, h);
  o[0] = h;
  o[1] = cvt_pk_f16(vsub_f32(a, (float)hv.x), vsub_f32(b, (float)hv.y));
}
// scale exponent of an operand whose largest |element| has the float bits mbits (the
// slot an absmax kernel filled, 0 when empty): max |x| 2^e < 2^14, e in [-120, 120]
__device__ __forceinline__ int f16_scale_exp(unsigned mbits) {
  const int eb = (int)((mbits >> 23) & 0xffu);  // max < 2^(eb - 126) (eb 255: inf / nan)
  if (mbits == 0u || eb == 255) return 0;
  const int e = 14 - (eb - 126);
  return e < -120 ? -120 : (e > 120 ? 120 : e);
}
__device__ __forceinline__ float exp2i(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }

// the split kernels' MFMAs on operand fragments held as bf16x8 bit patterns: the bf16
// form, or (HF, NS_F16 planes) the fp16 form of the same shape and rate
typedef __bf16 spff_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 spff_f16x8 __attribute__((ext_vector_type(8)));
typedef float spff_f32x4 __attribute__((ext_vector_type(4)));
typedef float spff_f32x16 __attribute__((ext_vector_type(16)));
template <bool HF>
__device__ __forceinline__ spff_f32x4 mfma16x32(spff_bf16x8 a, spff_bf16x8 b, spff_f32x4 c) {
  if constexpr (HF)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(spff_f16x8, a),
                                                  __builtin_bit_cast(spff_f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <bool HF>
__device__ __forceinline__ spff_f32x16 mfma32x16(spff_bf16x8 a, spff_bf16x8 b, spff_f32x16 c) {
  if constexpr (HF)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(spff_f16x8, a),
                                                  __builtin_bit_cast(spff_f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// float4 -> NS planes of 4 bf16 (x: values 0,1; y: values 2,3); NS_F16: 2 fp16 planes
template <int NS>
__device__ __forceinline__ void split4_pk(const float4& v, uint2 (&o)[nplanes(NS)]) {
  constexpr int NP = nplanes(NS);
  unsigned lo[NP], hi[NP];
  if constexpr (NS == NS_F16) {
    split_pair_f16(v.x, v.y, lo);
    split_pair_f16(v.z, v.w, hi);
  } else {
    split_pair<NS>(v.x, v.y, lo);
    split_pair<NS>(v.z, v.w, hi);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) o[p] = make_uint2(lo[p], hi[p]);
}

}  // namespace spff
