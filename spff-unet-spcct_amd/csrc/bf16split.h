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
// float4 -> NS planes of 4 bf16 (x: values 0,1; y: values 2,3)
template <int NS>
__device__ __forceinline__ void split4_pk(const float4& v, uint2 (&o)[NS]) {
  unsigned lo[NS], hi[NS];
  split_pair<NS>(v.x, v.y, lo);
  split_pair<NS>(v.z, v.w, hi);
#pragma unroll
  for (int p = 0; p < NS; ++p) o[p] = make_uint2(lo[p], hi[p]);
}

}  // namespace spff
