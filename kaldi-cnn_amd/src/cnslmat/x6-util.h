// cnslmat/x6-util.h -- fp32 products on the bf16 matrix cores ("bf16x6").
//
// An fp32 value splits exactly into three bf16 parts, x = h + m + l (the
// truncating split of bf16-split.h: h, m, l hold successive bytes of the
// significand).  A product is
//   a*b = hh + (hm + mh) + (mm + hl + lh) + (ml + lm + ll)
// with the groups of relative size 1, < 2^-7, < 2^-14, < 2^-21; the first six
// products, one v_mfma_f32_32x32x16_bf16 each (32 cycles per SIMD), replace
// the fp32-input MFMA (v_mfma_f32_32x32x2_f32: 1/8 the work in 64 cycles,
// holding the SIMD's vector issue).  Accumulation is fp32 throughout.
#ifndef KCNN_CNSLMAT_X6_UTIL_H_
#define KCNN_CNSLMAT_X6_UTIL_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bf16-split.h"
#include "lds-dma.h"
#include "conv-geom.h"

namespace kcnn {
namespace x6 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  f32x2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// split2 (x = h + m + l, truncating): bf16-split.h
// eight values -> the three bf16x8 fragments
__device__ __forceinline__ void split8(const float *v, bf16x8 &h, bf16x8 &m, bf16x8 &l) {
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split2(v[2 * i], v[2 * i + 1], hh[i], mm[i], ll[i]);
  h = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
  m = __builtin_bit_cast(bf16x8, make_uint4(mm[0], mm[1], mm[2], mm[3]));
  l = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
}

__device__ __forceinline__ floatx16 mfma(const bf16x8 &a, const bf16x8 &b,
                                         const floatx16 &c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// the six products of a split pair (index 0 = h, 1 = m, 2 = l), small to large
__device__ __forceinline__ floatx16 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3],
                                          floatx16 c) {
  c = mfma(a[2], b[0], c);
  c = mfma(a[0], b[2], c);
  c = mfma(a[1], b[1], c);
  c = mfma(a[1], b[0], c);
  c = mfma(a[0], b[1], c);
  c = mfma(a[0], b[0], c);
  return c;
}

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

}  // namespace x6
}  // namespace kcnn

#endif  // KCNN_CNSLMAT_X6_UTIL_H_
