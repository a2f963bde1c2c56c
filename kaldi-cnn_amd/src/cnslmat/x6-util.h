// cnslmat/x6-util.h -- fp32 products on the bf16 matrix cores ("bf16x6").
//
// An fp32 value splits exactly into three bf16 parts, x = h + m + l with
// h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (each residual is exact
// in fp32 and keeps at most 16, then 8, significant bits).  A product is
//   a*b = hh + (hm + mh) + (mm + hl + lh) + (ml + lm + ll)
// with the groups of relative size 1, 2^-8, 2^-16, < 2^-24; the first six
// products, one v_mfma_f32_32x32x16_bf16 each (32 cycles per SIMD), replace
// the fp32-input MFMA (v_mfma_f32_32x32x2_f32: 1/8 the work in 64 cycles,
// holding the SIMD's vector issue).  The dropped three are below fp32's own
// rounding of a product; accumulation is fp32 throughout.
#ifndef KCNN_CNSLMAT_X6_UTIL_H_
#define KCNN_CNSLMAT_X6_UTIL_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

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
// (x0, x1) -> bf16 pairs h, m, l with x = h + m + l exactly (finite x)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t &h, uint32_t &m,
                                       uint32_t &l) {
  h = pack_bf16(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = pack_bf16(r0, r1);
  l = pack_bf16(r0 - __uint_as_float(m << 16), r1 - __uint_as_float(m & 0xffff0000u));
}
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

// Wait for this wave's outstanding vector-memory loads, LDS-DMA included
// (s_waitcnt vmcnt(0); gfx9 encoding: expcnt and lgkmcnt fields at their
// no-wait maxima).  An LDS-DMA load writes LDS, not VGPRs, so the compiler's
// own waits (placed before uses of loaded VGPRs) do not cover the LDS
// readers of another wave: put this before the barrier that publishes it.
__device__ __forceinline__ void wait_dma() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

}  // namespace x6
}  // namespace kcnn

#endif  // KCNN_CNSLMAT_X6_UTIL_H_
