// cnslmat/bf16-split.h -- the exact three-way bf16 split of fp32 operands
// used by every bf16x6 kernel (x6-util.h, kaldi-lite/cu-gemm-x6.hip).
//
// x = h + m + l with h, m, l bf16: h is x truncated to bf16 (its top 16
// bits), m the residual x - h truncated the same way, l = x - h - m (at most
// 8 significant bits, so exact in bf16).  Truncation keeps |h| <= |x|, so
// no part overflows for any finite x (a rounding split sends finite
// |x| >= 3.3961e38 to h = Inf and the product to NaN), and every partial
// product is at most |a*b|.  Residual sizes: |m| < 2^-7 |x|, |l| < 2^-15 |x|;
// the three products the kernels drop (ml, lm, ll) are < 2^-21 |a*b|, well
// inside the 1e-5 * S parity bound.  Each pair costs the same 11 VALU ops as
// the rounding split (v_perm_b32 packs two truncated halves in one op).
// ±Inf / NaN operands give NaN parts (Inf - Inf): see DESIGN.md §4.
#ifndef KCNN_CNSLMAT_BF16_SPLIT_H_
#define KCNN_CNSLMAT_BF16_SPLIT_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kcnn {
namespace x6 {

// (x0, x1) -> packed bf16 pairs h, m, l (element 0 in the low half)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t &h, uint32_t &m,
                                       uint32_t &l) {
  const uint32_t b0 = __float_as_uint(x0), b1 = __float_as_uint(x1);
  const float r0 = x0 - __uint_as_float(b0 & 0xffff0000u);
  const float r1 = x1 - __uint_as_float(b1 & 0xffff0000u);
  const uint32_t c0 = __float_as_uint(r0), c1 = __float_as_uint(r1);
  const float l0 = r0 - __uint_as_float(c0 & 0xffff0000u);
  const float l1 = r1 - __uint_as_float(c1 & 0xffff0000u);
  h = __builtin_amdgcn_perm(b1, b0, 0x07060302u);
  m = __builtin_amdgcn_perm(c1, c0, 0x07060302u);
  l = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
}

}  // namespace x6
}  // namespace kcnn

#endif  // KCNN_CNSLMAT_BF16_SPLIT_H_
