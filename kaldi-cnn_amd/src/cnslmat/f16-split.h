// cnslmat/f16-split.h -- fp32 products on the f16 matrix cores ("f16x3").
//
// f16 carries 11 significant bits to bf16's 8, so two f16 parts hold an
// fp32 operand to 22 bits once it is scaled into f16's range by a power of
// two:
//
//   x' = x * 2^s   (s per scale group -- a GEMM row / column, a conv's whole
//                   kernel or one output position: the group's largest |x'|
//                   lies in [2^14, 2^15))
//   hi = f16(x'),  lo = f16(x' - hi)        (x' - hi is exact in fp32)
//
// x' = hi + lo to within 2^-22 |x'| while |x'| >= 2^-3; below that lo is an
// f16 subnormal and the error is under 2^-25 absolute, 2^-39 of the group's
// largest element.  Every f16 product is exact in fp32, so
//
//   a'b' = hi.hi + (hi.lo + lo.hi) + lo.lo
//
// and the kernels keep the first three (one v_mfma_f32_32x32x16_f16 each,
// smallest first, fp32 accumulation), then unscale by 2^-(s_a + s_b).  The
// error per product is under 3 * 2^-22 of |a b|, 14x inside the 1e-5 * S
// parity bound; the f16 MFMA runs at the bf16 rate, so this is
// half the matrix-core work of bf16x6 (x6-util.h) for fewer split VALU.
// Users: the FC GEMM (kaldi-lite/cu-gemm-f16x3.hip) and the frame-resident
// conv forward (cnsl-conv-frame.hip).
#ifndef KCNN_CNSLMAT_F16_SPLIT_H_
#define KCNN_CNSLMAT_F16_SPLIT_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kcnn {
namespace f16x3 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr uint32_t NONFINITE = 0x7f800000u;  // |x| bits >= this: Inf or NaN
constexpr int SKIP = 0x40000000;             // scale of an Inf / NaN group

// the scale exponent s for a group whose largest |x| has the bit pattern mb:
// max |x| * 2^s in [2^14, 2^15); SKIP for Inf / NaN, 0 for an all-zero group
__device__ __forceinline__ int scale_exp(uint32_t mb) {
  if (mb >= NONFINITE) return SKIP;
  if (mb == 0) return 0;
  const int e = mb >= 0x00800000u ? (int)(mb >> 23) - 127
                                  : (31 - (int)__builtin_clz(mb)) - 149;  // subnormal
  return 14 - e;
}

// a - (float)f16 half of h, in one v_fma_mix_f32 (a * 1.0 - h, exact here:
// h is a's f16 rounding, so the difference is an fp32 number)
#ifdef KCNN_F16_NOASM  // experiment: the same differences in plain C
__device__ __forceinline__ float sub_h0(float a, uint32_t h) {
  return a - (float)__builtin_bit_cast(f16x2, h)[0];
}
__device__ __forceinline__ float sub_h1(float a, uint32_t h) {
  return a - (float)__builtin_bit_cast(f16x2, h)[1];
}
#else
__device__ __forceinline__ float sub_h0(float a, uint32_t h) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(h));
  return r;
}
__device__ __forceinline__ float sub_h1(float a, uint32_t h) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r)
      : "v"(a), "v"(h));
  return r;
}
#endif
// (x0 * 2^e0, x1 * 2^e1) -> packed f16 pairs hi, lo: 6 VALU
__device__ __forceinline__ void split2h(float x0, float x1, int e0, int e1, uint32_t &h,
                                        uint32_t &l) {
  const float a = __builtin_amdgcn_ldexpf(x0, e0), b = __builtin_amdgcn_ldexpf(x1, e1);
  h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
  l = __builtin_bit_cast(uint32_t,
                         __builtin_convertvector((f32x2){sub_h0(a, h), sub_h1(b, h)}, f16x2));
}
// eight values under one scale -> the hi and lo f16x8 fragments
__device__ __forceinline__ void split8h(const float *v, int e, f16x8 &h, f16x8 &l) {
  uint32_t hh[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split2h(v[2 * i], v[2 * i + 1], e, e, hh[i], ll[i]);
  h = __builtin_bit_cast(f16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
  l = __builtin_bit_cast(f16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
}

__device__ __forceinline__ f32x16 mfma(const f16x8 &a, const f16x8 &b, const f32x16 &c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// the three kept products of a split pair, small to large
__device__ __forceinline__ f32x16 mfma3(const f16x8 &ah, const f16x8 &al, const f16x8 &bh,
                                        const f16x8 &bl, f32x16 c) {
  c = mfma(al, bh, c);
  c = mfma(ah, bl, c);
  c = mfma(ah, bh, c);
  return c;
}

}  // namespace f16x3
}  // namespace kcnn

#endif  // KCNN_CNSLMAT_F16_SPLIT_H_
