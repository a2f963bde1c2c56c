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
// error bound is normwise per group, not per product: elements far under
// their group's max keep only 2^-25 absolute.  spread() below names the
// groups where that can matter, and the kernels check (and recompute in
// fp32) the products that touch them, which restores the 1e-5 * S parity
// bar per element; the f16 MFMA runs at the bf16 rate, so this
// is half the matrix-core work of bf16x6 (x6-util.h) for fewer split VALU.
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

// exponent of a finite nonzero |x| bit pattern (subnormals by their leading
// bit)
__device__ __forceinline__ int ebits(uint32_t b) {
  return b >= 0x00800000u ? (int)(b >> 23) - 127 : (31 - (int)__builtin_clz(b)) - 149;
}
// A group is "spread" when its smallest nonzero |x| (bit pattern mn; 0: the
// group has none) lies below 2^-6 after the group's scale, i.e. more than 20
// binades under the group's max (mx).  In a group that is not spread every
// element is held to within 2^-19 of itself (the 2^-25 absolute floor of the
// lo part over an element of at least 2^-6); a spread group's small
// elements are held only to 2^-25 absolute (their lo part is an f16
// subnormal, their hi part too below 2^-14), which a dot product can show
// when they carry its sum (a large element meeting zeros in the other
// operand).  The kernels check products that touch a spread group (the GEMM's
// store, the conv forward's epilogue) and recompute the ones the check
// cannot clear in fp32.
__device__ __forceinline__ bool spread(uint32_t mx, uint32_t mn) {
  return mn != 0 && mx < NONFINITE && ebits(mn) < ebits(mx) - 20;
}
// The elements a spread group holds only to 2^-25 absolute (scaled): the
// nonzero |x| below small_bound(mx) = 2^(-3 - s), i.e. under 2^-3 after the
// scale.  A statistics block counts them per spread group (cnt).
__device__ __forceinline__ float small_bound(uint32_t mx) {
  return __builtin_amdgcn_ldexpf(1.0f, -3 - scale_exp(mx));
}
// A group's share of the GEMM store's check threshold in scaled units: each
// of its cnt such elements adds at most 2^-25 |hi| <= 2^-10 to a scaled sum,
// and a sum is kept when that part stays under 2^-19 |acc|: 2^9 per element
// (x (1 + 2^-10) for the rounding of the check itself).  cnt is 0 exactly
// when the group is not spread (a spread group's min is one of its small
// elements), so the weight is 0 then.
__device__ __forceinline__ float spread_weight(uint32_t cnt) {
  return 512.0f * (1.0f + 1.0f / 1024.0f) * (float)cnt;
}

// a - (float)f16 half of h, in one v_fma_mix_f32: fma(h, m1, a) with m1 = -1
// (exact here: h is a's f16 rounding, so the difference is an fp32 number).
// m1 comes from opaque_m1(), a -1.0f the compiler cannot fold: folded, the fma
// becomes a - h, i.e. a v_cvt_f32_f16 and a v_sub_f32 (one VALU more per
// value); opaque, the fma of an extended f16 is selected as v_fma_mix_f32 with
// the half picked by op_sel.  The instruction is then the compiler's own, so
// its hazard recognizer sees it (r04 wrote it as inline asm, which it cannot
// see through: DESIGN 3, "the f16x3 split and the hazard recognizer").
__device__ __forceinline__ float opaque_m1() {
  float v = -1.0f;
  asm volatile("" : "+s"(v));
  return v;
}
#ifdef KCNN_F16_ASM  // experiment build: r04's inline asm form, for the hazard study
__device__ __forceinline__ float sub_h0(float a, uint32_t h, float) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(h));
  return r;
}
__device__ __forceinline__ float sub_h1(float a, uint32_t h, float) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r)
      : "v"(a), "v"(h));
  return r;
}
#else
__device__ __forceinline__ float sub_h0(float a, uint32_t h, float m1) {
  return __builtin_fmaf((float)__builtin_bit_cast(f16x2, h)[0], m1, a);
}
__device__ __forceinline__ float sub_h1(float a, uint32_t h, float m1) {
  return __builtin_fmaf((float)__builtin_bit_cast(f16x2, h)[1], m1, a);
}
#endif
// (x0 * 2^e0, x1 * 2^e1) -> packed f16 pairs hi, lo: 6 VALU
__device__ __forceinline__ void split2h(float x0, float x1, int e0, int e1, uint32_t &h,
                                        uint32_t &l, float m1) {
  const float a = __builtin_amdgcn_ldexpf(x0, e0), b = __builtin_amdgcn_ldexpf(x1, e1);
  h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
  l = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                                       (f32x2){sub_h0(a, h, m1), sub_h1(b, h, m1)}, f16x2));
}
// eight values under one scale -> the hi and lo f16x8 fragments
__device__ __forceinline__ void split8h(const float *v, int e, f16x8 &h, f16x8 &l, float m1) {
  uint32_t hh[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split2h(v[2 * i], v[2 * i + 1], e, e, hh[i], ll[i], m1);
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
