// cnslmat/cnsl-conv-frame.hip -- frame-resident convolution kernels for
// layers with a small kernel volume (K = kh*kw*C <= 32, e.g. the fbank input
// layer of BASELINE c2: 8x1x3 = 24), where the contraction is too thin to
// feed MFMA from an im2col tile and the layer is HBM-bound.
//
// One workgroup walks frames (grid-stride over rows); per frame:
//   forward  Y[g][p] = sum_k W[k][g] X[c][p + off_k]
//            the frame's X map (5.3 KB) is staged in LDS, W in LDS; MFMA
//            32x32x2 with g on the accumulator rows and p on the lanes, so
//            each store writes two 128-B runs of Y; bias fused.
//   dgrad    Z[p][k] = sum_g dY[g][p] W[k][g]   (a plain GEMM: K = G, N = K)
//            with dY read straight from HBM as the MFMA A operand (lanes along
//            p: coalesced, no LDS), Z kept in LDS, then the col2im
//            dX[c][q] = sum_taps Z[q - tap][tap, c] from LDS.  No padded dY,
//            no flipped kernel, no im2col matrix (the reference's flip branch
//            moves ~30x the bytes).
//   wgrad    gW[k][g] = sum_{n,p} X[c][p + off_k] dY[g][p]; each wave owns a
//            32-wide g block, stages its dY tile through LDS (transpose), and
//            gathers the im2col operand from the LDS-resident X map.  Row
//            K of the A operand is all ones, so the bias gradient sum_p dY
//            falls out of the same MFMAs.  Per-workgroup partials are reduced
//            in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "conv-geom.h"
#include "conv-update.h"
#include "f16-split.h"
#include "momentum-step.h"
#include "pool-stats-dev.h"
#include "x6-util.h"

using namespace kcnn;

namespace {

constexpr int kFrameLdsMax = 96 * 1024;
constexpr int kBwdLdsMax = 160 * 1024;  // the fused backward: one workgroup per CU
constexpr int ZS = 33;  // padded row stride (floats) of the LDS Z / dY tiles

__host__ __device__ inline int align16(int bytes) { return (bytes + 15) & ~15; }

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

// ---------------------------------------------------------------------------
template <int NGB>
__global__ __launch_bounds__(256) void conv_fwd_frame_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ K, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os, int Kpad, int Gp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int2 *koff = reinterpret_cast<int2 *>(smem);
  float *Ws = reinterpret_cast<float *>(smem + align16(Kpad * 8));
  float *Xs = Ws + Kpad * Gp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  for (int e = tid; e < Kpad * Gp; e += 256) {
    const int k = e / Gp, gg = e - k * Gp;
    Ws[e] = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  for (int k = tid; k < Kpad; k += 256) {
    int2 v = make_int2(0, 0x7fff << 16);  // padded tap: never in bounds
    if (k < g.Kdim) {
      uint32_t c, r, kx, ky;
      g.div_khkw.divmod((uint32_t)k, c, r);
      g.div_kh.divmod(r, kx, ky);
      v = make_int2((int)c * g.HW, (int)((kx << 16) | ky));
    }
    koff[k] = v;
  }
  const int CHW = g.C * g.HW;
  const int ntile = (g.P + 31) >> 5;
  const int ksteps = Kpad >> 1;

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();
    const float *xr = X + (int64_t)n * xs;
    for (int e = tid; e < CHW; e += 256) Xs[e] = xr[e];
    __syncthreads();
    for (int pt = wave; pt < ntile; pt += 4) {
      const int p = pt * 32 + (lane & 31);
      const bool pv = p < g.P;
      uint32_t px = 0, py = 0;
      if (pv) g.div_oh.divmod((uint32_t)p, px, py);
      for (int gs = 0; gs < Gp; gs += 32 * NGB) {  // Gp: multiple of 32*NGB
        floatx16 acc[NGB];
#pragma unroll
        for (int b = 0; b < NGB; b++) acc[b] = zero16();
        for (int s = 0; s < ksteps; s++) {
          const int k = 2 * s + (lane >> 5);
          // branch-free gather: padded taps (k >= Kdim) carry zero weights,
          // invalid positions / padding read a clamped address and are
          // zeroed by a select (no exec-masked regions around the MFMAs).
          const int2 ko = koff[k];
          const int xx = (int)px + (ko.y >> 16) - g.pad_w;
          const int yy = (int)py + (ko.y & 0xffff) - g.pad_h;
          const bool ok = pv && (unsigned)xx < (unsigned)g.W &&
                          (unsigned)yy < (unsigned)g.H;
          const float xv = Xs[ok ? ko.x + xx * g.H + yy : 0];
          const float bv = ok ? xv : 0.0f;
          const float *wrow = Ws + k * Gp + gs + (lane & 31);
#pragma unroll
          for (int b = 0; b < NGB; b++)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(wrow[b * 32], bv, acc[b], 0, 0, 0);
        }
        if (pv) {
          float *orow = out + (int64_t)n * os + p;
#pragma unroll
          for (int b = 0; b < NGB; b++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
              const int gg = gs + b * 32 + mfma32_row(r, lane);
              if (gg < g.G) {
                float v = acc[b][r];
                if (bias) v = v + bias[gg];
                orow[(int64_t)gg * g.P] = v;
              }
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Forward, slab-streamed: the workgroup computes one 32-map slab of a frame's
// output (32 x P, a contiguous run of Y) into LDS, then streams it to HBM as
// linear 16-byte-per-lane stores of whole lines.
__global__ __launch_bounds__(256) void conv_fwd_slab_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ K, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os, int Kpad, int Gp, int vec_ok) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int2 *koff = reinterpret_cast<int2 *>(smem);
  float *T = reinterpret_cast<float *>(smem + align16(Kpad * 8));   // [32][P]
  float *Ws = T + ((32 * g.P + 3) & ~3);                             // [Kpad][Gp]
  float *Xs = Ws + Kpad * Gp;                                        // [C*HW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < Kpad * Gp; e += 256) {
    const int k = e / Gp, gg = e - k * Gp;
    Ws[e] = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  for (int k = tid; k < Kpad; k += 256) {
    int2 v = make_int2(0, 0x7fff << 16);
    if (k < g.Kdim) {
      uint32_t c, r, kx, ky;
      g.div_khkw.divmod((uint32_t)k, c, r);
      g.div_kh.divmod(r, kx, ky);
      v = make_int2((int)c * g.HW, (int)((kx << 16) | ky));
    }
    koff[k] = v;
  }
  const int CHW = g.C * g.HW;
  const int ntile = (g.P + 31) >> 5;
  const int ksteps = Kpad >> 1;
  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();
    const float *xr = X + (int64_t)n * xs;
    for (int e = tid; e < CHW; e += 256) Xs[e] = xr[e];
    __syncthreads();
    for (int gb = 0; gb < Gp; gb += 32) {
      for (int pt = wave; pt < ntile; pt += 4) {
        const int p = pt * 32 + (lane & 31);
        const bool pv = p < g.P;
        uint32_t px = 0, py = 0;
        if (pv) g.div_oh.divmod((uint32_t)p, px, py);
        floatx16 acc = zero16();
        const float *wcol = Ws + gb + (lane & 31);
        for (int s = 0; s < ksteps; s++) {
          const int k = 2 * s + (lane >> 5);
          const int2 ko = koff[k];
          const int xx = (int)px + (ko.y >> 16) - g.pad_w;
          const int yy = (int)py + (ko.y & 0xffff) - g.pad_h;
          const bool ok = pv && (unsigned)xx < (unsigned)g.W &&
                          (unsigned)yy < (unsigned)g.H;
          const float xv = Xs[ok ? ko.x + xx * g.H + yy : 0];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wcol[k * Gp], ok ? xv : 0.0f,
                                                     acc, 0, 0, 0);
        }
        if (pv) {
#pragma unroll
          for (int r = 0; r < 16; r++) {
            const int gl = mfma32_row(r, lane);
            const int gg = gb + gl;
            T[gl * g.P + p] = acc[r] + (bias && gg < g.G ? bias[gg] : 0.0f);
          }
        }
      }
      __syncthreads();
      const int rows = g.G - gb < 32 ? g.G - gb : 32;
      const int cnt = rows * g.P;
      float *dst = out + (int64_t)n * os + (int64_t)gb * g.P;
      if (vec_ok) {
        const float4 *src4 = reinterpret_cast<const float4 *>(T);
        float4 *dst4 = reinterpret_cast<float4 *>(dst);
        for (int e = tid; e < (cnt >> 2); e += 256) dst4[e] = src4[e];
        for (int e = (cnt & ~3) + tid; e < cnt; e += 256) dst[e] = T[e];
      } else {
        for (int e = tid; e < cnt; e += 256) dst[e] = T[e];
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// Forward with every MFMA operand in registers.  Per wave: the kernel
// W[k][g] for all (up to 4) 32-filter groups is loaded once (KS*4 VGPRs); per
// frame the im2col values of the wave's position tiles are gathered once
// from the LDS-resident map (FT*KS VGPRs) and reused by every filter group,
// so the MFMA chains run with no LDS traffic.  Each 32-filter output slab
// (a contiguous 32 x P run of Y) is staged in LDS and streamed out with
// 16-B stores; bias fused.  KS = k-steps (Kdim <= 2*KS, padded taps carry
// zero weights), FT = position tiles per wave (P <= 4*32*FT).
// PC > 0 also runs the channel-only max pool that follows the convolution
// (MaxpoolComponent with pool 1 x 1 x PC, nnet-component-nnet0.cc:869-880)
// on the LDS-resident slab: pool[n][j*P + q] = max over maps PC*j .. PC*j+PC-1
// (same start value and comparison as A.8), plus the routing mask
// mask[n][j*P + q] bit c = (Y[PC*j + c][q] == pool value) that the pool's
// Backprop (A.9) would recompute from Y.
// PC == -1: a 3-D window (ph x pw x pc, runtime; pc divides 32) pooled from
// the same slab, with a 16-bit mask (bit c*pw*ph + w*ph + h); PC == -3 the
// same for the 3 x 1 x 4 window (c5's P1) fixed at compile time, so the
// window's 12 values are read once into registers.
// X6: the products on the bf16 matrix cores (x6-util.h).  KS is then the
// number of k16 steps; A = W^T split into its three bf16 planes once per
// kernel (4 groups x KS x 3 fragments in VGPRs), with the bias as row k =
// Kdim against a constant-1 row of B, so the accumulators hold conv + bias
// and no epilogue add remains; B = the gathered im2col values, split in
// registers once per frame and tile.  Unpadded maps only (host check).
// F16 (AR = 2): the products on the f16 matrix cores (f16-split.h), three
// per k16 step.  A = W^T scaled by 2^sa (one exponent for the whole kernel,
// from the wave's max |W|: every wave holds all of W), split once per kernel
// into hi / lo planes; B = the gathered im2col values of one position scaled
// by 2^sb(p) (the position's own max |x| over its taps: lanes l and l + 32
// hold the two halves of a column), split per frame and tile.  The bias is
// not a row of the product: y = fma(acc, 2^-(sa + sb(p)), b) exactly unscales
// and adds it in one rounding.  A tile whose column max is Inf, or whose
// unscale factor would leave fp32's range, sends the wave's whole frame to
// fwd_item_fp32 (plain fp32 sums, the reference's IEEE Inf / NaN pattern);
// a kernel with Inf in W sends every frame.  The decision is per (frame,
// wave) in every epilogue, so fused and unfused runs compute the same y.
struct PoolWin {
  int ph, pw, pc, oh2, OP;
  FastDiv div_OP, div_oh2;
};

// The F16 fallback for one item (32 filters gb*32.. x the 32 positions of
// p's tile) in fp32: y = sum_k W[k][g] x_k(p), then + b[g] (the reference's
// GEMM then bias add, conv2D.cc:138-145), the accumulator layout of the MFMA.
__device__ __forceinline__ floatx16 fwd_item_fp32(
    const ConvGeom &g, const float *__restrict__ K, int ks, const float *__restrict__ bias,
    const float *Xs, const int2 *koff, int gb, int tile, int lane) {
  const int h = lane >> 5;
  const int p = min(tile * 32 + (lane & 31), g.P - 1);
  uint32_t px, py;
  g.div_oh.divmod((uint32_t)p, px, py);
  const int pb = (int)px * g.H + (int)py;
  floatx16 y;
#pragma unroll
  for (int r = 0; r < 16; r++) y[r] = 0.0f;
  for (int k = 0; k < g.Kdim; k++) {
    const float x = Xs[koff[k].x + pb];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int gg = gb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      y[r] = fmaf(gg < g.G ? K[(int64_t)k * ks + gg] : 0.0f, x, y[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int gg = gb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    y[r] = y[r] + (bias && gg < g.G ? bias[gg] : 0.0f);
  }
  return y;
}

// The F16 forward's check of an item touching a spread group (f16-split.h):
// with |W'|, |x'| <= 2^15 the elements the split holds only to 2^-25
// (scaled) add at most 2^-9 Kdim to a scaled sum, fct times that to y; an
// output with |y| >= 2^10 Kdim fct therefore carries at most 2^-19 |y| <=
// 2^-19 S of it.  True when some output of the item is below that bound:
// the caller then recomputes the whole item by fwd_item_fp32 (every lane: a
// wave-uniform decision, the same in the fused and the unfused epilogue).
__device__ __forceinline__ bool spread_reject(const floatx16 &y, float fct, const ConvGeom &g) {
  const float thr = fct * (1024.0f * (float)g.Kdim * (1.0f + 1.0f / 1024.0f));
  float mn = fabsf(y[0]);
#pragma unroll
  for (int r = 1; r < 16; r++) mn = fminf(mn, fabsf(y[r]));
  return __builtin_amdgcn_ballot_w64(!(mn >= thr)) != 0;
}

// The routing mask of a 4-way pool group, bit c = (v_c == mx): the four
// compares first, then the four selects, so each select reads a compare
// result three VALU later and needs no wait states (hipcc's order, compare /
// select pairs, pads every pair with s_nop 1).
__device__ __forceinline__ unsigned tie_mask4(float v0, float v1, float v2, float v3, float mx) {
  unsigned m, t0, t1, t2, t3;
  uint64_t c0, c1, c2, c3;
  asm("v_cmp_eq_f32_e64 %5, %9, %13\n\t"
      "v_cmp_eq_f32_e64 %6, %10, %13\n\t"
      "v_cmp_eq_f32_e64 %7, %11, %13\n\t"
      "v_cmp_eq_f32_e64 %8, %12, %13\n\t"
      "v_cndmask_b32_e64 %1, 0, 1, %5\n\t"
      "v_cndmask_b32_e64 %2, 0, 2, %6\n\t"
      "v_cndmask_b32_e64 %3, 0, 4, %7\n\t"
      "v_cndmask_b32_e64 %4, 0, 8, %8\n\t"
      "v_or3_b32 %0, %1, %2, %3\n\t"
      "v_or_b32_e32 %0, %0, %4"
      : "=v"(m), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&s"(c0), "=&s"(c1),
        "=&s"(c2), "=&s"(c3)
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "v"(mx));
  return m;
}

// The register-pooled forward's statistics outputs (pool-stats.h): the
// per-frame block rowmax [max[R], min[R], cnt[R]], the per-workgroup column
// partials (the maxima's exponent bytes, [nblk][npool]) and the column block
// colmax [max[npool], min[npool], cnt[npool]], which this kernel initialises
// for pool_colmax_kernel (the maxima) and pool_count_kernel (the minima and
// counts)
struct RpStats {
  uint32_t *rowmax = nullptr, *partials = nullptr, *colmax = nullptr;
};

// The wave's max |pooled| bits of the frame and its min (|pooled| - 1,
// wrapping: a zero never wins; f16-split.h's spread groups) into its slots of
// rslot (LDS: [2][4] maxima, then [2][4] minima; the frame's four slots are
// combined after the next barrier)
__device__ __forceinline__ void frame_row_max(uint32_t *rslot, uint32_t v, uint32_t u, int lane) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    v = max(v, (uint32_t)__shfl_xor((int)v, o));
    u = min(u, (uint32_t)__shfl_xor((int)u, o));
  }
  if (lane == 0) {
    rslot[0] = v;
    rslot[8] = u;
  }
}

// The pooled output's column statistics (pool-stats-dev.h), as kernels of
// their own: the forward launches them unless its caller leaves them to the
// consumer (PoolColDeferred)
__global__ __launch_bounds__(256) void pool_colmax_kernel(const uint8_t *__restrict__ pcol,
                                                           int nblk, int npool,
                                                           uint32_t *__restrict__ colmax) {
  pool_colmax_block(pcol, nblk, npool, colmax, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void pool_count_kernel(const float *__restrict__ P, int ps,
                                                         int R, int npool, int vec,
                                                         uint32_t *__restrict__ rowblk,
                                                         uint32_t *colblk) {
  __shared__ PoolCountSmem sm;
  pool_count_block(P, ps, R, npool, vec, rowblk, colblk, blockIdx.x, gridDim.x, sm);
}

// RP: the register-pooled form only (out == nullptr, PC 2 or 4, G = 128 and
// every wave with FT position tiles: c2), without the generic item loop and
// the LDS epilogue, whose uniform conditions otherwise overflow the SGPRs.
template <int KS, int FT, int PC, int AR, bool RP = false>
__global__ __launch_bounds__(256, 2) void conv_fwd_regs_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ K, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os, int vec_ok, int dbg,
    float *__restrict__ pool, int ps, unsigned char *__restrict__ mask, int ms,
    PoolWin pw3, RpStats rps) {
  constexpr bool X6 = AR == 1, F16 = AR == 2, SPL = AR != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *T = reinterpret_cast<float *>(smem);                 // [32][P]
  float *Bs = T + ((32 * g.P + 3) & ~3);                      // [128] bias
  float *Bz = Bs + 128;                                       // [32] -0 (F16 fp32 items)
  int2 *koff = reinterpret_cast<int2 *>(Bs + 160);             // [2*KS] taps
  constexpr int NKT = SPL ? 16 * KS : 2 * KS;                   // tap entries (<= 32)
  float *Xs = reinterpret_cast<float *>(koff + NKT);            // [C*HW]
  uint32_t *rslot = reinterpret_cast<uint32_t *>(Xs + g.C * g.HW);  // [2][2][4] RP row max / min
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31, h = lane >> 5;
  const int NG = (g.G + 31) >> 5;  // <= 4 (host check)
  if (tid < 128) Bs[tid] = (bias && tid < g.G) ? bias[tid] : 0.0f;
  if (tid < 32) Bz[tid] = -0.0f;
  // A operand: W[k = 2s + h][gb*32 + l]
  float wreg[X6 ? 1 : 4][X6 ? 1 : KS];
  // X6: W^T[gb*32 + l][k = 16s + 8h + e] (e < 8), the bias at k = Kdim
  x6::bf16x8 w6[X6 ? 4 : 1][X6 ? KS : 1][3];
  // F16: W^T[gb*32 + l][k = 16s + 8h + e] * 2^sa, hi and lo planes
  f16x3::f16x8 wh[F16 ? 4 : 1][F16 ? KS : 1], wl[F16 ? 4 : 1][F16 ? KS : 1];
  int sa = 0;
  bool wslow = false;  // Inf in W: every item in fp32
  bool wspread = false;  // W is a spread group (f16-split.h): every item checked
  const float m1 = F16 ? f16x3::opaque_m1() : 0.0f;  // the split's -1 (f16-split.h)
  if constexpr (F16) {
    float wv[4][KS][8];
    float m = 0.0f;
    uint32_t mn = 0xffffffffu;  // min 2|w| - 2 (wrapping: a zero never wins)
#pragma unroll
    for (int gb = 0; gb < 4; gb++)
#pragma unroll
      for (int s = 0; s < KS; s++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const int k = 16 * s + 8 * h + e, gg = gb * 32 + l;
          wv[gb][s][e] = gg < g.G && k < g.Kdim ? K[(int64_t)k * ks + gg] : 0.0f;
          m = fmaxf(m, fabsf(wv[gb][s][e]));  // NaN ignored: it propagates by itself
          mn = min(mn, (__float_as_uint(wv[gb][s][e]) << 1) - 2u);
        }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      m = fmaxf(m, __shfl_xor(m, o));
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
    }
    const uint32_t mwb = __builtin_amdgcn_readfirstlane(__float_as_uint(m));
    wspread = f16x3::spread(mwb, (__builtin_amdgcn_readfirstlane(mn) >> 1) + 1u);
    const int s0 = f16x3::scale_exp(mwb);
    wslow = s0 == f16x3::SKIP;
    sa = wslow ? 0 : s0;
#pragma unroll
    for (int gb = 0; gb < 4; gb++)
#pragma unroll
      for (int s = 0; s < KS; s++) f16x3::split8h(wv[gb][s], sa, wh[gb][s], wl[gb][s], m1);
  }
  if constexpr (X6) {
#pragma unroll
    for (int gb = 0; gb < 4; gb++)
#pragma unroll
      for (int s = 0; s < KS; s++) {
        const int gg = gb * 32 + l;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const int k = 16 * s + 8 * h + e;
          v[e] = gg >= g.G ? 0.0f
                 : k < g.Kdim ? K[(int64_t)k * ks + gg]
                 : (k == g.Kdim && bias) ? bias[gg] : 0.0f;
        }
        x6::split8(v, w6[gb][s][0], w6[gb][s][1], w6[gb][s][2]);
      }
  } else {
#pragma unroll
    for (int gb = 0; gb < 4; gb++)
#pragma unroll
      for (int s = 0; s < KS; s++) {
        const int k = 2 * s + h, gg = gb * 32 + l;
        wreg[gb][s] = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
      }
  }
  // tap k -> (channel offset, kx << 16 | ky); padded taps never in bounds.
  // X6 (unpadded maps): tap k -> its map offset c*HW + kx*H + ky in .x
  if (tid < NKT) {
    int2 v = make_int2(0, 0x3fff << 16);
    if (tid < g.Kdim) {
      uint32_t c, r, qx, qy;
      g.div_khkw.divmod((uint32_t)tid, c, r);
      g.div_kh.divmod(r, qx, qy);
      v = SPL ? make_int2((int)c * g.HW + (int)qx * g.H + (int)qy, 0)
             : make_int2((int)c * g.HW, (int)((qx << 16) | qy));
    }
    koff[tid] = v;
  }
  const int CHW = g.C * g.HW;
  const int ntile = (g.P + 31) >> 5;
  // X6: every aligned group of 8 taps one run of consecutive map offsets
  // (c2's 8 x 1 kernel: taps c*8 + ky at c*HW + ky)?  Then a group's 8 values
  // are read at one offset + e, without the per-tap table reads
  bool run8 = false;
  if constexpr (SPL) {
    run8 = !(dbg & 64);
    for (int k = 0; k + 1 < g.Kdim && run8; k++) {
      if ((k + 1) % 8 == 0) continue;
      uint32_t c0, r0, x0, y0, c1, r1, x1, y1;
      g.div_khkw.divmod((uint32_t)k, c0, r0);
      g.div_kh.divmod(r0, x0, y0);
      g.div_khkw.divmod((uint32_t)(k + 1), c1, r1);
      g.div_kh.divmod(r1, x1, y1);
      const int o0 = (int)c0 * g.HW + (int)x0 * g.H + (int)y0;
      const int o1 = (int)c1 * g.HW + (int)x1 * g.H + (int)y1;
      run8 = o1 == o0 + 1;
    }
  }
#ifdef KCNN_PHASE_TIMING  // per-phase s_memtime totals of block 0 (dbg & 16)
  long long tm[6] = {0, 0, 0, 0, 0, 0};
  long long tprev = clock64();
#define KCNN_TMARK(i) if (dbg & 16) { const long long tn = clock64(); tm[i] += tn - tprev; tprev = tn; }
#else
#define KCNN_TMARK(i)
#endif
  // RP: the pooled output's statistics for the FC GEMM that reads it
  // (cu-gemm-f16x3.hip's operand scales): max |value| bits per frame (prow,
  // atomic max) and per pooled column over this workgroup's frames, kept in
  // the LDS slab T (unused by this form; npool = 32 * P words) by ds_max and
  // stored to the workgroup's row of the partials pcol at the end
  uint32_t *Tcol = reinterpret_cast<uint32_t *>(T);
  uint32_t *const prow = rps.rowmax, *const pcol = rps.partials;
  if constexpr (RP) {
    for (int e = tid; e < g.G / PC * g.P; e += 256) Tcol[e] = 0;
    // the column block for the kernels after this grid: pool_colmax_kernel's
    // atomic maxima start from 0, pool_count_kernel's minima from 0xffffffff
    // and its counts from 0
    const int c = blockIdx.x * 256 + tid;
    if (rps.colmax && c < g.G / PC * g.P) {
      rps.colmax[c] = 0;
      rps.colmax[g.G / PC * g.P + c] = 0xffffffffu;
      rps.colmax[2 * g.G / PC * g.P + c] = 0;
    }
  }
  // the next frame's map is prefetched into registers while this one runs
  constexpr int XV = 8;  // CHW <= 2048 (host check)
  float xv[XV];
#pragma unroll
  for (int i = 0; i < XV; i++)
    if (blockIdx.x < (unsigned)g.R && tid + 256 * i < CHW)
      xv[i] = X[(int64_t)blockIdx.x * xs + tid + 256 * i];
  int it = 0;  // this workgroup's frame count
  for (int n = blockIdx.x; n < g.R; n += gridDim.x, ++it) {
    // lane ids made opaque per frame: the frame-invariant LDS / global
    // addresses are recomputed instead of hoisted out of the loop (hoisted,
    // they overflow the register file)
    int tid_f = tid;
    asm volatile("" : "+v"(tid_f));
    int wave_q = wave;  // likewise the wave id (held, the wave-derived item
    asm volatile("" : "+s"(wave_q));  // constants overflow the SGPRs)
    const int lane_f = tid_f & 63, l_f = lane_f & 31, h_f = lane_f >> 5;
    __syncthreads();  // previous frame's Xs / T reads done
    if constexpr (RP) {  // the previous frame's row maximum from its four wave slots
      if (it > 0 && tid_f == 0 && prow) {
        const uint32_t *q = rslot + ((it - 1) & 1) * 4;
        prow[n - (int)gridDim.x] = max(max(q[0], q[1]), max(q[2], q[3]));
        prow[g.R + n - (int)gridDim.x] = min(min(q[8], q[9]), min(q[10], q[11])) + 1u;
      }
    }
    KCNN_TMARK(5)
#pragma unroll
    for (int i = 0; i < XV; i++)
      if (tid_f + 256 * i < CHW) Xs[tid_f + 256 * i] = xv[i];
    if (n + (int)gridDim.x < g.R) {
#pragma unroll
      for (int i = 0; i < XV; i++)
        if (tid_f + 256 * i < CHW)
          xv[i] = X[(int64_t)(n + gridDim.x) * xs + tid_f + 256 * i];
    }
    __syncthreads();
    KCNN_TMARK(0)
    float bx[SPL ? 1 : FT][SPL ? 1 : KS];
    x6::bf16x8 bx6[X6 ? FT : 1][X6 ? KS : 1][3];
    f16x3::f16x8 bxh[F16 ? FT : 1][F16 ? KS : 1], bxl[F16 ? FT : 1][F16 ? KS : 1];
    float ft[F16 ? FT : 1];  // F16: the unscale factor 2^-(sa + sb(p)) of tile t
    bool slow = false;       // F16: this wave_q's items of the frame in fp32
    int tsp = 0;             // F16: bit t, tile t has a spread position column
#pragma unroll
    for (int t = 0; t < FT; t++) {
      if constexpr (F16) {
        // B[k = 16s + 8h + e][p] = x_k(p) for k < Kdim, 0 past it
        if ((wave_q + 4 * t) * 32 >= g.P) continue;  // wave_q-uniform: no tile
        const int p = min((wave_q + 4 * t) * 32 + l_f, g.P - 1);
        uint32_t px, py;
        g.div_oh.divmod((uint32_t)p, px, py);
        const int pb = (int)px * g.H + (int)py;
        float v[KS][8];
        float m = 0.0f;
        uint32_t mn = 0xffffffffu;  // min 2|x| - 2 (wrapping: a zero never wins)
#pragma unroll
        for (int s = 0; s < KS; s++) {
          const int k0 = 16 * s + 8 * h_f;
          if (run8) {  // uniform
            const float *xr = Xs + koff[k0].x + pb;
#pragma unroll
            for (int e = 0; e < 8; e++) v[s][e] = xr[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; e++) v[s][e] = Xs[koff[k0 + e].x + pb];
          }
#pragma unroll
          for (int e = 0; e < 8; e++) {
            v[s][e] = k0 + e < g.Kdim ? v[s][e] : 0.0f;
            m = fmaxf(m, fabsf(v[s][e]));
#ifdef KCNN_EXPERIMENTS  // A/B: dbg & 2048 drops the position columns' min
            if (!(dbg & 2048))
#endif
            mn = min(mn, (__float_as_uint(v[s][e]) << 1) - 2u);
          }
        }
        // the column's other half: lane l ^ 32, through ds_bpermute.  (With
        // v_permlane32_swap here, one accumulator register of 16 lanes of a
        // wave's last item came out wrong in about one call in four of a
        // 601-frame forward, G = 96, Kdim 12; experiments/diag_det2.py.)
#ifdef KCNN_FWD_PERMLANE  // experiment: the swap variant of the hazard study
        {
          auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m),
                                                     false, false);
#ifdef KCNN_FWD_PERMLANE_NOP  // two wait states between the swap and its readers
          uint32_t s0 = sw[0], s1 = sw[1];
          asm volatile("s_nop 1" : "+v"(s0), "+v"(s1));
          sw[0] = s0;
          sw[1] = s1;
#endif
          m = fmaxf(m, __uint_as_float(h_f ? sw[1] : sw[0]));
        }
#else
        m = fmaxf(m, __shfl_xor(m, 32));
#endif
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, 32));
        const uint32_t mb = __float_as_uint(m);
        // a spread position column (f16-split.h): the tile's items are checked
        if (__builtin_amdgcn_ballot_w64(f16x3::spread(mb, (mn >> 1) + 1u)) != 0) tsp |= 1 << t;
        int sb = mb == 0 ? -sa : f16x3::scale_exp(mb);
        const int E = -(sa + sb);
        const bool bad = sb == f16x3::SKIP || E < -149 || E > 127;
        if (bad) sb = 0;
        ft[t] = __builtin_amdgcn_ldexpf(1.0f, bad ? 0 : E);
        if (__builtin_amdgcn_ballot_w64(bad) != 0) slow = true;
#pragma unroll
        for (int s = 0; s < KS; s++) f16x3::split8h(v[s], sb, bxh[t][s], bxl[t][s], m1);
        continue;
      }
      if constexpr (X6) {
        // B[k = 16s + 8h + e][p]: the map value of tap k at p (one add: the
        // maps are unpadded, so every tap of a valid position is inside),
        // 1 at k = Kdim (the bias row), 0 past it; positions past P read a
        // clamped position and are never stored
        if ((wave_q + 4 * t) * 32 >= g.P) continue;  // wave_q-uniform: no tile
        const int p = min((wave_q + 4 * t) * 32 + l_f, g.P - 1);
        uint32_t px, py;
        g.div_oh.divmod((uint32_t)p, px, py);
        const int pb = (int)px * g.H + (int)py;
#pragma unroll
        for (int s = 0; s < KS; s++) {
          float v[8];
          const int k0 = 16 * s + 8 * h_f;
          if (run8) {  // uniform
            const float *xr = Xs + koff[k0].x + pb;
#pragma unroll
            for (int e = 0; e < 8; e++) {
              const float xval = xr[e];
              v[e] = k0 + e < g.Kdim ? xval : (k0 + e == g.Kdim ? 1.0f : 0.0f);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; e++) {
              const int k = k0 + e;
              const float xval = Xs[koff[k].x + pb];
              v[e] = k < g.Kdim ? xval : (k == g.Kdim ? 1.0f : 0.0f);
            }
          }
          x6::split8(v, bx6[t][s][0], bx6[t][s][1], bx6[t][s][2]);
        }
        continue;
      }
      const int p = (wave_q + 4 * t) * 32 + l_f;
      const bool pv = p < g.P;
      uint32_t px = 0, py = 0;
      g.div_oh.divmod((uint32_t)(pv ? p : 0), px, py);
#pragma unroll
      for (int s = 0; s < KS; s++) {
        const int2 ko = koff[2 * s + h_f];
        const int xx = (int)px + (ko.y >> 16) - g.pad_w;
        const int yy = (int)py + (ko.y & 0xffff) - g.pad_h;
        const bool ok = pv && (unsigned)xx < (unsigned)g.W && (unsigned)yy < (unsigned)g.H;
        const float v = Xs[ok ? ko.x + xx * g.H + yy : 0];
        bx[t][s] = ok ? v : 0.0f;
      }
    }
    if constexpr (F16) slow = slow || wslow;
    KCNN_TMARK(1)
    if constexpr (SPL && (PC == 2 || PC == 4)) {
      if (out == nullptr) {  // uniform: pooled straight from the registers
        // items (gb, t) in order; the MFMA chain of item i is issued before
        // the pooling of item i - 1, so that VALU work runs under the chain
        constexpr int NI = 4 * FT;
        const int npool = g.G / PC * g.P;  // pooled values of one frame row
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(pool + (int64_t)n * ps), (short)0, npool * 4, 0x00020000);
        const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(mask + (int64_t)n * ms), (short)0, npool, 0x00020000);
        auto valid = [&](int i) { return i / FT < NG && wave_q + 4 * (i % FT) < ntile; };
        // the pooling of one item's accumulators (F16: y = acc * 2^-(sa +
        // sb(p)) + b first, in one rounding; fp32 items: acc * 1 + -0, i.e.
        // acc itself)
        uint32_t redo = 0;    // F16: items (bit gb * FT + t) recomputed in fp32
        uint32_t rowrun = 0;  // RP: max |pooled| bits of this lane in the frame
        uint32_t rowmn = 0xffffffffu;  // RP: min (|pooled| - 1) of this lane in the frame
        // (chk: std::true_type in the frames that touch a spread group, which
        // run their own copy of the item sequence, so the common one stays
        // free of the check's branches)
        auto pool_item = [&](floatx16 &acc, int gb, int t, bool sl, auto chk) {
          const int p = (wave_q + 4 * t) * 32 + l_f;
          // accumulator r = 4k + i of lane (l, h) is filter 8k + 4h + i at
          // position p: a pool group is PC consecutive registers (the
          // compares and order of the LDS epilogue, so the same bits).  Its
          // pooled row is U + h * 4 / PC with U uniform: buffer stores take
          // the lane part as voffset and U as soffset (no vector address
          // arithmetic).  Positions past P, and rows past G (G not a
          // multiple of 32), get a voffset past the descriptors' ranges and
          // are dropped (the range check covers voffset, not soffset).
          const unsigned vo = p < g.P ? (unsigned)(h_f * (4 / PC) * g.P + p) : 0x3ffffff0u;
          // the rows' soffsets U * P recomputed per item (SALU) instead of
          // hoisted out of the frame loop (held, they spill SGPRs)
          int Pq = g.P;
          asm volatile("" : "+s"(Pq));
          const float fct = F16 && !sl ? ft[F16 ? t : 0] : 1.0f;
          // the bias rows' offset made opaque per item: the loads are not
          // hoisted or shared across items (held for all four filter groups
          // they would take 64 VGPRs and spill)
          int boff = (sl ? 128 : gb * 32) + 4 * h_f;  // Bz = Bs + 128
          asm volatile("" : "+v"(boff));
          const float *bb = Bs + boff;
          if constexpr (F16) {
            // y = acc * 2^-(sa + sb(p)) + b in one rounding (fp32 items:
            // acc * 1 + -0, i.e. acc itself)
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const float4 b4 = *reinterpret_cast<const float4 *>(bb + 8 * k);
              acc[4 * k + 0] = fmaf(acc[4 * k + 0], fct, b4.x);
              acc[4 * k + 1] = fmaf(acc[4 * k + 1], fct, b4.y);
              acc[4 * k + 2] = fmaf(acc[4 * k + 2], fct, b4.z);
              acc[4 * k + 3] = fmaf(acc[4 * k + 3], fct, b4.w);
            }
            if constexpr (decltype(chk)::value) {
              if (!sl && (wspread || (tsp >> t) & 1) && spread_reject(acc, fct, g)) {
                redo |= 1u << (gb * FT + t);  // uniform, rare: pooled after the sequence
                return;
              }
            }
          }
          // The pool value by IEEE max (v_max3: NaN skipped like the
          // reference's `val < x` test, ties between equal nonzero values
          // are the same bits).  The one case max and the reference's
          // first-wins scan differ is a +0 / -0 tie: any group whose max is
          // zero is rescanned the reference's way (uniform branch, rare).
          constexpr int NGP = 16 / PC;
          float mx[NGP];
          unsigned msk[NGP];
          bool anyz = false;
#pragma unroll
          for (int j = 0; j < NGP; j++) {
            float m = fmaxf(-1e20f, acc[j * PC]);
#pragma unroll
            for (int c = 1; c < PC; c++) m = fmaxf(m, acc[j * PC + c]);
            mx[j] = m;
            anyz |= m == 0.0f;
          }
          if (__builtin_expect(anyz, 0)) {
#pragma unroll
            for (int j = 0; j < NGP; j++) {
              if (mx[j] == 0.0f) {
                float m = -1e20f;
#pragma unroll
                for (int c = 0; c < PC; c++)
                  if (m < acc[j * PC + c]) m = acc[j * PC + c];
                mx[j] = m;
              }
            }
          }
          if constexpr (RP) {
            // lanes past P hold position P - 1's values: their max lands there
            const int pc = min(p, g.P - 1) + h_f * (4 / PC) * Pq;
#pragma unroll
            for (int j = 0; j < NGP; j++) {
              const uint32_t a = __float_as_uint(mx[j]) & 0x7fffffffu;  // never NaN
              const int r0 = j * PC;
              const int U = (gb * 32 + (r0 & 3) + 8 * (r0 >> 2)) / PC;
              __hip_atomic_fetch_max(Tcol + U * Pq + pc, a, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              rowrun = max(rowrun, a);
              const uint32_t u = a - 1u;  // wraps for 0: never the min
#ifdef KCNN_EXPERIMENTS  // A/B: dbg & 4096 drops the row min
              if (!(dbg & 4096))
#endif
              rowmn = min(rowmn, u);
            }
            // (pinned per item: left free, the scheduler spreads the items'
            // statistics and holds 34 more VGPRs)
            asm volatile("" : "+v"(rowrun), "+v"(rowmn));
          }
#pragma unroll
          for (int j = 0; j < NGP; j++) {
            if constexpr (PC == 4) {
              msk[j] = tie_mask4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3], mx[j]);
            } else {
              unsigned m = 0;
#pragma unroll
              for (int c = 0; c < PC; c++) m |= (acc[j * PC + c] == mx[j] ? 1u : 0u) << c;
              msk[j] = m;
            }
          }
#pragma unroll
          for (int j = 0; j < NGP; j++) {
            const int r0 = j * PC;
            const int U = (gb * 32 + (r0 & 3) + 8 * (r0 >> 2)) / PC;
            const unsigned vv =
                g.G % 32 == 0 || U + h_f * (4 / PC) < g.G / PC ? vo : 0x3ffffff0u;
#ifdef KCNN_EXPERIMENTS  // store A/B: dbg & 256 drops the pooled values, & 512 the masks
            if (!(dbg & 256))
#endif
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mx[j]), prs, vv * 4u,
                                                  (unsigned)(U * Pq) * 4u, 0);
#ifdef KCNN_EXPERIMENTS
            if (!(dbg & 512))
#endif
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)msk[j], mrs, vv,
                                                 (unsigned)(U * Pq), 0);
          }
        };
        // the items in fp32 (fwd_item_fp32, then pooled like any other):
        // every valid item of a slow frame (Inf, range), or the items a
        // spread check rejected; one code copy for both
        auto fp32_items = [&]() {
#pragma unroll 1
          while (redo) {  // uniform
            const int i = __builtin_ctz(redo);
            redo &= redo - 1;
            const int gb = i / FT, t = i % FT;
            floatx16 a = fwd_item_fp32(g, K, ks, bias, Xs, koff, gb, wave_q + 4 * t, lane_f);
            pool_item(a, gb, t, true, std::false_type{});
          }
        };
        if constexpr (F16) {
          if (slow) {  // uniform: the frame's items in fp32 (rare: Inf, range)
#pragma unroll 1
            for (int i = 0; i < NI; i++)
              if (RP || valid(i)) redo |= 1u << i;
            fp32_items();
            if constexpr (RP) frame_row_max(rslot + (it & 1) * 4 + wave_q, rowrun, rowmn, lane_f);
            KCNN_TMARK(2)
            continue;  // next frame
          }
        }
        auto chain = [&](int gb, int t) {
          floatx16 a = zero16();
#pragma unroll
          for (int s = 0; s < KS; s++) {
            if constexpr (F16)
              a = f16x3::mfma3(wh[gb][s], wl[gb][s], bxh[t][s], bxl[t][s], a);
            else
              a = x6::mfma6(w6[gb][s], bx6[t][s], a);
          }
          return a;
        };
        auto sequence = [&](auto chk) {
          if (RP || (NG == 4 && wave_q + 4 * (FT - 1) < ntile)) {
            // every item valid (c2: G = 128, P = 363): one straight-line
            // sequence, the MFMA chain of item i beside the pooling of i - 1
            floatx16 prev = chain(0, 0);
#pragma unroll
            for (int i = 1; i <= NI; i++) {
              floatx16 cur;
              if (i < NI) cur = chain(i / FT, i % FT);
              pool_item(prev, (i - 1) / FT, (i - 1) % FT, false, chk);
              if (i < NI) prev = cur;
            }
          } else if constexpr (!RP) {
#pragma unroll
            for (int i = 0; i < NI; i++) {
              if (!valid(i)) continue;  // uniform
              floatx16 a = chain(i / FT, i % FT);
              pool_item(a, i / FT, i % FT, false, chk);
            }
          }
        };
#ifdef KCNN_EXPERIMENTS  // A/B: dbg & 8192 never takes the checked sequence
        if (dbg & 8192) tsp = 0;
#endif
        if (F16 && (wspread || tsp != 0)) sequence(std::true_type{});  // uniform, rare
        else sequence(std::false_type{});
        if constexpr (F16) fp32_items();  // the items a spread check rejected (rare)
        if constexpr (RP) frame_row_max(rslot + (it & 1) * 4 + wave_q, rowrun, rowmn, lane_f);
        KCNN_TMARK(2)
        continue;  // next frame
      }
    }
    if constexpr (RP) continue;  // (never reached: host check)
#pragma unroll
    for (int gb = 0; gb < 4; gb++) {
      if (gb >= NG) break;
      float bsv[16];  // this lane_f's 16 accumulator rows' bias, read ahead (X6: 0, in acc)
#pragma unroll
      for (int r = 0; r < 16; r++) bsv[r] = X6 ? 0.0f : Bs[gb * 32 + mfma32_row(r, lane_f)];
#pragma unroll
      for (int t = 0; t < FT; t++) {
        const int pt = wave_q + 4 * t;
        if (pt >= ntile) continue;  // wave_q-uniform
        floatx16 acc = zero16();
        if constexpr (F16) {
          bool fp = slow;  // uniform
          if (!fp) {
#pragma unroll
            for (int s = 0; s < KS; s++)
              acc = f16x3::mfma3(wh[gb][s], wl[gb][s], bxh[t][s], bxl[t][s], acc);
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = fmaf(acc[r], ft[t], bsv[r]);
            fp = (wspread || (tsp >> t) & 1) && spread_reject(acc, ft[t], g);  // rare
          }
          if (fp) acc = fwd_item_fp32(g, K, ks, bias, Xs, koff, gb, pt, lane_f);
        } else if constexpr (X6) {
#pragma unroll
          for (int s = 0; s < KS; s++) acc = x6::mfma6(w6[gb][s], bx6[t][s], acc);
        } else {
#pragma unroll
          for (int s = 0; s < KS; s++)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wreg[gb][s], bx[t][s], acc, 0, 0, 0);
        }
        const int p = pt * 32 + l_f;
        if constexpr (PC == 2 || PC == 4) {
          if (out == nullptr) {  // uniform: pooled straight from the registers
            // accumulator r = 4k + i of lane (l, h) is filter 8k + 4h + i of
            // the slab at position p: a pool group of PC filters is PC
            // consecutive registers of one lane.  Same adds, compares and
            // order as the LDS epilogue below, so the same bits.
            if (p < g.P) {
              float *pd = pool + (int64_t)n * ps + p;
              unsigned char *md = mask + (int64_t)n * ms + p;
#pragma unroll
              for (int r0 = 0; r0 < 16; r0 += PC) {
                const int row = gb * 32 + mfma32_row(r0, lane_f);
                if (row >= g.G) continue;
                float mx = -1e20f, v[PC];
#pragma unroll
                for (int c = 0; c < PC; c++) {
                  v[c] = SPL ? acc[r0 + c] : acc[r0 + c] + bsv[r0 + c];
                  if (mx < v[c]) mx = v[c];
                }
                unsigned m = 0;
#pragma unroll
                for (int c = 0; c < PC; c++) m |= (v[c] == mx ? 1u : 0u) << c;
                const int64_t off = (int64_t)(row / PC) * g.P;
                pd[off] = mx;
                md[off] = (unsigned char)m;
              }
            }
            continue;
          }
        }
        if (p < g.P) {
#pragma unroll
          for (int r = 0; r < 16; r++)
            T[mfma32_row(r, lane_f) * g.P + p] = SPL ? acc[r] : acc[r] + bsv[r];
        }
      }
      KCNN_TMARK(2)
      if constexpr (PC == 2 || PC == 4) {
        if (out == nullptr) continue;  // nothing staged in T
      }
      __syncthreads();
      KCNN_TMARK(3)
      const int rows = g.G - gb * 32 < 32 ? g.G - gb * 32 : 32;
      const int cnt = rows * g.P;
      // out == nullptr (pooled variants): the caller needs only the pooled
      // output and the routing mask, Y itself is never stored
      float *dst = out ? out + (int64_t)n * os + (int64_t)gb * 32 * g.P : nullptr;
      if (dst == nullptr) {
      } else if (vec_ok & 2) {  // streaming stores: Y is not re-read here
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 *src4 = reinterpret_cast<const f4 *>(T);
        f4 *dst4 = reinterpret_cast<f4 *>(dst);
        for (int e = tid_f; e < (cnt >> 2); e += 256)
          __builtin_nontemporal_store(src4[e], dst4 + e);
        for (int e = (cnt & ~3) + tid_f; e < cnt; e += 256) dst[e] = T[e];
      } else if (vec_ok) {
        const float4 *src4 = reinterpret_cast<const float4 *>(T);
        float4 *dst4 = reinterpret_cast<float4 *>(dst);
        for (int e = tid_f; e < (cnt >> 2); e += 256) dst4[e] = src4[e];
        for (int e = (cnt & ~3) + tid_f; e < cnt; e += 256) dst[e] = T[e];
      } else {
        for (int e = tid_f; e < cnt; e += 256) dst[e] = T[e];
      }
      if constexpr (PC < 0) {  // 3-D window; rows % pc == 0 (host check)
        constexpr int CPH = PC == -3 ? 3 : 0, CPW = PC == -3 ? 1 : 0, CPC = PC == -3 ? 4 : 0;
        const int wph = CPH ? CPH : pw3.ph, wpw = CPW ? CPW : pw3.pw, wpc = CPC ? CPC : pw3.pc;
        const int cnt_p = rows / wpc * pw3.OP;
        const int64_t pb = (int64_t)(gb * 32 / wpc) * pw3.OP;
        float *pd = pool + (int64_t)n * ps + pb;
        unsigned short *md = reinterpret_cast<unsigned short *>(mask) + (int64_t)n * ms + pb;
        for (int e = tid_f; e < cnt_p; e += 256) {
          uint32_t j, q, wi, hi;
          pw3.div_OP.divmod((uint32_t)e, j, q);
          pw3.div_oh2.divmod(q, wi, hi);
          const float *t = T + (int)j * wpc * g.P + (int)wi * wpw * g.oh + (int)hi * wph;
          float val = -1e20f;  // A.8: c, then w, then h
          unsigned m = 0;
          if constexpr (CPH > 0) {
            float v[CPC * CPW * CPH];
#pragma unroll
            for (int c = 0; c < CPC; c++)
#pragma unroll
              for (int w = 0; w < CPW; w++)
#pragma unroll
                for (int h = 0; h < CPH; h++)
                  v[(c * CPW + w) * CPH + h] = t[c * g.P + w * g.oh + h];
#pragma unroll
            for (int b = 0; b < CPC * CPW * CPH; b++)
              if (val < v[b]) val = v[b];
#pragma unroll
            for (int b = 0; b < CPC * CPW * CPH; b++) m |= (v[b] == val ? 1u : 0u) << b;
          } else {
            for (int c = 0; c < wpc; c++)
              for (int w = 0; w < wpw; w++)
                for (int h = 0; h < wph; h++) {
                  const float v = t[c * g.P + w * g.oh + h];
                  if (val < v) val = v;
                }
            int bit = 0;
            for (int c = 0; c < wpc; c++)
              for (int w = 0; w < wpw; w++)
                for (int h = 0; h < wph; h++, bit++)
                  m |= (t[c * g.P + w * g.oh + h] == val ? 1u : 0u) << bit;
          }
          pd[e] = val;
          md[e] = (unsigned short)m;
        }
      }
      if constexpr (PC > 0) {  // rows % PC == 0 (host check)
        const int cnt_p = rows / PC * g.P;
        const int64_t pb = (int64_t)(gb * 32 / PC) * g.P;
        float *pd = pool + (int64_t)n * ps + pb;
        unsigned char *md = mask + (int64_t)n * ms + pb;
        for (int e = tid_f; e < cnt_p; e += 256) {
          uint32_t j, q;
          g.div_P.divmod((uint32_t)e, j, q);
          const float *t = T + (int)j * PC * g.P + (int)q;
          float v[PC];
#pragma unroll
          for (int c = 0; c < PC; c++) v[c] = t[c * g.P];
          float val = -1e20f;
#pragma unroll
          for (int c = 0; c < PC; c++)
            if (val < v[c]) val = v[c];
          unsigned m = 0;
#pragma unroll
          for (int c = 0; c < PC; c++) m |= (v[c] == val ? 1u : 0u) << c;
          pd[e] = val;
          md[e] = (unsigned char)m;
        }
      }
      KCNN_TMARK(4)
      __syncthreads();
      KCNN_TMARK(5)
    }
  }
  if constexpr (RP) {
    // this workgroup's row of the column partials, and its last frame's row
    // maximum
    __syncthreads();
    if (it > 0 && tid == 0 && prow) {
      const uint32_t *q = rslot + ((it - 1) & 1) * 4;
      const int fr = blockIdx.x + (it - 1) * (int)gridDim.x;
      prow[fr] = max(max(q[0], q[1]), max(q[2], q[3]));
      prow[g.R + fr] = min(min(q[8], q[9]), min(q[10], q[11])) + 1u;
    }
    if (pcol) {  // exponent bytes (pool_colmax_kernel), four per dword store
      const int npool = g.G / PC * g.P;
      uint8_t *dst = reinterpret_cast<uint8_t *>(pcol) + (int64_t)blockIdx.x * npool;
      if (npool % 4 == 0) {
        for (int e = 4 * tid; e < npool; e += 1024)
          *reinterpret_cast<uint32_t *>(dst + e) =
              (Tcol[e] >> 23) | (Tcol[e + 1] >> 23) << 8 | (Tcol[e + 2] >> 23) << 16 |
              (Tcol[e + 3] >> 23) << 24;
      } else {
        for (int e = tid; e < npool; e += 256) dst[e] = (uint8_t)(Tcol[e] >> 23);
      }
    }
  }
#ifdef KCNN_PHASE_TIMING
  if ((dbg & 16) && blockIdx.x == 0 && lane == 0)
    printf("fwd wave %d: xload %lld gather %lld mfma %lld bar1 %lld store %lld bar2 %lld\n",
           wave, tm[0], tm[1], tm[2], tm[3], tm[4], tm[5]);
#endif
#undef KCNN_TMARK
}

// ---------------------------------------------------------------------------
// Fused backward: data AND weight gradient from a single pass over dY.
// dY of one frame is streamed in 32-map slabs (32 x P floats, contiguous and
// 16-B aligned in HBM): linear dwordx4 loads, prefetched into registers one
// slab ahead, committed to LDS.  From the LDS slab
//   dgrad: Z[p][k] += sum_{g in slab} dY[g][p] W[k][g]   (lanes along p)
//   wgrad: gW[k][g] += sum_p X[k-tap](p) dY[g][p]         (lanes along g;
//          row K of the A operand = 1 gives the bias gradient)
// Each wave owns position tiles {wave, wave+4, wave+8} for both products, so
// no cross-wave reduction is needed; Z is col2im'ed from LDS per frame and
// the weight-gradient partials are reduced across workgroups in fixed order.
constexpr int BWD_THREADS = 512;  // 8 waves, one workgroup per CU
constexpr int BWD_WAVES = BWD_THREADS / 64;
constexpr int BWD_MAXT = 2;   // position tiles per wave (P <= 512)
constexpr int BWD_MAXV = 8;   // float4 prefetch registers per thread
constexpr int BWD_MAXX = 4;   // X prefetch registers per thread (C*H*W <= 2048)

// slab buffer: a 32 x SP slab, later Z [P][ZZ] and the wave-partial sums
__host__ __device__ inline int bwd_sd_floats(int SP) {
  const int slab = (32 * SP + 3) & ~3;
  return slab > BWD_WAVES * 1024 ? slab : BWD_WAVES * 1024;
}

template <int NCH, bool DX>
__global__ __launch_bounds__(BWD_THREADS, 1) void conv_bwd_frame_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ dY, int dys, const float *__restrict__ K, int ks,
    float *__restrict__ dX, int dxs, float *__restrict__ ws_part, int ZZ,
    int SP, FastDiv div_hp, FastDiv div_hpwp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *Wt = reinterpret_cast<float *>(smem);         // [NCH*32][32]
  float *Sd = Wt + NCH * 32 * 32;                      // [32][SP]  (16-B aligned)
  float *Xs = Sd + bwd_sd_floats(SP) + 32;             // [C][Wp][Hp] + {1}
  int *qtab = reinterpret_cast<int *>(Xs + ((g.C * (g.H + 2 * g.pad_h) *
                                              (g.W + 2 * g.pad_w) + 4) & ~3));
  float *Zs = Sd;                                       // [P][ZZ] after the slabs
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31, h = lane >> 5;
  for (int e = tid; e < NCH * 32 * 32; e += BWD_THREADS) {
    const int gg = e >> 5, k = e & 31;
    Wt[e] = (gg < g.G && k < g.Kdim) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  // wgrad A operand of this lane = row l of the [Kdim+1 x P] im2col tile,
  // read as Xs[min(abase + qmul * qtab[p], CHWp)] (byte offsets):
  //   conv row l < Kdim: abase = its tap offset in the zero-padded frame
  //     map, qtab[p] = px*Hp + py (no bounds tests);
  //   row Kdim and above: the constant slot Xs[CHWp] = 1 (row Kdim is the
  //     bias gradient, rows above are never stored);
  //   p >= P: qtab = huge, clamps to the constant slot, and B is masked to
  //     +0, so padded positions add exact zeros (finite * +0).
  const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
  const int CHWp = g.C * Hp * Wp;
  int abase = CHWp * 4, qmul = 0;
  if (l < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)l, c, r);
    g.div_kh.divmod(r, qx, qy);
    abase = ((int)c * Hp * Wp + (int)qx * Hp + (int)qy) * 4;
    qmul = 1;
  }
  if (tid == 0) Xs[CHWp] = 1.0f;
  for (int p = tid; p < ((g.P + 31) & ~31); p += BWD_THREADS) {
    uint32_t px, py;
    g.div_oh.divmod((uint32_t)p, px, py);
    qtab[p] = p < g.P ? ((int)px * Hp + (int)py) * 4 : 0x3fffffff;
  }
  const uint32_t amax = (uint32_t)CHWp * 4;
  const char *Xb = reinterpret_cast<const char *>(Xs);
  const bool unpadded = g.pad_h == 0 && g.pad_w == 0;
  const int CHW = g.C * g.HW;
  const int ntile = (g.P + 31) >> 5;
  const int nv4 = 8 * g.P;  // float4 per slab (32 * P / 4)

  floatx16 wacc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; c++) wacc[c] = zero16();
  // one slab in flight per thread: BWD_MAXV float4 registers (scalars, so
  // they stay in VGPRs), 16-B aligned linear loads of the 32 x P slab
  float4 p0, p1, p2, p3, p4, p5, p6, p7;
#define KCNN_SLAB_REGS(X) X(0, p0) X(1, p1) X(2, p2) X(3, p3) X(4, p4) X(5, p5) \
  X(6, p6) X(7, p7)
#define KCNN_SLAB_LOAD(i, r) \
  if (tid + BWD_THREADS * (i) < nv4) r = src4[tid + BWD_THREADS * (i)];
#define KCNN_SLAB_STORE(i, r) \
  if (tid + BWD_THREADS * (i) < nv4) dst4[tid + BWD_THREADS * (i)] = r;
  float4 *dst4 = reinterpret_cast<float4 *>(Sd);
  if (blockIdx.x < (unsigned)g.R) {
    const float4 *src4 = reinterpret_cast<const float4 *>(dY + (int64_t)blockIdx.x * dys);
    KCNN_SLAB_REGS(KCNN_SLAB_LOAD)
  }
  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();  // previous frame's Zs / Xs reads are done
    const float *xr = X + (int64_t)n * xs;
    if (unpadded) {
      for (int e = tid; e < CHW; e += BWD_THREADS) Xs[e] = xr[e];
    } else {
      for (int e = tid; e < CHWp; e += BWD_THREADS) {
        uint32_t c, r, wp, hp;
        div_hpwp.divmod((uint32_t)e, c, r);
        div_hp.divmod(r, wp, hp);
        const int wi = (int)wp - g.pad_w, hi = (int)hp - g.pad_h;
        Xs[e] = ((unsigned)wi < (unsigned)g.W && (unsigned)hi < (unsigned)g.H)
                    ? xr[(int)c * g.HW + wi * g.H + hi] : 0.0f;
      }
    }
    floatx16 zacc[BWD_MAXT];
#pragma unroll
    for (int t = 0; t < BWD_MAXT; t++) zacc[t] = zero16();
    // wgrad A operands of this frame (im2col values of the wave's tiles):
    // identical for every slab, so gathered once per frame into registers
    float ain[BWD_MAXT][16];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      KCNN_SLAB_REGS(KCNN_SLAB_STORE)
      __syncthreads();
      {
        const int nn = ch + 1 < NCH ? n : n + (int)gridDim.x;
        const int cc = ch + 1 < NCH ? ch + 1 : 0;
        if (nn < g.R) {
          const float4 *src4 = reinterpret_cast<const float4 *>(
              dY + (int64_t)nn * dys + (int64_t)cc * 32 * g.P);
          KCNN_SLAB_REGS(KCNN_SLAB_LOAD)
        }
      }
      const float *wrow = Wt + (ch * 32 + h) * 32 + l;
#pragma unroll
      for (int t = 0; t < BWD_MAXT; t++) {
        // tiles wave, wave + 8: with waves w and w + 4 sharing a SIMD, every
        // SIMD gets the same tile count (wave-uniform skip of surplus tiles)
        __builtin_amdgcn_sched_barrier(0);
        const int pt = wave + BWD_WAVES * t;
        if (pt >= ntile) continue;
        int pb = pt * 32;
        // opaque per iteration: keeps the frame-invariant operand addresses
        // of all tiles from being hoisted out of the frame loop (that would
        // pin ~150 VGPRs)
        asm volatile("" : "+s"(pb));
        const int ph = pb + h;
        if (ch == 0) {
          const int *qrow = qtab + ph;
#pragma unroll
          for (int s = 0; s < 16; s++) {
            const uint32_t off = min((uint32_t)(abase + qmul * qrow[2 * s]), amax);
            ain[t][s] = *reinterpret_cast<const float *>(Xb + off);
          }
        }
        if (DX) {
          const int pa = pb + l < g.P ? pb + l : g.P - 1;
          const float *srow = Sd + h * SP + pa;
#pragma unroll
          for (int s = 0; s < 16; s++)
            zacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                srow[2 * s * SP], wrow[2 * s * 32], zacc[t], 0, 0, 0);
        }
        const float *scol = Sd + l * SP + ph;
        if (pb + 32 <= g.P) {  // wave-uniform: a full tile
#pragma unroll
          for (int s = 0; s < 16; s++)
            wacc[ch] = __builtin_amdgcn_mfma_f32_32x32x2f32(ain[t][s], scol[2 * s],
                                                           wacc[ch], 0, 0, 0);
        } else {
          // B bit-masked to +0 past P (the row tail reads the next map's
          // data); A is finite there (the clamped constant slot)
#pragma unroll
          for (int s = 0; s < 16; s++) {
            const bool pin = ph + 2 * s < g.P;
            const float bv = __uint_as_float(__float_as_uint(scol[2 * s]) &
                                             (pin ? 0xffffffffu : 0u));
            wacc[ch] = __builtin_amdgcn_mfma_f32_32x32x2f32(ain[t][s], bv, wacc[ch], 0, 0, 0);
          }
        }
      }
      __syncthreads();  // slab consumed
    }
    if (DX) {
#pragma unroll
      for (int t = 0; t < BWD_MAXT; t++) {
        const int pt = wave + BWD_WAVES * t;
        if (pt >= ntile) continue;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int pl = pt * 32 + mfma32_row(r, lane);
          if (pl < g.P && l < g.Kdim) Zs[pl * ZZ + l] = zacc[t][r];
        }
      }
      __syncthreads();
      float *dxr = dX + (int64_t)n * dxs;
      const int khkw = g.kh * g.kw;
      for (int e = tid; e < CHW; e += BWD_THREADS) {
        uint32_t c, q, wi, hi;
        g.div_HW.divmod((uint32_t)e, c, q);
        g.div_H.divmod(q, wi, hi);
        float sum = 0.0f;
        for (int kxx = 0; kxx < g.kw; kxx++) {
          const int px = (int)wi + g.pad_w - kxx;
          if ((unsigned)px >= (unsigned)g.ow) continue;
          const float *zr = Zs + (int64_t)(px * g.oh) * ZZ + (int)c * khkw + kxx * g.kh;
          for (int kyy = 0; kyy < g.kh; kyy++) {
            const int py = (int)hi + g.pad_h - kyy;
            if ((unsigned)py < (unsigned)g.oh) sum += zr[py * ZZ + kyy];
          }
        }
        dxr[e] = sum;
      }
    }
  }
  // sum the waves' partials (each covers its own position tiles) through
  // LDS in a fixed wave order, then one [Kdim+1][G] partial per workgroup
  const int E = (g.Kdim + 1) * g.G;
  float *dst = ws_part + (int64_t)blockIdx.x * E;
  float *red = Sd;  // [BWD_WAVES][32 * 32]; 32 KB <= the slab buffer
#pragma unroll
  for (int ch = 0; ch < NCH; ch++) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++)
      red[wave * 1024 + mfma32_row(r, lane) * 32 + l] = wacc[ch][r];
    __syncthreads();
    for (int e = tid; e < 1024; e += BWD_THREADS) {
      const int i = e >> 5, j = e & 31;
      if (i > g.Kdim) continue;
      float sum = 0.0f;
#pragma unroll
      for (int w = 0; w < BWD_WAVES; w++) sum += red[w * 1024 + e];
      dst[i * g.G + ch * 32 + j] = sum;
    }
  }
}
#undef KCNN_SLAB_LOAD
#undef KCNN_SLAB_STORE
#undef KCNN_SLAB_REGS

// ---------------------------------------------------------------------------
// Fused backward, variant 3: dY slabs reach LDS by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, no VGPRs), double
// buffered, one slab ahead; one barrier per slab.  From the slab in LDS the
// waves run the data gradient (owner waves of each position tile: Z lives
// in their registers for the whole frame) and the weight gradient (tiles
// handed out by the host so every wave carries the same number of 16-MFMA
// chunks; A operands = the frame's im2col values, gathered once per frame
// into the registers of the wave that uses them).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

__host__ __device__ inline int bwd_dma_buf_floats(int P) {
  return ((32 * P * 4 + 1023) & ~1023) / 4;  // whole 1-KiB DMA chunks
}
// both slab buffers; also holds Z [P][Kdim|1] (< 32 P) and the final
// [8 waves][32 x 32] reduction
__host__ __device__ inline int bwd_dma_sd_floats(int P) {
  const int two = 2 * bwd_dma_buf_floats(P);
  return two > BWD_WAVES * 1024 ? two : BWD_WAVES * 1024;
}

//
// PCM > 0: dY is not in HBM.  It is the Backprop of a channel-only Maxpool
// (1 x 1 x PCM) from its routing mask: dY[g][p] = bit g % PCM of
// mask[g / PCM][p] ? dP[g / PCM][p] : 0 (hipF_maxpool_backprop_mask).  dY /
// dys then point at dP, pmask / pms at the mask, and each slab is built in
// LDS from its 32 / PCM rows of dP and mask, loaded into registers at the
// start of the phase before it and expanded after that phase's MFMA chains.
template <int NCH, bool DX, bool WG, int PCM>
__global__ __launch_bounds__(BWD_THREADS, 1) void conv_bwd_dma_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ dY, int dys, const float *__restrict__ K, int ks,
    float *__restrict__ dX, int dxs, float *__restrict__ ws_part, int ZZ,
    unsigned long long wg0, unsigned long long wg1, int zsep, int dx_acc, int dbg,
    const unsigned char *__restrict__ pmask, int pms) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int P = g.P;
  const int BUF = bwd_dma_buf_floats(P);
  float *Wt = reinterpret_cast<float *>(smem);         // [NCH*32][32]
  float *Sd0 = Wt + NCH * 32 * 32;                     // [32][P] x 2 buffers
  float *Xs = Sd0 + bwd_dma_sd_floats(P);              // [C][Wp][Hp] + {1}
  int *qtab = reinterpret_cast<int *>(Xs + ((g.C * (g.H + 2 * g.pad_h) *
                                              (g.W + 2 * g.pad_w) + 4) & ~3));
  // zsep: Z [P][ZZ] has its own buffer, so frame n's col2im runs inside frame
  // n+1's slab phases (next to the other waves' MFMAs) instead of in a
  // barrier-bounded tail; else Z reuses the last slab's buffer
  float *Zsep = reinterpret_cast<float *>(qtab + ((P + 31) & ~31));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31;
  if (DX)  // K and X are only read by the pass that needs them
    for (int e = tid; e < NCH * 32 * 32; e += BWD_THREADS) {
      const int gg = e >> 5, k = e & 31;
      Wt[e] = (gg < g.G && k < g.Kdim) ? K[(int64_t)k * ks + gg] : 0.0f;
    }
  const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
  const int CHWp = g.C * Hp * Wp;
  int abase = CHWp * 4, qmul = 0;
  if (l < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)l, c, r);
    g.div_kh.divmod(r, qx, qy);
    abase = ((int)c * Hp * Wp + (int)qx * Hp + (int)qy) * 4;
    qmul = 1;
  }
  for (int e = tid; e < CHWp; e += BWD_THREADS) Xs[e] = 0.0f;  // padded border
  if (tid == 0) Xs[CHWp] = 1.0f;
  for (int p = tid; p < ((P + 31) & ~31); p += BWD_THREADS) {
    uint32_t px, py;
    g.div_oh.divmod((uint32_t)p, px, py);
    qtab[p] = p < P ? ((int)px * Hp + (int)py) * 4 : 0x3fffffff;
  }
  const uint32_t amax = (uint32_t)CHWp * 4;
  const char *Xb = reinterpret_cast<const char *>(Xs);
  const bool unpadded = g.pad_h == 0 && g.pad_w == 0;
  const int CHW = g.C * g.HW;
  const int ntile = (P + 31) >> 5;
  const int nchunk = BUF / 256;  // 1-KiB chunks per slab
  const int slab = 32 * P;

  // LDS-DMA of slab (n, c) into buffer b: wave w moves chunks w, w+8, ...
  // by buffer_load ... lds -- the chunk offset is a scalar (soffset), the
  // lane's 16 B a constant voffset, so the issue loop costs no VALU work.
  // The descriptor spans the frame's row: a last chunk running past the
  // row reads zeros (hardware range check); past the slab it reads the
  // next slab's first values into an LDS tail that is never read.
  const uint32_t row_bytes = (uint32_t)g.G * (uint32_t)P * 4u;
  auto dma_slab = [&](int n, int c, int b, int ln) {
    const float *base = dY + (int64_t)n * dys;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)row_bytes, 0x00020000);
    float *dst = Sd0 + b * BUF;
    for (int q = wave; q < nchunk; q += BWD_WAVES)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)(dst + q * 256), 16,
                                               (uint32_t)ln * 16u,
                                               (uint32_t)(c * slab + q * 256) * 4u, 0, 0);
  };

  // PCM: a slab's 32 / PCM rows of dP and mask (contiguous in the pooled
  // row).  Thread t < P stages position t of every row (P <= 512), so its
  // slab offsets are j * PCM * P + t: no per-element index arithmetic.
  constexpr int NJ = PCM > 0 ? 32 / PCM : 1;
  float pv[NJ];
  unsigned pm[(NJ + 3) / 4];  // mask bytes, 4 to a register
  auto stage_load = [&](int n, int c, int tt) {
    if (tt >= P) return;
    const int64_t off = (int64_t)c * NJ * P + tt;
    const float *src = dY + (int64_t)n * dys + off;
    const unsigned char *msrc = pmask + (int64_t)n * pms + off;
#pragma unroll
    for (int i = 0; i < (NJ + 3) / 4; i++) pm[i] = 0;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
      pv[j] = src[j * P];
      pm[j / 4] |= (unsigned)msrc[j * P] << (8 * (j % 4));
    }
  };
  auto stage_commit = [&](int b, int tt) {
    if (tt >= P) return;
    float *d = Sd0 + b * BUF + tt;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
      const unsigned v = __float_as_uint(pv[j]);
#pragma unroll
      for (int c = 0; c < PCM; c++) {
        // bit c of the element's mask byte, sign-extended to 0 / ~0
        const int sel = __builtin_amdgcn_sbfe((int)pm[j / 4], 8 * (j % 4) + c, 1);
        d[(j * PCM + c) * P] = __uint_as_float(v & (unsigned)sel);
      }
    }
  };
  floatx16 wacc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; c++) wacc[c] = zero16();
  float xv[BWD_MAXX];
#define KCNN_XLOAD(nn)                                                               \
  _Pragma("unroll") for (int i = 0; i < BWD_MAXX; i++)                              \
    if (WG && tid + BWD_THREADS * i < CHW)                                         \
      xv[i] = X[(int64_t)(nn) * xs + tid + BWD_THREADS * i];
  // X values (in xv) into the padded frame buffer
#define KCNN_XCOMMIT()                                                               \
  _Pragma("unroll") for (int i = 0; i < BWD_MAXX; i++) {                            \
    const int e = tid + BWD_THREADS * i;                                             \
    if (WG && e < CHW) {                                                             \
      int slot = e;                                                                  \
      if (!unpadded) {                                                               \
        uint32_t c, q, wi, hi;                                                       \
        g.div_HW.divmod((uint32_t)e, c, q);                                          \
        g.div_H.divmod(q, wi, hi);                                                   \
        slot = (int)c * Hp * Wp + ((int)wi + g.pad_w) * Hp + (int)hi + g.pad_h;      \
      }                                                                              \
      Xs[slot] = xv[i];                                                              \
    }                                                                                \
  }
  // col2im: dX[nn][e] = sum over the valid taps (kx, ky) of
  // Z[(px*oh + py)*ZZ + c*kh*kw + kx*kh + ky], px = wi + pad_w - kx,
  // py = hi + pad_h - ky.  The output elements of a thread are the same in
  // every frame (e = tid + 512 i), so their Z base offset and valid tap
  // ranges are computed once; per tap that leaves an address subtract, a
  // range test, the read and the add (VALU work is not hidden behind the
  // MFMAs of this kernel: it executes on the same SIMDs, serially).
  const int khkw = g.kh * g.kw;
  const int zax = g.oh * ZZ - g.kh, zby = ZZ - 1;  // Z offset per kx / ky step
  int c2b[BWD_MAXX], c2r[BWD_MAXX];
#pragma unroll
  for (int i = 0; i < BWD_MAXX; i++) {
    const int e = tid + BWD_THREADS * i;
    c2b[i] = 0;
    c2r[i] = (int)0xff000000u;  // no taps (nx = -1)
    if (DX && e < CHW) {
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      const int ty = (int)hi + g.pad_h, tx = (int)wi + g.pad_w;
      c2b[i] = (tx * g.oh + ty) * ZZ + (int)c * khkw;
      const int ylo = max(0, ty - g.oh + 1), yhi = min(g.kh - 1, ty);
      const int xlo = max(0, tx - g.ow + 1), xhi = min(g.kw - 1, tx);
      if (ylo <= yhi && xlo <= xhi)
        c2r[i] = ylo | (yhi - ylo) << 8 | xlo << 16 | (xhi - xlo) << 24;
    }
  }
  auto col2im = [&](const float *Zs, int nn, int i, int tt) {
    const int e = tt + BWD_THREADS * i;
    if (e >= CHW) return;
    const int rg = c2r[i];
    const int ylo = rg & 255, ny = (rg >> 8) & 255, xlo = (rg >> 16) & 255, nx = rg >> 24;
    float sum = 0.0f;
    for (int kx = xlo; kx <= xlo + nx; kx++) {  // kw = 1: one pass
      const int zk = c2b[i] - kx * zax;
      for (int k0 = 0; k0 < g.kh; k0 += 8) {
        // the 8 taps' reads first (one wait), then the masked sum.  A tap
        // outside the map reads another position's Z (or, off the LDS
        // allocation, 0) and is dropped by the mask: no address select
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = Zs[zk - (k0 + u) * zby];
#pragma unroll
        for (int u = 0; u < 8; u++)
          sum += (unsigned)(k0 + u - ylo) <= (unsigned)ny ? v[u] : 0.0f;
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // the reads
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float *d = dX + (int64_t)nn * dxs + e;
    *d = dx_acc ? *d + sum : sum;  // dx_acc: a later filter chunk (G > 128)
  };
  // deferred col2im: pieces in phases 0 .. npiece-1 of the next frame, all
  // before that frame's last slab barrier (Z is rewritten after it)
  const int npiece = NCH > 1 ? NCH - 1 : 1;
  int cur = 0, nprev = -1;
#ifdef KCNN_PHASE_TIMING  // per-phase s_memtime totals of block 0 (dbg & 16)
  long long tm[7] = {0, 0, 0, 0, 0, 0, 0};
  long long tprev = clock64();
#define KCNN_TMARK(i) if (dbg & 16) { const long long tn = clock64(); tm[i] += tn - tprev; tprev = tn; }
#else
#define KCNN_TMARK(i)
#endif
  if (blockIdx.x < (unsigned)g.R) {
    if constexpr (PCM > 0) {
      stage_load(blockIdx.x, 0, tid);
      stage_commit(0, tid);
    } else {
      dma_slab(blockIdx.x, 0, 0, lane);
    }
    KCNN_XLOAD(blockIdx.x)
  }
  __syncthreads();  // zeroed border before the first commit
  if (blockIdx.x < (unsigned)g.R) { KCNN_XCOMMIT() }
  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    // lane ids made opaque per frame (see conv_fwd_regs_kernel)
    int tid_f = tid;
    asm volatile("" : "+v"(tid_f));
    const int lane_f = tid_f & 63, l_f = lane_f & 31, h_f = lane_f >> 5;
    floatx16 zacc[BWD_MAXT];
#pragma unroll
    for (int t = 0; t < BWD_MAXT; t++) zacc[t] = zero16();
    float ain[2][16];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      // slab (n, ch) landed; the other buffer's readers are done.  The
      // explicit vmcnt(0): an LDS-DMA writes LDS, not VGPRs, so no wait of
      // the compiler's covers another wave's reads of it
      KCNN_TMARK(6)
      x6::publish_dma();
      KCNN_TMARK(0)
      {
        const int nn = ch + 1 < NCH ? n : n + (int)gridDim.x;
        const int cc = ch + 1 < NCH ? ch + 1 : 0;
        if (nn < g.R) {
          if constexpr (PCM > 0) stage_load(nn, cc, tid_f);
          else dma_slab(nn, cc, cur ^ 1, lane_f);
          if (ch + 1 == NCH) { KCNN_XLOAD(nn) }
        }
      }
      if (DX && zsep && nprev >= 0) {
#pragma unroll
        for (int i = 0; i < BWD_MAXX; i++)
          if (i % npiece == ch) col2im(Zsep, nprev, i, tid_f);
      }
      KCNN_TMARK(1)
      const float *Sd = Sd0 + cur * BUF;
      const float *wrow = Wt + (ch * 32 + h_f) * 32 + l_f;
      if (DX && wave < ntile) {
        // Z[p][k] += dY[g][p] W[k][g] on the wave's own tiles (wave, wave +
        // 8): the W operand of this slab is read once and shared by both
        // tiles' chains; operand reads are all issued before the chains
        float db[16], da0[16];
#pragma unroll
        for (int s = 0; s < 16; s++) db[s] = wrow[2 * s * 32];
        int pb0 = wave * 32;
        asm volatile("" : "+s"(pb0));
        const float *srow0 = Sd + h_f * P + (pb0 + l_f < P ? pb0 + l_f : P - 1);
#pragma unroll
        for (int s = 0; s < 16; s++) da0[s] = srow0[2 * s * P];
#pragma unroll
        for (int s = 0; s < 16; s++)
          zacc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(da0[s], db[s], zacc[0], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);  // operand reads
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);  // MFMAs
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 1; t < BWD_MAXT; t++) {
          const int pt = wave + BWD_WAVES * t;
          if (pt >= ntile) break;  // wave-uniform; the chain below is in place
          int pb = pt * 32;
          asm volatile("" : "+s"(pb));
          const float *srow = Sd + h_f * P + (pb + l_f < P ? pb + l_f : P - 1);
          float da[16];
#pragma unroll
          for (int s = 0; s < 16; s++) da[s] = srow[2 * s * P];
#pragma unroll
          for (int s = 0; s < 16; s++)
            zacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(da[s], db[s], zacc[t], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      KCNN_TMARK(2)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        if (!WG) break;
        const int pt = (int)(((j ? wg1 : wg0) >> (8 * wave)) & 0xff);
        if (pt == 0xff) continue;
        int pb = pt * 32;
        asm volatile("" : "+s"(pb));
        const int ph = pb + h_f;
        if (ch == 0) {  // the frame's im2col values of this tile
          const int *qrow = qtab + ph;
#pragma unroll
          for (int s = 0; s < 16; s++) {
            const uint32_t off = min((uint32_t)(abase + qmul * qrow[2 * s]), amax);
            ain[j][s] = *reinterpret_cast<const float *>(Xb + off);
          }
        }
        const float *scol = Sd + l_f * P + ph;
        // one MFMA chain for full and partial tiles (a branch around the
        // chain makes the compiler copy the accumulator between register
        // sets, draining the MFMA pipeline at every tile); only the B
        // operand masking of the partial tile sits in a branch.  Past P a
        // row's tail reads the next map's values: bit-masked to +0.
        float wb[16];
#pragma unroll
        for (int s = 0; s < 16; s++) wb[s] = scol[2 * s];
        if (pb + 32 > P) {  // wave-uniform
          // k-step s covers positions ph + 2s, ph = pb + h: with lim =
          // P - pb - 2s (uniform) both halves are in for lim >= 2, only
          // h = 0 for lim == 1, neither below
#pragma unroll
          for (int s = 0; s < 16; s++) {
            const int lim = P - pb - 2 * s;
            if (lim <= 0 || (lim == 1 && h_f)) wb[s] = 0.0f;
          }
        }
#pragma unroll
        for (int s = 0; s < 16; s++)
          wacc[ch] = __builtin_amdgcn_mfma_f32_32x32x2f32(ain[j][s], wb[s], wacc[ch], 0, 0, 0);
      }
      if constexpr (PCM > 0) {  // the next slab, expanded into the other buffer
        const int nn = ch + 1 < NCH ? n : n + (int)gridDim.x;
        if (nn < g.R) stage_commit(cur ^ 1, tid_f);
      }
      KCNN_TMARK(3)
      if (ch + 1 < NCH) cur ^= 1;
    }
    // with one slab per frame, this frame's gather / col2im readers are
    // only fenced by a barrier here
    if (NCH == 1) __syncthreads();
    if (DX) {
      // zsep: Z's readers (the previous col2im) finished before the last slab
      // barrier; else every wave must be done with the last slab's buffer
      if (!zsep) __syncthreads();
      float *Zs = zsep ? Zsep : Sd0 + cur * BUF;
#pragma unroll
      for (int t = 0; t < BWD_MAXT; t++) {
        const int pt = wave + BWD_WAVES * t;
        if (pt >= ntile) continue;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int pl = pt * 32 + mfma32_row(r, lane_f);
          if (pl < P && l_f < g.Kdim) Zs[pl * ZZ + l_f] = zacc[t][r];
        }
      }
      if (zsep) {
        nprev = n;
      } else {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < BWD_MAXX; i++) col2im(Zs, n, i, tid_f);
        __syncthreads();  // Zs (slab buffer) readers done before its next DMA
      }
    }
    // the next frame's X: this frame's gather (phase 0) is behind a barrier
    if (WG && n + (int)gridDim.x < g.R) { KCNN_XCOMMIT() }
    KCNN_TMARK(4)
    cur ^= 1;  // the next frame's first slab is in the other buffer
  }
  if (DX && zsep && nprev >= 0) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < BWD_MAXX; i++) col2im(Zsep, nprev, i, tid);
  }
  KCNN_TMARK(5)
#ifdef KCNN_PHASE_TIMING
  if ((dbg & 16) && blockIdx.x == 0 && lane == 0)
    printf("bwd3 wave %d: barrier %lld dma %lld dgrad %lld wgrad %lld tail %lld end %lld other %lld\n",
           wave, tm[0], tm[1], tm[2], tm[3], tm[4], tm[5], tm[6]);
#endif
#undef KCNN_TMARK
#undef KCNN_XLOAD
#undef KCNN_XCOMMIT
  if (!WG) return;
  const int E = (g.Kdim + 1) * g.G;
  float *dst = ws_part + (int64_t)blockIdx.x * E;
  float *red = Sd0;  // [BWD_WAVES][32 * 32]; no DMA in flight any more
#pragma unroll
  for (int ch = 0; ch < NCH; ch++) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++)
      red[wave * 1024 + mfma32_row(r, lane) * 32 + l] = wacc[ch][r];
    __syncthreads();
    for (int e = tid; e < 1024; e += BWD_THREADS) {
      const int i = e >> 5, j = e & 31;
      if (i > g.Kdim) continue;
      float sum = 0.0f;
#pragma unroll
      for (int w = 0; w < BWD_WAVES; w++) sum += red[w * 1024 + e];
      dst[i * g.G + ch * 32 + j] = sum;
    }
  }
}

// ---------------------------------------------------------------------------
// NK = G/2 k-steps, fully unrolled: every A load of a 32-position tile is
// issued before the MFMA chain consumes it (64 x 256 B in flight per wave at
// G = 128), which is what hides HBM latency here.  Lanes past the last
// position read a clamped address; their Z rows are never stored.
template <int NK>
__global__ __launch_bounds__(256) void conv_dgrad_frame_kernel(
    ConvGeom g, const float *__restrict__ dY, int dys,
    const float *__restrict__ K, int ks, float *__restrict__ dX, int dxs,
    int ZZ) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *Wt = reinterpret_cast<float *>(smem);   // [2*NK][32]: Wt[g][k] = W[k][g]
  float *Zs = Wt + 2 * NK * 32;                  // [P][ZZ]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 2 * NK * 32; e += 256) {
    const int gg = e >> 5, k = e & 31;
    Wt[e] = (gg < g.G && k < g.Kdim) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  const int ntile = (g.P + 31) >> 5;
  const int CHW = g.C * g.HW;
  const int khkw = g.kh * g.kw;
  const float *wcol = Wt + (lane >> 5) * 32 + (lane & 31);

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();  // Wt ready / previous col2im done with Zs
    const float *dyr = dY + (int64_t)n * dys;
    for (int pt = wave; pt < ntile; pt += 4) {
      const int p = pt * 32 + (lane & 31);
      const int pc = p < g.P ? p : g.P - 1;
      const float *col = dyr + pc + (int64_t)(lane >> 5) * g.P;
      float a[NK];
#pragma unroll
      for (int s = 0; s < NK; s++) a[s] = col[(int64_t)(2 * s) * g.P];
      floatx16 acc = zero16();
#pragma unroll
      for (int s = 0; s < NK; s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], wcol[s * 64], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int pl = pt * 32 + mfma32_row(r, lane);
        if (pl < g.P && (lane & 31) < g.Kdim) Zs[pl * ZZ + (lane & 31)] = acc[r];
      }
    }
    __syncthreads();
    float *dxr = dX + (int64_t)n * dxs;
    for (int e = tid; e < CHW; e += 256) {
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      float sum = 0.0f;
      for (int kx = 0; kx < g.kw; kx++) {
        const int px = (int)wi + g.pad_w - kx;
        if ((unsigned)px >= (unsigned)g.ow) continue;
        const float *zr = Zs + (int64_t)(px * g.oh) * ZZ + (int)c * khkw + kx * g.kh;
        for (int ky = 0; ky < g.kh; ky++) {
          const int py = (int)hi + g.pad_h - ky;
          if ((unsigned)py < (unsigned)g.oh) sum += zr[py * ZZ + ky];
        }
      }
      dxr[e] = sum;
    }
  }
}

// ---------------------------------------------------------------------------
template <int NSUP>
__global__ __launch_bounds__(256) void conv_wgrad_frame_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ dY, int dys, float *__restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *Ds = reinterpret_cast<float *>(smem);   // [4 waves][32][ZS]
  float *Xs = Ds + 4 * 32 * ZS;                   // [C*HW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float *myD = Ds + wave * 32 * ZS;

  // A-row of this lane: conv row j (< Kdim), the ones row (== Kdim), or pad.
  const int j = lane & 31;
  int koff = 0, kx = 0, ky = 0;
  if (j < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)j, c, r);
    g.div_kh.divmod(r, qx, qy);
    koff = (int)c * g.HW;
    kx = (int)qx;
    ky = (int)qy;
  }
  const bool is_ones = (j == g.Kdim);
  const int CHW = g.C * g.HW;

  floatx16 acc[NSUP];
#pragma unroll
  for (int su = 0; su < NSUP; su++) acc[su] = zero16();

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();
    const float *xr = X + (int64_t)n * xs;
    for (int e = tid; e < CHW; e += 256) Xs[e] = xr[e];
    __syncthreads();
    const float *dyr = dY + (int64_t)n * dys;
#pragma unroll
    for (int su = 0; su < NSUP; su++) {
      const int g0 = (su * 4 + wave) * 32;
      if (g0 >= g.G) continue;  // wave-uniform
      // dY tile rows g0 + 2i + (lane >> 5), column pc + (lane & 31); rows past
      // G or columns past P read a clamped address and are zeroed.
      const int gl0 = lane >> 5, pl0 = lane & 31;
      float nxt[16];
      auto load_tile = [&](int pc) {
        const bool pv = pc + pl0 < g.P;
        const int pcl = pv ? pc + pl0 : g.P - 1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
          const int gg = g0 + 2 * i + gl0;
          const bool v = pv && gg < g.G;
          const float x = dyr[(int64_t)(v ? gg : 0) * g.P + pcl];
          nxt[i] = v ? x : 0.0f;
        }
      };
      load_tile(0);
      for (int pc = 0; pc < g.P; pc += 32) {
#pragma unroll
        for (int i = 0; i < 16; i++) myD[(2 * i + gl0) * ZS + pl0] = nxt[i];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (pc + 32 < g.P) load_tile(pc + 32);  // in flight during the MFMAs
        // im2col operand for p = pc + 2s + (lane >> 5), walked incrementally
        uint32_t px, py;
        g.div_oh.divmod((uint32_t)(pc + gl0), px, py);
        int ipx = (int)px, ipy = (int)py;
#pragma unroll 4
        for (int s = 0; s < 16; s++) {
          const int p = pc + 2 * s + gl0;
          const int xx = ipx + kx - g.pad_w, yy = ipy + ky - g.pad_h;
          const bool ok = j < g.Kdim && p < g.P && (unsigned)xx < (unsigned)g.W &&
                          (unsigned)yy < (unsigned)g.H;
          const float xv = Xs[ok ? koff + xx * g.H + yy : 0];
          const float av = ok ? xv : ((is_ones && p < g.P) ? 1.0f : 0.0f);
          const float bv = myD[(lane & 31) * ZS + 2 * s + gl0];
          acc[su] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[su], 0, 0, 0);
          ipy += 2;
          while (ipy >= g.oh) { ipy -= g.oh; ipx++; }
        }
      }
    }
  }
  // partial [Kdim + 1][G] of this workgroup
  const int E = (g.Kdim + 1) * g.G;
  float *dst = ws + (int64_t)blockIdx.x * E;
#pragma unroll
  for (int su = 0; su < NSUP; su++) {
    const int gl = (su * 4 + wave) * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int i = mfma32_row(r, lane);
      if (i <= g.Kdim && gl < g.G) dst[i * g.G + gl] = acc[su][r];
    }
  }
}

// ---------------------------------------------------------------------------
// Pass 1 of the implicit-GEMM v1 split-K reduction: sums groups of 32
// partial rows (conv_splitk_reduce_kernel adds the groups in order).
__global__ __launch_bounds__(256) void reduce_pass1(const float *__restrict__ in,
                                                    int S, int E,
                                                    float *__restrict__ tmp) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const int s0 = blockIdx.y * 32, s1 = min(S, s0 + 32);
  float acc = 0.0f;
  for (int s = s0; s < s1; s++) acc += in[(int64_t)s * E + e];
  tmp[(int64_t)blockIdx.y * E + e] = acc;
}

// One-pass deterministic reduction of S partial rows [S][E]: a block takes 64
// columns; its 4 waves sum interleaved rows (s = w, w + 4, ...) with the loads
// of 16 rows in flight, then add the 4 wave sums in order through LDS.  Same
// output mapping: e < nw -> gW[row][col] with (row, col) = gk_layout ?
// (e % inner, e / inner) : (e / inner, e % inner); e >= nw -> gb[e - nw].
// (Two passes of 32-row groups spent ~14 us of latency at c2, for 3.3 MB.)
// u.W != NULL (conv-update.h): the sums step W / prev (momentum_step) and b
// instead of being stored in gW / gb (W and prev with gW's (row, col)).
__global__ __launch_bounds__(256) void reduce_splits_kernel(
    const float *__restrict__ in, int S, int E, int nw, int inner, int gk_layout,
    float *__restrict__ gW, int gws, float *__restrict__ gb, ConvUpdateEpi u) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + c;
  float acc = 0.0f;
  if (e < E) {
    int s = w;
    for (; s + 4 * 15 < S; s += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; u++) v[u] = in[(int64_t)(s + 4 * u) * E + e];
#pragma unroll
      for (int u = 0; u < 16; u++) acc += v[u];
    }
    for (; s < S; s += 4) acc += in[(int64_t)s * E + e];
  }
  red[w][c] = acc;
  __syncthreads();
  if (w != 0 || e >= E) return;
  const float sum = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
  if (e < nw) {
    const int a = e / inner, b = e - a * inner;
    const int row = gk_layout ? b : a, col = gk_layout ? a : b;
    if (u.W) {  // ApplyGradient's MomentumUpdate on this element
      float *pw = u.W + (int64_t)row * u.ldw + col, *pp = u.prev + (int64_t)row * u.ldp + col;
      float p = *pp, w = *pw;
      kcnn::momentum_step(sum, p, w, u.momentum, u.a_wd, u.a_g);
      *pp = p;
      *pw = w;
    } else {
      gW[(int64_t)row * gws + col] = sum;
    }
  } else if (u.W) {  // its BiasUpdate
    u.b[e - nw] = __builtin_fmaf(u.a_g, sum, u.b[e - nw]);
  } else if (gb) {
    gb[e - nw] = sum;
  }
}

size_t fwd_lds(const ConvGeom &g, int Kpad, int Gp) {
  return (size_t)align16(Kpad * 8) + (size_t)Kpad * Gp * 4 + (size_t)g.C * g.HW * 4;
}

// conv_fwd_regs_kernel: 3 resident blocks per CU when their LDS fits (c2:
// 52 KB each; VGPRs allow 3).  The third block overlaps the others' store
// and barrier phases: c2 forward+pool 224 -> 200 us, although 4096 frames
// then split 5/6 per block instead of 8.
int fwd_regs_blocks_per_cu(size_t lds) {
  return lds * 3 <= 160 * 1024 ? 3 : 2;
}

// The register forward on the bf16 matrix cores (X6): unpadded maps with
// Kdim <= 31 (the bias takes row Kdim of at most two k16 steps) and one
// filter chunk (G <= 128).  Its ~200 VGPRs hold two workgroups per CU where
// the fp32 kernel holds three, and the kernel is bound by its gather and
// pool/store epilogue more than by its MFMAs: c2 fused forward + pool 137 ->
// 132 us, but c5 C1 (G = 256 in two chunks, 3-D pool from LDS) 0.52 ->
// 0.62 ms with the runtime window, and the same speed (c5 447.0 k vs 446.5 k
// frames/s) once the 3 x 1 x 4 window is compiled in, so chunked layers keep
// the fp32 MFMA.  The rule depends on the
// layer's shape only, so a fused and an unfused run of a layer use the same
// arithmetic (bitwise-equal outputs).  KCNN_FWD_X6=0 keeps the fp32 MFMA.
// The f16x3 form (family value 2, the default) has the same limits except
// Kdim <= 32 (no bias row) and half the MFMAs per item.
// Returns the kernel's AR: 0 fp32 MFMA, 1 bf16x6, 2 f16x3.
int fwd_arith(const ConvGeom &g, int use) {
  if (!use || g.pad_h != 0 || g.pad_w != 0 || g.Gtot > 128) return 0;
  if (use == 2) return g.Kdim <= 32 ? 2 : 0;
  return g.Kdim <= 31 ? 1 : 0;
}

unsigned frame_grid(const ConvGeom &g, int blocks_per_cu) {
  int64_t b = 256LL * blocks_per_cu;
  if (b > g.R) b = g.R;
  return (unsigned)(b > 0 ? b : 1);
}

}  // namespace

// The fused conv + pool forward's Y stores (fusion mode 2, Y kept for later)
// as streaming stores (vec_ok bit 1): c2 213 -> 206 us.  Not for the unfused
// conv, whose Y the pool reads right after (155 -> 181 us there).
// KCNN_CONV_Y_NT=0 plain stores
static int y_nt() {
  static const int v = KCNN_KNOB("KCNN_CONV_Y_NT", 1) ? 2 : 0;
  return v;
}

int kcnn_conv_fwd_frame(const ConvGeom &g, const float *X, int xs,
                        const float *K, int ks, const float *bias, float *out,
                        int os, hipStream_t st) {
  if (g.Kdim > 64 || g.P < 16) return -1;
  if (g.G > 128 && g.G % 32 == 0 && g.Kdim <= 32) {
    // filter chunks of 128: each is a column range of W, b and Y
    for (int g0 = 0; g0 < g.G; g0 += 128) {
      ConvGeom gc = g;
      gc.G = g.G - g0 < 128 ? g.G - g0 : 128;
      const int rc = kcnn_conv_fwd_frame(gc, X, xs, K + g0, ks, bias ? bias + g0 : nullptr,
                                         out + (int64_t)g0 * g.P, os, st);
      if (rc) return g0 == 0 ? rc : (rc < 0 ? (int)hipErrorLaunchFailure : rc);
    }
    return 0;
  }
  const int Kpad = (g.Kdim + 1) & ~1;
  static const int variant = KCNN_KNOB("KCNN_FWD_VARIANT", 2);
  if (variant == 2 && g.Kdim <= 32 && g.G <= 128 && g.P <= 4 * 32 * 3 &&
      g.C * g.HW <= 256 * 8) {
    const size_t lds = (size_t)((32 * g.P + 3) & ~3) * 4 + 160 * 4 + 32 * 8 +
                       (size_t)g.C * g.HW * 4 + 8 * 4;
    if (lds <= (size_t)kFrameLdsMax) {
      const int vec_ok = ((uintptr_t)out % 16 == 0) && (os % 4 == 0);
      const int ksn = (g.Kdim + 1) / 2;
      static const int bpc_env = KCNN_KNOB("KCNN_FWD_BPC", 0);
      const int ar = fwd_arith(g, family(kFamFwdX6));
      const unsigned grid = frame_grid(
          g, bpc_env > 0 ? bpc_env : ar ? 2 : fwd_regs_blocks_per_cu(lds));
#define KCNN_FWD_REGS_T(KS_, AR_)                                                       \
  hipLaunchKernelGGL((conv_fwd_regs_kernel<KS_, 3, 0, AR_>), dim3(grid), dim3(256), lds, \
                     st, g, X, xs, K, ks, bias, out, os, vec_ok, dbg, nullptr, 0, nullptr, \
                     0, PoolWin{}, RpStats{})
#define KCNN_FWD_REGS(KS_) KCNN_FWD_REGS_T(KS_, 0)
      static const int dbg = KCNN_KNOB("KCNN_FWD_DEBUG", 0);
      if (ar == 2 && g.Kdim <= 16) KCNN_FWD_REGS_T(1, 2);
      else if (ar == 2) KCNN_FWD_REGS_T(2, 2);
      else if (ar == 1 && g.Kdim < 16) KCNN_FWD_REGS_T(1, 1);
      else if (ar == 1) KCNN_FWD_REGS_T(2, 1);
      else if (ksn <= 4) KCNN_FWD_REGS(4);
      else if (ksn <= 8) KCNN_FWD_REGS(8);
      else if (ksn <= 12) KCNN_FWD_REGS(12);
      else KCNN_FWD_REGS(16);
#undef KCNN_FWD_REGS
#undef KCNN_FWD_REGS_T
      return (int)hipGetLastError();
    }
  }
  if (variant >= 1) {
    // slab-streamed: T [32][P] staged in LDS, written as whole 16-B lines
    const int Gp = (g.G + 31) & ~31;
    const size_t lds = (size_t)align16(Kpad * 8) + (size_t)((32 * g.P + 3) & ~3) * 4 +
                       (size_t)Kpad * Gp * 4 + (size_t)g.C * g.HW * 4;
    if (lds <= (size_t)kFrameLdsMax) {
      const int vec_ok = ((uintptr_t)out % 16 == 0) && (os % 4 == 0);
      hipLaunchKernelGGL(conv_fwd_slab_kernel, dim3(frame_grid(g, 2)), dim3(256),
                         lds, st, g, X, xs, K, ks, bias, out, os, Kpad, Gp, vec_ok);
      return (int)hipGetLastError();
    }
  }
  const int ngb = g.G > 64 ? 4 : (g.G > 32 ? 2 : 1);
  const int Gp = (g.G + 32 * ngb - 1) / (32 * ngb) * (32 * ngb);
  const size_t lds = fwd_lds(g, Kpad, Gp);
  if (lds > (size_t)kFrameLdsMax) return -1;
  const unsigned grid = frame_grid(g, 4);
  if (ngb == 4) {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<4>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  } else if (ngb == 2) {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<2>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  } else {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<1>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  }
  return (int)hipGetLastError();
}

// Forward + channel-only max pool (pool 1 x 1 x pc) in one pass; -1 when the
// geometry is outside the register-resident kernel's limits.
int kcnn_conv_fwd_frame_pool(const ConvGeom &g, const float *X, int xs,
                             const float *K, int ks, const float *bias,
                             float *out, int os, float *pool, int ps,
                             unsigned char *mask, int ms, int pc,
                             hipStream_t st, int ph, int pw, PoolStatsOut *stats) {
  if (stats) stats->produced = 0;
  const bool win3 = ph > 1 || pw > 1;  // 16-bit mask; ms in mask elements
  if (win3) {
    if (pc < 1 || 32 % pc != 0 || ph * pw * pc > 16 || g.oh % ph != 0 || g.ow % pw != 0)
      return -1;
  } else if (!(pc == 2 || pc == 4 || pc == 8)) {
    return -1;
  }
  if (g.G % pc != 0) return -1;
  const int OP = win3 ? (g.oh / ph) * (g.ow / pw) : g.P;  // pooled positions per map
  if (g.G > 128 && g.G % 32 == 0) {  // filter chunks of 128 (pool groups never straddle)
    for (int g0 = 0; g0 < g.G; g0 += 128) {
      ConvGeom gc = g;
      gc.G = g.G - g0 < 128 ? g.G - g0 : 128;
      const int64_t pofs = (int64_t)(g0 / pc) * OP;
      unsigned char *mc = win3 ? reinterpret_cast<unsigned char *>(
                                     reinterpret_cast<unsigned short *>(mask) + pofs)
                               : mask + pofs;
      const int rc = kcnn_conv_fwd_frame_pool(gc, X, xs, K + g0, ks, bias ? bias + g0 : nullptr,
                                              out ? out + (int64_t)g0 * g.P : nullptr, os,
                                              pool + pofs, ps,
                                              mc, ms, pc, st, ph, pw, nullptr);
      if (rc) return g0 == 0 ? rc : (rc < 0 ? (int)hipErrorLaunchFailure : rc);
    }
    return 0;
  }
  PoolWin pw3{};
  if (win3) {
    pw3.ph = ph; pw3.pw = pw; pw3.pc = pc;
    pw3.oh2 = g.oh / ph;
    pw3.OP = OP;
    pw3.div_OP = FastDiv((uint32_t)OP);
    pw3.div_oh2 = FastDiv((uint32_t)pw3.oh2);
  }
  if (g.Kdim > 32 || g.G > 128 || g.P < 16 || g.P > 4 * 32 * 3 ||
      g.C * g.HW > 256 * 8)
    return -1;
  const size_t lds = (size_t)((32 * g.P + 3) & ~3) * 4 + 160 * 4 + 32 * 8 +
                     (size_t)g.C * g.HW * 4 + 8 * 4;
  if (lds > (size_t)kFrameLdsMax) return -1;
  const int vec_ok = ((uintptr_t)out % 16 == 0) && (os % 4 == 0) ? 1 | y_nt() : 0;
  const int ksn = (g.Kdim + 1) / 2;
  static const int grid_env = KCNN_KNOB("KCNN_FWD_GRID", 0);
  const int ar = fwd_arith(g, family(kFamFwdX6));
  const unsigned grid = grid_env > 0 ? (unsigned)std::min<int64_t>(grid_env, g.R)
                                     : frame_grid(g, ar ? 2 : fwd_regs_blocks_per_cu(lds));
  static const int dbg = KCNN_KNOB("KCNN_FWD_DEBUG", 0);
  // the register-pooled-only form: pooled output only, pc 4, G = 128 and
  // exactly 12 position tiles, so each of the 4 waves has all 3 (the form
  // runs every item unfiltered: with 9-11 tiles a wave's third tile would
  // pool and take statistics from registers no gather wrote)
  const int ntile = (g.P + 31) / 32;
  // (its LDS: 8 more words of row slots)
  const size_t lds_rp = lds + 8 * 4;
  const bool rp = out == nullptr && pc == 4 && !win3 && g.G == 128 && ntile == 4 * 3 &&
                  ar == 2 && lds_rp <= (size_t)kFrameLdsMax;
  // the register-pooled kernel also gives the pooled output's max |value|
  // bits per frame and per column (stats, when the caller passes room)
  RpStats rps;
  if (rp && stats && stats->partials &&
      stats->partial_words >= ((size_t)grid * (g.G / pc) * g.P + 3) / 4 &&
      (size_t)grid * 256 >= (size_t)(g.G / pc) * g.P) {
    rps.rowmax = stats->rowmax;
    rps.partials = stats->partials;
    rps.colmax = stats->colmax;
  }
  uint32_t *pcol = rps.partials;
#define KCNN_FWD_POOL_T(KS_, PC_, AR_)                                                      \
  do {                                                                                       \
    if (rp && PC_ == 4 && AR_ == 2)                                                          \
      hipLaunchKernelGGL((conv_fwd_regs_kernel<KS_, 3, PC_, AR_, PC_ == 4 && AR_ == 2>),     \
                         dim3(grid), dim3(256), lds_rp, st, g, X, xs, K, ks, bias, out, os,  \
                         vec_ok, dbg, pool, ps, mask, ms, pw3, rps);                         \
    else                                                                                     \
      hipLaunchKernelGGL((conv_fwd_regs_kernel<KS_, 3, PC_, AR_>), dim3(grid), dim3(256), lds, \
                         st, g, X, xs, K, ks, bias, out, os, vec_ok, dbg, pool, ps, mask, ms, pw3, \
                         RpStats{});                                                         \
  } while (0)
#define KCNN_FWD_POOL(KS_, PC_) KCNN_FWD_POOL_T(KS_, PC_, 0)
#define KCNN_FWD_POOL_KS(PC_)                     \
  do {                                            \
    if (ar == 2 && g.Kdim <= 16) KCNN_FWD_POOL_T(1, PC_, 2); \
    else if (ar == 2) KCNN_FWD_POOL_T(2, PC_, 2); \
    else if (ar == 1 && g.Kdim < 16) KCNN_FWD_POOL_T(1, PC_, 1); \
    else if (ar == 1) KCNN_FWD_POOL_T(2, PC_, 1); \
    else if (ksn <= 4) KCNN_FWD_POOL(4, PC_);     \
    else if (ksn <= 8) KCNN_FWD_POOL(8, PC_);     \
    else if (ksn <= 12) KCNN_FWD_POOL(12, PC_);   \
    else KCNN_FWD_POOL(16, PC_);                  \
  } while (0)
  static const int win_ct = KCNN_KNOB("KCNN_FWD_WIN_CT", 1);  // 0: the runtime window
  if (win3 && win_ct && ph == 3 && pw == 1 && pc == 4) KCNN_FWD_POOL_KS(-3);
  else if (win3) KCNN_FWD_POOL_KS(-1);
  else if (pc == 2) KCNN_FWD_POOL_KS(2);
  else if (pc == 4) KCNN_FWD_POOL_KS(4);
  else KCNN_FWD_POOL_KS(8);
#undef KCNN_FWD_POOL_KS
#undef KCNN_FWD_POOL
#undef KCNN_FWD_POOL_T
  if (pcol) {
    PoolColDeferred d;
    d.pcol = reinterpret_cast<const uint8_t *>(pcol);
    d.nblk = (int)grid;
    d.npool = g.G / pc * g.P;
    d.P = pool;
    d.ps = ps;
    d.R = g.R;
    d.vec = ps % 4 == 0 && (uintptr_t)pool % 16 == 0;
    d.rowblk = stats->rowmax;
    d.colblk = stats->colmax;
    d.pending = 1;
    stats->produced = 1;
    if (PoolColDeferred *req = kcnn_pool_defer_current())
      *req = d;  // the consumer's statistics launches take it
    else return kcnn_pool_cols_complete(&d, reinterpret_cast<kcnn_stream_t>(st));
  }
  return (int)hipGetLastError();
}

int kcnn_pool_cols_complete(PoolColDeferred *d, kcnn_stream_t stream) {
  if (!d || !d->pending) return 0;
  d->pending = 0;
  hipStream_t st = kcnn::as_stream(stream);
  const int ncq = d->npool % 4 == 0 ? d->npool / 4 : d->npool;  // pool_colmax_kernel's threads
  hipLaunchKernelGGL(pool_colmax_kernel,
                     dim3((ncq + 255) / 256, (d->nblk + COLMAX_ROWS - 1) / COLMAX_ROWS),
                     dim3(256), 0, st, d->pcol, d->nblk, d->npool, d->colblk);
  // 256 blocks (c2: 41 suspect frames of 4096, at most one each); a pass
  // of 4096 frames gives a block at most 4096 / 256 = CNT_LIST of them
  const int cgrid = std::min(d->R, 256);
  hipLaunchKernelGGL(pool_count_kernel, dim3(cgrid), dim3(256), 0, st, d->P, d->ps, d->R,
                     d->npool, d->vec, d->rowblk, d->colblk);
  return (int)hipGetLastError();
}

size_t kcnn_pool_stats_partial_words(const ConvGeom &g, int pc) {
  // frame_grid(g, 2) workgroups (the f16x3 register kernel) x pooled columns
  // exponent bytes of the maxima
  return pc > 0 ? ((size_t)frame_grid(g, 2) * (g.G / pc) * g.P + 3) / 4 : 0;
}

int kcnn_conv_dgrad_frame(const ConvGeom &g, const float *dY, int dys,
                          const float *K, int ks, float *dX, int dxs,
                          hipStream_t st) {
  if (g.Kdim > 32) return -1;
  if (g.G != 64 && g.G != 128) return -1;  // NK = G/2, fully unrolled
  const int ZZ = g.Kdim | 1;               // odd row stride: conflict-free col2im
  const size_t lds = ((size_t)g.G * 32 + (size_t)g.P * ZZ) * 4;
  if (lds > (size_t)kFrameLdsMax) return -1;
  if (g.G == 128)
    hipLaunchKernelGGL(conv_dgrad_frame_kernel<64>, dim3(frame_grid(g, 3)),
                       dim3(256), lds, st, g, dY, dys, K, ks, dX, dxs, ZZ);
  else
    hipLaunchKernelGGL(conv_dgrad_frame_kernel<32>, dim3(frame_grid(g, 3)),
                       dim3(256), lds, st, g, dY, dys, K, ks, dX, dxs, ZZ);
  return (int)hipGetLastError();
}

static int wgrad_frame_blocks(const ConvGeom &g) { return (int)frame_grid(g, 2); }

size_t kcnn_conv_wgrad_frame_ws(const ConvGeom &g) {
  if (g.Kdim > 31 || g.G > 256) return 0;
  const size_t lds = (size_t)(4 * 32 * ZS + g.C * g.HW) * 4;
  if (lds > (size_t)kFrameLdsMax) return 0;
  const int S = wgrad_frame_blocks(g);
  const int E = (g.Kdim + 1) * g.G;
  return (size_t)S * E * 4 + kcnn_reduce_splits_ws(S, E);
}

int kcnn_conv_wgrad_frame(const ConvGeom &g, const float *X, int xs,
                          const float *dY, int dys, float *gW, int gws,
                          float *gb, void *ws, size_t ws_bytes, hipStream_t st) {
  const size_t need = kcnn_conv_wgrad_frame_ws(g);
  if (need == 0 || ws == nullptr || ws_bytes < need) return -1;
  const int S = wgrad_frame_blocks(g);
  const int E = (g.Kdim + 1) * g.G;
  float *part = static_cast<float *>(ws);
  float *tmp = part + (size_t)S * E;
  const size_t lds = (size_t)(4 * 32 * ZS + g.C * g.HW) * 4;
  if (g.G <= 128)
    hipLaunchKernelGGL(conv_wgrad_frame_kernel<1>, dim3(S), dim3(256), lds, st,
                       g, X, xs, dY, dys, part);
  else
    hipLaunchKernelGGL(conv_wgrad_frame_kernel<2>, dim3(S), dim3(256), lds, st,
                       g, X, xs, dY, dys, part);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  (void)tmp;
  hipLaunchKernelGGL(reduce_splits_kernel, dim3((E + 63) / 64), dim3(256), 0, st, part, S,
                     E, g.Kdim * g.G, g.G, 0, gW, gws, gb, ConvUpdateEpi{});
  return (int)hipGetLastError();
}

static size_t bwd_lds(const ConvGeom &g, int SP) {
  const int NCH = g.G / 32;
  const size_t chwp = (size_t)g.C * (g.H + 2 * g.pad_h) * (g.W + 2 * g.pad_w);
  return ((size_t)NCH * 32 * 32 + (size_t)bwd_sd_floats(SP) + 32 +
          ((chwp + 4) & ~(size_t)3) + (size_t)((g.P + 31) & ~31)) * 4;
}

static int bwd_sp(const ConvGeom &g) { return g.P; }  // P odd: conflict-free slab reads

size_t kcnn_conv_bwd_frame_ws(const ConvGeom &g) {
  if (g.G > 128 && g.G % 32 == 0) {  // chunks of 128 filters share the workspace
    ConvGeom gc = g;
    gc.G = 128;
    return kcnn_conv_bwd_frame_ws(gc);
  }
  if (g.Kdim > 31 || g.G % 32 != 0 || g.G > 128 || g.G == 0) return 0;
  if ((g.P < 16 || g.P > 32 * BWD_WAVES * BWD_MAXT || 8 * g.P > BWD_THREADS * BWD_MAXV) &&
      !kcnn_conv_bwd_x6_eligible(g, true, 0))
    return 0;
  const int S = (int)frame_grid(g, 1);
  const int E = (g.Kdim + 1) * g.G;
  return (size_t)S * E * 4 + kcnn_reduce_splits_ws(S, E);
}

static size_t bwd_dma_lds(const ConvGeom &g) {
  return ((size_t)(g.G / 32) * 32 * 32 + (size_t)bwd_dma_sd_floats(g.P) +
          (((size_t)g.C * (g.H + 2 * g.pad_h) * (g.W + 2 * g.pad_w) + 4) & ~(size_t)3) +
          (size_t)((g.P + 31) & ~31)) * 4;
}

// One filter chunk (G <= 128) of kcnn_conv_bwd_frame; dx_acc adds to dX.
// pc > 0: dY / dys are the pooled derivative dP of a 1 x 1 x pc Maxpool and
// pmask / pms its routing mask (see conv_bwd_dma_kernel).
static int bwd_frame_chunk(const ConvGeom &g, const float *X, int xs,
                           const float *dY, int dys, const float *K, int ks,
                           float *dX, int dxs, float *gW, int gws, float *gb,
                           void *ws, size_t ws_bytes, int dx_acc, hipStream_t st,
                           const unsigned char *pmask, int pms, int pc, int ph,
                           const ConvUpdateEpi *ue) {
  static const int enabled = KCNN_KNOB("KCNN_FUSED_BWD", 1);
  static const int variant = KCNN_KNOB("KCNN_BWD_VARIANT", 3);  // 1: register-staged
  static const int bdbg = KCNN_KNOB("KCNN_BWD_DEBUG", 0);
  if (!enabled || (dX == nullptr && gW == nullptr)) return -1;
  if (g.Kdim > 31 || g.G % 32 != 0 || g.G > 128 || g.G == 0) return -1;
  // the bf16x6 kernel (cnsl-conv-x6.hip) where the shape allows; KCNN_BWD_X6=0
  // keeps the fp32-MFMA kernels below
  if (family(kFamBwdX6) && variant == 3 && kcnn_conv_bwd_x6_eligible(g, dX != nullptr, pc, ph)) {
    const int S = (int)frame_grid(g, 1);
    const int E = (g.Kdim + 1) * g.G;
    float *part = static_cast<float *>(ws);
    if (gW != nullptr) {
      const size_t need = kcnn_conv_bwd_frame_ws(g);
      if (need == 0 || ws == nullptr || ws_bytes < need) return -1;
    }
    // The gradient's bf16-MFMA accumulation chains are kept to 16 frames per
    // workgroup: a longer chain grows its error linearly with the frames
    // (c2 stack, prev' normwise against fp64: 2.6e-6 at 4096 frames, 9.2e-6
    // at 16384, 3.8e-5 at 65536; an fp32 contraction 1.5e-6 at each;
    // experiments/diag_wgrad_acc.py).  Larger batches run as launches over
    // frame ranges of at most BWD_X6_FRAMES, each workgroup adding its range's
    // partial to its slot in fp32 (fixed order: deterministic).
    constexpr int BWD_X6_FRAMES = 4096;
    const int nch = gW != nullptr ? (g.R + BWD_X6_FRAMES - 1) / BWD_X6_FRAMES : 1;
    int rc = 0;
    for (int c = 0; c < nch && !rc; ++c) {
      const int r0 = (int)((int64_t)g.R * c / nch), r1 = (int)((int64_t)g.R * (c + 1) / nch);
      ConvGeom gc = g;
      gc.R = r1 - r0;
      gc.M = (int64_t)gc.R * g.P;
      // every range holds at least 2048 frames (nch > 1), so the same S slots
      rc = kcnn_conv_bwd_x6(gc, X ? X + (int64_t)r0 * xs : X, xs, dY + (int64_t)r0 * dys, dys,
                            K, ks, dX ? dX + (int64_t)r0 * dxs : dX, dxs, gW ? part : nullptr,
                            nch > 1 ? (int)frame_grid(gc, 1) : S, dx_acc, st,
                            pmask ? pmask + (int64_t)r0 * pms : pmask, pms, pc, ph,
                            bdbg | (c > 0 ? 1 << 30 : 0));
    }
    if (rc || gW == nullptr) return rc;
    hipLaunchKernelGGL(reduce_splits_kernel, dim3((E + 63) / 64), dim3(256), 0, st, part, S,
                       E, g.Kdim * g.G, g.G, 0, gW, gws, gb, ue ? *ue : ConvUpdateEpi{});
    return (int)hipGetLastError();
  }
  if (ph != 1) return -1;  // 3-D windows: the bf16x6 kernel only
  if (g.P < 16 || g.P > 32 * BWD_WAVES * BWD_MAXT || 8 * g.P > BWD_THREADS * BWD_MAXV)
    return -1;
  if (pc == 0 && ((uintptr_t)dY % 16 != 0 || dys % 4 != 0)) return -1;  // 16-B slab loads
  // pc = 2 would stage 16 rows per slab: past the register budget
  if (pc != 0 && (!(pc == 4 || pc == 8) || variant != 3)) return -1;
  const int S = (int)frame_grid(g, 1);
  const int E = (g.Kdim + 1) * g.G;
  const int ZZ = g.Kdim | 1;
  float *part = static_cast<float *>(ws);
  if (gW != nullptr) {
    const size_t need = kcnn_conv_bwd_frame_ws(g);
    if (need == 0 || ws == nullptr || ws_bytes < need) return -1;
  }
  // weight-gradient tiles per wave: dgrad tile T belongs to wave T % 8; the
  // wgrad tiles go to the least-loaded waves, so all waves carry the same
  // number of 16-MFMA chunks (deterministic: the same table with or without dX)
  unsigned long long wg[2] = {~0ull, ~0ull};
  {
    const int ntile = (g.P + 31) / 32;
    int load[BWD_WAVES] = {0}, nw[BWD_WAVES] = {0};
    for (int T = 0; T < ntile; T++) load[T % BWD_WAVES]++;
    for (int T = 0; T < ntile; T++) {
      int best = -1;
      for (int w = 0; w < BWD_WAVES; w++)
        if (nw[w] < 2 && (best < 0 || load[w] < load[best])) best = w;
      load[best]++;
      wg[nw[best]] &= ~(0xffull << (8 * best));
      wg[nw[best]] |= (unsigned long long)T << (8 * best);
      nw[best]++;
    }
  }
  size_t lds3 = bwd_dma_lds(g);
  // a separate Z buffer when it fits (deferred col2im, see the kernel)
  const size_t zbytes = (size_t)g.P * ZZ * 4;
  const int zsep = dX != nullptr && lds3 + zbytes <= (size_t)kBwdLdsMax &&
                   !(bdbg & 32);
  if (zsep) lds3 += zbytes;
  if (variant == 3 && g.C * g.HW <= BWD_THREADS * BWD_MAXX &&
      lds3 <= (size_t)kBwdLdsMax) {
#define KCNN_BWD3P(NCH, DXB, WGB, PCM)                                                 \
  hipLaunchKernelGGL((conv_bwd_dma_kernel<NCH, DXB, WGB, PCM>), dim3(S), dim3(BWD_THREADS), \
                     lds3, st, g, X, xs, dY, dys, K, ks, dX, dxs, part, ZZ, wg[0], wg[1], zsep, \
                     dx_acc, bdbg, pmask, pms)
#define KCNN_BWD3(NCH, DXB, WGB)                  \
  do {                                            \
    if (pc == 4) KCNN_BWD3P(NCH, DXB, WGB, 4);    \
    else if (pc == 8) KCNN_BWD3P(NCH, DXB, WGB, 8); \
    else KCNN_BWD3P(NCH, DXB, WGB, 0);            \
  } while (0)
#define KCNN_BWD3_NCH(NCH)                                  \
  do {                                                      \
    if (dX && gW) KCNN_BWD3(NCH, true, true);               \
    else if (gW) KCNN_BWD3(NCH, false, true);               \
    else KCNN_BWD3(NCH, true, false);                       \
  } while (0)
    switch (g.G / 32) {
      case 1: KCNN_BWD3_NCH(1); break;
      case 2: KCNN_BWD3_NCH(2); break;
      case 3: KCNN_BWD3_NCH(3); break;
      default: KCNN_BWD3_NCH(4); break;
    }
#undef KCNN_BWD3_NCH
#undef KCNN_BWD3
#undef KCNN_BWD3P
  } else {
    // register-staged variant: needs the gradient outputs, writes dX
    if (gW == nullptr || dx_acc || pc) return -1;
    const int SP = bwd_sp(g);
    const size_t lds = bwd_lds(g, SP);
    if (lds > (size_t)kFrameLdsMax) return -1;
    const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
    const FastDiv dhp((uint32_t)Hp), dhpwp((uint32_t)(Hp * Wp));
#define KCNN_BWD1(NCH)                                                              \
  do {                                                                              \
    if (dX)                                                                         \
      hipLaunchKernelGGL((conv_bwd_frame_kernel<NCH, true>), dim3(S), dim3(BWD_THREADS), \
                         lds, st, g, X, xs, dY, dys, K, ks, dX, dxs, part, ZZ, SP, dhp, dhpwp); \
    else                                                                            \
      hipLaunchKernelGGL((conv_bwd_frame_kernel<NCH, false>), dim3(S), dim3(BWD_THREADS), \
                         lds, st, g, X, xs, dY, dys, K, ks, dX, dxs, part, ZZ, SP, dhp, dhpwp); \
  } while (0)
    switch (g.G / 32) {
      case 1: KCNN_BWD1(1); break;
      case 2: KCNN_BWD1(2); break;
      case 3: KCNN_BWD1(3); break;
      default: KCNN_BWD1(4); break;
    }
#undef KCNN_BWD1
  }
  int rc = (int)hipGetLastError();
  if (rc || gW == nullptr) return rc;
  float *tmp = part + (size_t)S * E;
  (void)tmp;
  hipLaunchKernelGGL(reduce_splits_kernel, dim3((E + 63) / 64), dim3(256), 0, st, part, S,
                     E, g.Kdim * g.G, g.G, 0, gW, gws, gb, ue ? *ue : ConvUpdateEpi{});
  return (int)hipGetLastError();
}

// dX (nullable) and/or gW, gb (nullable) from one pass over dY.  gW == NULL
// runs the data gradient only and needs no workspace.  G > 128 (c5's
// 256-filter layers) runs in chunks of 128 filters: dY columns, W columns
// and gW/gb columns of a chunk are plain offsets into the same matrices, and
// the chunks after the first add their data gradient into dX (fixed order).
int kcnn_conv_bwd_frame(const ConvGeom &g, const float *X, int xs,
                        const float *dY, int dys, const float *K, int ks,
                        float *dX, int dxs, float *gW, int gws, float *gb,
                        void *ws, size_t ws_bytes, hipStream_t st,
                        const unsigned char *pmask, int pms, int pc, int ph) {
  // the caller's update request (conv-update.h), for this layer's W
  ConvUpdateEpi *u = kcnn_conv_update_current();
  if (u && !(gW && gb && u->Kdim == g.Kdim && u->G == g.G)) u = nullptr;
  if (g.G <= 128) {
    const int rc = bwd_frame_chunk(g, X, xs, dY, dys, K, ks, dX, dxs, gW, gws, gb, ws,
                                   ws_bytes, 0, st, pmask, pms, pc, ph, u);
    if (rc == 0 && u) u->applied = 1;
    return rc;
  }
  if (g.G % 32 != 0 || (int64_t)g.G * g.P * 4 % 16 != 0) return -1;
  static const int variant = KCNN_KNOB("KCNN_BWD_VARIANT", 3);
  if (variant != 3 && dX != nullptr) return -1;  // chunking needs dX accumulation
  for (int g0 = 0; g0 < g.G; g0 += 128) {
    ConvGeom gc = g;
    gc.G = g.G - g0 < 128 ? g.G - g0 : 128;
    // pooled rows of P / ph values when pc, masks of 1 (ph == 1) or 2 bytes
    const int64_t dofs = pc ? (int64_t)(g0 / pc) * (g.P / ph) : (int64_t)g0 * g.P;
    const int64_t mofs = dofs * (ph > 1 ? 2 : 1);
    ConvUpdateEpi uc{};
    if (u) {  // the chunk's filter columns of W, prev and b
      uc = *u;
      uc.W += g0;
      uc.prev += g0;
      uc.b += g0;
      uc.G = gc.G;
    }
    const int rc = bwd_frame_chunk(
        gc, X, xs, dY + dofs, dys, K + g0, ks, dX, dxs, gW ? gW + g0 : nullptr, gws,
        gb ? gb + g0 : nullptr, ws, ws_bytes, g0 > 0, st, pmask ? pmask + mofs : nullptr,
        pms, pc, ph, u ? &uc : nullptr);
    if (rc) {
      // only the first chunk may decline (nothing written yet); a later
      // failure is a launch error
      return g0 == 0 ? rc : (rc < 0 ? (int)hipErrorLaunchFailure : rc);
    }
  }
  if (u) u->applied = 1;
  return 0;
}

size_t kcnn_reduce_splits_ws(int S, int E) {
  return (size_t)((S + 31) / 32) * (size_t)E * 4;
}

// Generic: in [S][E] -> out (with the gW/gb mapping of the implicit-GEMM
// wgrad: e = g*Kdim + k for e < G*Kdim); tmp is unused (one pass).  The
// caller's update request for this layer's W (conv-update.h: Kdim = inner,
// G = nw / inner) is applied here instead of storing gW / gb, as the frame
// kernels' reduction does (the long-kernel weight gradients run after the
// data gradient, so W is stepped after its last read).
int kcnn_reduce_splits_wgrad(const float *in, int S, int E, float *tmp, int nw,
                             int inner, float *gW, int gws, float *gb,
                             hipStream_t st) {
  (void)tmp;
  ConvUpdateEpi *u = kcnn_conv_update_current();
  if (u && !(gW && gb && inner > 0 && u->Kdim == inner && (int64_t)u->G * inner == nw &&
             E == nw + u->G))
    u = nullptr;
  hipLaunchKernelGGL(reduce_splits_kernel, dim3((E + 63) / 64), dim3(256), 0, st, in, S, E,
                     nw, inner, 1, gW, gws, gb, u ? *u : ConvUpdateEpi{});
  const int rc = (int)hipGetLastError();
  if (rc == 0 && u) u->applied = 1;
  return rc;
}

int kcnn_reduce_splits_pass1(const float *in, int S, int E, float *tmp,
                             hipStream_t st) {
  const int Q = (S + 31) / 32;
  hipLaunchKernelGGL(reduce_pass1, dim3((E + 255) / 256, Q), dim3(256), 0, st,
                     in, S, E, tmp);
  return (int)hipGetLastError();
}

int kcnn_reduce_splits(const float *in, int S, int E, float *tmp, float *out,
                       hipStream_t st) {
  (void)tmp;
  hipLaunchKernelGGL(reduce_splits_kernel, dim3((E + 63) / 64), dim3(256), 0, st, in, S, E,
                     E, E, 0, out, 0, nullptr, ConvUpdateEpi{});
  return (int)hipGetLastError();
}
