// cnslmat/cnsl-conv-mfma.hip -- convolution on gfx950 matrix cores.
//
// CuMatrixBase::Conv2D (conv2D.cc:43-201) materialises an im2col matrix
// ("spanThis", up to 0.5 GB per split), runs cuBLAS sgemm into a zero-filled
// temporary, copies it into a second temporary and finally col2im's it into
// `out` (four launches, ~10x the compulsory HBM traffic).  Here the same
// contraction is one implicit GEMM:
//
//   D[g][m] = sum_k K[k][g] * B[k][m],     m = n*P + p   (sample-major),
//   B[k][m] = X[n][c*H*W + (px+kx-pad_w)*H + (py+ky-pad_h)]  (0 outside),
//   k = c*kh*kw + kx*kh + ky,  p = px*oh + py                
//
// on v_mfma_f32_32x32x2_f32 (exact fp32, fma-chain numerics): the B tile is
// gathered straight from X (L1/L2-resident rows) into LDS, the kernel tile is
// staged beside it, and the accumulator is stored directly in the reference's
// output layout -- concat: out[n][g*P + p] with lanes along p (two 128-B
// segments per store), or plain: out[p*R + n][g] -- with the bias add of
// AddMatRepVec fused.  Virtual zero padding replaces PaddingZero.  Long
// reductions split K across workgroups into a workspace and are reduced in a
// fixed order (deterministic).
//
// Small output-channel counts (the data gradient of a 1- or 3-channel input
// layer: G' = C) use a direct VALU kernel instead: an MFMA tile would be
// >= 80 % padding there.
//
// The weight gradient of ConvolutionComponent::Update gets its own fused
// kernel (TpBlock + TpInsideBlock + Conv2D + ModPermuteRow + AddRowSumMat,
// nnet-component-nnet0.cc:745-775) reading X and dY once each.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "conv-geom.h"

using kcnn::FastDiv;
using kcnn::ConvGeom;
using kcnn::floatx16;
using kcnn::make_geom;

namespace {

// Input element of im2col row k for output position (px, py) of one sample.
__device__ __forceinline__ float gather_x(const ConvGeom &g,
                                          const float *__restrict__ xrow,
                                          int k, int px, int py) {
  uint32_t c, r, kx, ky;
  g.div_khkw.divmod((uint32_t)k, c, r);
  g.div_kh.divmod(r, kx, ky);
  const int xx = px + (int)kx - g.pad_w, yy = py + (int)ky - g.pad_h;
  if (xx < 0 || xx >= g.W || yy < 0 || yy >= g.H) return 0.0f;
  return xrow[(int64_t)c * g.HW + (int64_t)xx * g.H + yy];
}

// ---------------------------------------------------------------------------
// Implicit-GEMM kernel: block tile 64 (g) x 64 (m), K step 16, 4 waves each
// owning one 32x32 MFMA accumulator.
constexpr int IG_BG = 64, IG_BM = 64, IG_BK = 16;
enum { ST_CONCAT = 0, ST_PLAIN = 1, ST_PARTIAL = 2 };

template <int STORE>
__global__ __launch_bounds__(256) void conv_igemm_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ Kmat, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os, float *__restrict__ ws, int k_per_split) {
  __shared__ float As[IG_BK][IG_BG];
  __shared__ float Bs[IG_BK][IG_BM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = wave & 1, wm = wave >> 1;
  const int64_t m0 = (int64_t)blockIdx.x * IG_BM;
  const int g0 = blockIdx.y * IG_BG;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(g.Kdim, kbeg + k_per_split);

  // This thread's B column (fixed over the K loop).
  const int bm = tid & 63, bk = tid >> 6;
  const int64_t m = m0 + bm;
  const bool mvalid = m < g.M;
  uint32_t n = 0, p = 0, px = 0, py = 0;
  if (mvalid) {
    g.div_P.divmod((uint32_t)m, n, p);
    g.div_oh.divmod(p, px, py);
  }
  const float *xrow = X + (int64_t)n * xs;
  const int ak = tid >> 4, ag = (tid & 15) * 4;

  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;

  for (int k0 = kbeg; k0 < kend; k0 += IG_BK) {
    {
      const int kk = k0 + ak;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int gg = g0 + ag + j;
        As[ak][ag + j] =
            (kk < kend && gg < g.G) ? Kmat[(int64_t)kk * ks + gg] : 0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int kk = k0 + bk + 4 * j;
      Bs[bk + 4 * j][bm] = (mvalid && kk < kend)
                               ? gather_x(g, xrow, kk, (int)px, (int)py)
                               : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < IG_BK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wg * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue.  D[i][j]: j = lane & 31 (m), i = (r&3) + 8(r>>2) + 4(lane>>5) (g).
  const int64_t mm = m0 + wm * 32 + (lane & 31);
  if (mm >= g.M) return;
  uint32_t on, op;
  g.div_P.divmod((uint32_t)mm, on, op);
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int gg = g0 + wg * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (gg >= g.G) continue;
    float v = acc[r];
    if (STORE == ST_CONCAT) {
      if (bias) v = v + bias[gg];
      out[(int64_t)on * os + (int64_t)gg * g.P + op] = v;
    } else if (STORE == ST_PLAIN) {
      out[((int64_t)op * g.R + on) * os + gg] = v;
    } else {
      ws[((int64_t)blockIdx.z * g.G + gg) * g.M + mm] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Implicit GEMM, variant 2 (large kernel volumes: c5 C2-C4, the flipped-
// kernel data gradient).  out[g][m] = sum_k W[k][g] im2col(X)[k][m] with
// m = n*P + p.  Block = 4 waves, each owning a 64 (g) x 64 (m) block of four
// 32x32 accumulators; WGG waves along g (tile 64*WGG x 64*(4/WGG)).  K steps
// of 16 are double-buffered in LDS with one barrier per step; the next
// step's operands are in flight (registers) while the current one runs.
//   * VALU work is budgeted: on gfx950 it does not execute beside the fp32
//     MFMAs, so every VALU op is MFMA idle time.  The im2col row offset of
//     k (c*H*W + kx*H + ky) and the tap are wave-uniform (scalar ALU); per
//     gathered element one add builds the offset, and for padded maps a
//     per-lane bitmask of the taps that fall inside the map (kh*kw <= 32)
//     drops the others (buffer loads make any stray offset safe).
//   * Operands per MFMA: one LDS read (A: W tile, B: im2col tile).
constexpr int IG2_KTAB = 2304;  // im2col-row table entries (c5 C3: Kdim 2304)

// flags bit: RectifiedLinearComponent's Propagate in the epilogue (the other
// bits are timing switches of the phase-timing build)
constexpr int kIg2Relu = 1 << 16;

template <int WGG, bool PADDED, int IG2_BK, bool TAB>
__global__ __launch_bounds__(256) void conv_igemm2_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ Kmat,
    int ks, const float *__restrict__ bias, float *__restrict__ out, int os, int dbg) {
  constexpr int WGM = 4 / WGG;
  constexpr int BG = 64 * WGG, BM = 64 * WGM;
  constexpr int ANF = IG2_BK * BG / 256;  // A floats per thread per K step (4 or 8)
  constexpr int BNF = IG2_BK * BM / 256;  // B floats per thread per K step (8 or 16)
  __shared__ __attribute__((aligned(16))) float As[2][IG2_BK][BG];
  __shared__ __attribute__((aligned(16))) float Bs[2][IG2_BK][BM];
  // TAB: per im2col row k its map offset (bytes) and tap, stored per
  // row-parity class [k % B_RSTEP][k / B_RSTEP] so that a thread's BNF rows
  // of one K step are consecutive (16-B LDS reads, wave-uniform address).
  __shared__ __attribute__((aligned(16))) unsigned ktab_off[TAB ? IG2_KTAB : 1];
  __shared__ __attribute__((aligned(16))) unsigned ktab_tap[TAB && PADDED ? IG2_KTAB : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = wave % WGG, wm = wave / WGG;
  const int l = lane & 31, h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int g0 = blockIdx.y * BG;
  const int nk = (g.Kdim + IG2_BK - 1) / IG2_BK;

  // A (W rows, float4 along g): thread -> (row ar + 16/ANF*i?, cols ag..ag+3)
  constexpr int A_TPR = BG / 4;            // threads per A row
  const int ar = tid / A_TPR, ag = (tid % A_TPR) * 4;  // rows ar, ar + 256/A_TPR
  constexpr int A_RSTEP = 256 / A_TPR;
  // B (im2col): thread's column m, rows br + B_RSTEP * j (br wave-uniform)
  const int bm = tid % BM;
  const int br = __builtin_amdgcn_readfirstlane(tid / BM);
  constexpr int B_RSTEP = 256 / BM;
  const int64_t mcol = m0 + bm;
  const bool mvalid = mcol < g.M;
  int xoff = 0;                  // frame row + (px, py) part of the offset
  unsigned tapmask = 0xffffffffu;  // taps inside the map (PADDED)
  {
    uint32_t n = 0, p = 0, px = 0, py = 0;
    if (mvalid) {
      g.div_P.divmod((uint32_t)mcol, n, p);
      g.div_oh.divmod(p, px, py);
    }
    xoff = (int)n * xs + ((int)px - g.pad_w) * g.H + (int)py - g.pad_h;
    if (PADDED) {
      tapmask = 0;
      for (int kx = 0; kx < g.kw; kx++)
        for (int ky = 0; ky < g.kh; ky++) {
          const int xx = (int)px + kx - g.pad_w, yy = (int)py + ky - g.pad_h;
          if ((unsigned)xx < (unsigned)g.W && (unsigned)yy < (unsigned)g.H)
            tapmask |= 1u << (kx * g.kh + ky);
        }
    }
    if (!mvalid) tapmask = 0;
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)X, (short)0,
      (dbg & 4) ? 0 : (int)((int64_t)g.R * xs * 4 < 0x7fffffff ? (int64_t)g.R * xs * 4 : 0x7fffffff),
      0x00020000);  // dbg & 4: zero records (timing: same instructions, no traffic)

  // W rows through a descriptor too: rows past Kdim read 0 (range check)
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)Kmat, (short)0, (dbg & 8) ? 0 : g.Kdim * ks * 4, 0x00020000);
  if (!PADDED) tapmask = mvalid ? 0xffffffffu : 0u;
  // TAB: rows past Kdim have tap 31, which no lane's mask admits (kh*kw <= 31)
  const unsigned nmask = PADDED ? ~(tapmask & 0x7fffffffu) : 0u;
  const unsigned xoff4 = (unsigned)xoff * 4u;
  const int kq = (nk * IG2_BK) / B_RSTEP;  // table entries per parity class
  if (TAB) {
    for (int k = tid; k < nk * IG2_BK; k += 256) {
      uint32_t c = 0, r = 0, kx = 0, ky = 0;
      if (k < g.Kdim) {
        g.div_khkw.divmod((uint32_t)k, c, r);
        g.div_kh.divmod(r, kx, ky);
      }
      const int slot = (k % B_RSTEP) * kq + k / B_RSTEP;
      ktab_off[slot] = k < g.Kdim
                           ? (unsigned)(((int)c * g.HW + (int)kx * g.H + (int)ky) * 4)
                           : (PADDED ? 0u : 0x80000000u);
      if (PADDED) ktab_tap[slot] = k < g.Kdim ? kx * (uint32_t)g.kh + ky : 31u;
    }
    __syncthreads();
  }
  float4 areg[ANF / 4];
  float breg[BNF];
  unsigned bok = 0;  // bit j: element j of breg is inside the map
  // branch-free: every load issues back to back; nothing reads a loaded
  // value before store(), so the loads land while the MFMAs run
  auto load = [&](int kt) {
    if (dbg & 1) return;  // timing experiments: no operand loads
    const int kb = kt * IG2_BK;
#pragma unroll
    for (int i = 0; i < ANF / 4; i++) {
      const int k = kb + ar + A_RSTEP * i;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(
          wr, (unsigned)(k * ks + g0 + ag) * 4u, 0, 0);
      areg[i] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]),
                            __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
    if (TAB) {
      // one add per element; padded maps: the tap's bit of this lane's
      // outside-mask moves the offset out of range (the load returns 0)
      const int t0 = br * kq + kb / B_RSTEP;
#pragma unroll
      for (int q = 0; q < BNF / 4; q++) {
        const uint4 ko = *reinterpret_cast<const uint4 *>(&ktab_off[t0 + 4 * q]);
        uint4 kt = make_uint4(0, 0, 0, 0);
        if (PADDED) kt = *reinterpret_cast<const uint4 *>(&ktab_tap[t0 + 4 * q]);
        const unsigned kov[4] = {ko.x, ko.y, ko.z, ko.w};
        const unsigned ktv[4] = {kt.x, kt.y, kt.z, kt.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          unsigned off = xoff4 + kov[e];
          if (PADDED) off |= ((nmask >> ktv[e]) & 1u) << 31;
          breg[4 * q + e] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < BNF; j++) {
      const int k = kb + br + B_RSTEP * j;  // wave-uniform: scalar index math
      const int kc = k < g.Kdim ? k : g.Kdim - 1;
      uint32_t c, r, kx, ky;
      g.div_khkw.divmod((uint32_t)kc, c, r);
      g.div_kh.divmod(r, kx, ky);
      const int koff = (int)c * g.HW + (int)kx * g.H + (int)ky;
      const int tap = (int)(kx * g.kh + ky);
      const unsigned vm = k < g.Kdim ? tapmask : 0u;
      breg[j] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(xr, (unsigned)(xoff + koff) * 4u, 0, 0));
      bok = j == 0 ? ((vm >> tap) & 1u) : bok | (((vm >> tap) & 1u) << j);
    }
  };
  auto store = [&](int b) {
    if (dbg & 2) return;  // timing experiments: no LDS stores
#pragma unroll
    for (int i = 0; i < ANF / 4; i++)
      *reinterpret_cast<float4 *>(&As[b][ar + A_RSTEP * i][ag]) = areg[i];
#pragma unroll
    for (int j = 0; j < BNF; j++)
      Bs[b][br + B_RSTEP * j][bm] = (TAB || ((bok >> j) & 1u)) ? breg[j] : 0.0f;
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[a][b][i] = 0.0f;

  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; kt++) {
    if (kt + 1 < nk) load(kt + 1);
#pragma unroll
    for (int s = 0; s < IG2_BK / 2; s++) {
      const float a0 = As[cur][2 * s + h][wg * 64 + l];
      const float a1 = As[cur][2 * s + h][wg * 64 + 32 + l];
      const float b0 = Bs[cur][2 * s + h][wm * 64 + l];
      const float b1 = Bs[cur][2 * s + h][wm * 64 + 32 + l];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // Epilogue: D[g][m], row (r&3) + 8(r>>2) + 4h, column l (concat layout).
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int64_t mm = m0 + wm * 64 + 32 * b + l;
    if (mm >= g.M) continue;
    uint32_t on, op;
    g.div_P.divmod((uint32_t)mm, on, op);
    float *orow = out + (int64_t)on * os + op;
#pragma unroll
    for (int a = 0; a < 2; a++) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int gg = g0 + wg * 64 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gg >= g.G) continue;
        float v = acc[a][b][r];
        if (bias) v = v + bias[gg];
        if (dbg & kIg2Relu) v = v < 0.0f ? 0.0f : v;  // ApplyFloor(0)
        orow[(int64_t)gg * g.P] = v;
      }
    }
  }
}

// Fixed-order reduction of split-K partials [S][G][M] + the store epilogue.// Fixed-order reduction of split-K partials [S][G][M] + the store epilogue.
__global__ __launch_bounds__(256) void conv_splitk_reduce_kernel(
    ConvGeom g, const float *__restrict__ ws, int S,
    const float *__restrict__ bias, float *__restrict__ out, int os,
    int concat) {
  const int64_t total = (int64_t)g.G * g.M;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int gg = (int)(e / g.M);
    const int64_t mm = e - (int64_t)gg * g.M;
    float outer = 0.0f;
    for (int s0 = 0; s0 < S; s0 += 32) {  // two-level: error ~ sqrt(32)+sqrt(S/32)
      float inner = 0.0f;
      const int s1 = min(S, s0 + 32);
      for (int s = s0; s < s1; s++) inner += ws[((int64_t)s * g.G + gg) * g.M + mm];
      outer += inner;
    }
    uint32_t on, op;
    g.div_P.divmod((uint32_t)mm, on, op);
    if (concat) {
      if (bias) outer = outer + bias[gg];
      out[(int64_t)on * os + (int64_t)gg * g.P + op] = outer;
    } else {
      out[((int64_t)op * g.R + on) * os + gg] = outer;
    }
  }
}

// ---------------------------------------------------------------------------
// Direct kernel for few output channels (G <= NG): thread per output
// position, sequential k loop (same order as the reference GEMM's k), the
// kernel row read through the scalar cache (k is wave-uniform).
template <int NG>
__global__ __launch_bounds__(256) void conv_direct_smallg_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ Kmat, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= g.M) return;
  uint32_t n, p, px, py;
  g.div_P.divmod((uint32_t)m, n, p);
  g.div_oh.divmod(p, px, py);
  const float *xrow = X + (int64_t)n * xs;
  float acc[NG];
#pragma unroll
  for (int j = 0; j < NG; j++) acc[j] = 0.0f;
  int k = 0;
  for (int c = 0; c < g.C; c++) {
    const float *xc = xrow + (int64_t)c * g.HW;
    for (int kx = 0; kx < g.kw; kx++) {
      const int xx = (int)px + kx - g.pad_w;
      const bool vx = xx >= 0 && xx < g.W;
      const float *xcol = xc + (int64_t)xx * g.H;
      for (int ky = 0; ky < g.kh; ky++, k++) {
        const int yy = (int)py + ky - g.pad_h;
        const float xv = (vx && yy >= 0 && yy < g.H) ? xcol[yy] : 0.0f;
        const float *krow = Kmat + (int64_t)k * ks;
#pragma unroll
        for (int j = 0; j < NG; j++)
          if (j < g.G) acc[j] += xv * krow[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NG; j++)
    if (j < g.G) {
      float v = acc[j];
      if (bias) v = v + bias[j];
      out[(int64_t)n * os + (int64_t)j * g.P + p] = v;
    }
}

// ---------------------------------------------------------------------------
// Fused weight gradient.  D[g][k] = sum_t dY[n][g*P + p] * B[t][k] over
// t = n*P + p in this block's split; block tile 64 (g) x 64 (k), t step 32.
constexpr int WG_BG = 64, WG_BK = 64, WG_BT = 32;

__global__ __launch_bounds__(256) void conv_wgrad_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ dY, int dys, float *__restrict__ ws_w,
    float *__restrict__ ws_b, int64_t t_per_split) {
  __shared__ float As[WG_BT][WG_BG + 1];  // dY tile, [t][g]
  __shared__ float Bs[WG_BT][WG_BK];      // im2col tile, [t][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = wave & 1, wk = wave >> 1;
  const int split = blockIdx.x;
  const int g0 = blockIdx.y * WG_BG, k0 = blockIdx.z * WG_BK;
  const int64_t T = g.M;
  const int64_t tbeg = (int64_t)split * t_per_split;
  const int64_t tend = min(T, tbeg + t_per_split);

  // B: this thread's conv-k column.
  const int bk = tid & 63, bt = tid >> 6;
  const int kk = k0 + bk;
  const bool kvalid = kk < g.Kdim;
  int koff = 0, kx = 0, ky = 0;
  if (kvalid) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)kk, c, r);
    g.div_kh.divmod(r, qx, qy);
    kx = (int)qx; ky = (int)qy;
    koff = (int)c * g.HW;
  }
  // A: this thread's g row and 8 consecutive t.
  const int ag = tid >> 2, at = (tid & 3) * 8;
  const int agg = g0 + ag;

  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;
  float bsum = 0.0f;

  for (int64_t t0 = tbeg; t0 < tend; t0 += WG_BT) {
    {
      int64_t t = t0 + at;
      uint32_t n = 0, p = 0;
      if (t < tend) g.div_P.divmod((uint32_t)t, n, p);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        float v = 0.0f;
        if (t + i < tend && agg < g.G)
          v = dY[(int64_t)n * dys + (int64_t)agg * g.P + p];
        As[at + i][ag] = v;
        if (++p == (uint32_t)g.P) { p = 0; ++n; }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int64_t t = t0 + bt + 4 * j;
      float v = 0.0f;
      if (kvalid && t < tend) {
        uint32_t n, p, px, py;
        g.div_P.divmod((uint32_t)t, n, p);
        g.div_oh.divmod(p, px, py);
        const int xx = (int)px + kx - g.pad_w, yy = (int)py + ky - g.pad_h;
        if (xx >= 0 && xx < g.W && yy >= 0 && yy < g.H)
          v = X[(int64_t)n * xs + koff + (int64_t)xx * g.H + yy];
      }
      Bs[bt + 4 * j][bk] = v;
    }
    __syncthreads();
    if (blockIdx.z == 0 && tid < 64) {
#pragma unroll 8
      for (int i = 0; i < WG_BT; i++) bsum += As[i][tid];
    }
#pragma unroll
    for (int i = 0; i < WG_BT; i += 2) {
      const float a = As[i + (lane >> 5)][wg * 32 + (lane & 31)];
      const float b = Bs[i + (lane >> 5)][wk * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // partial row of this split: [G*Kdim (e = g*Kdim + k) | G (bias)]
  const int64_t E = (int64_t)g.G * g.Kdim + g.G;
  const int kl = k0 + wk * 32 + (lane & 31);
  if (kl < g.Kdim) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int gl = g0 + wg * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (gl < g.G) ws_w[split * E + (int64_t)gl * g.Kdim + kl] = acc[r];
    }
  }
  if (blockIdx.z == 0 && tid < 64 && g0 + tid < g.G)
    ws_b[split * E + g0 + tid] = bsum;
}

// ---------------------------------------------------------------------------
// Weight gradient v2, for long kernels (c5 C2-C4, nnet.config layer 1):
//   D[g][k] = sum_t dY[n][g*P + p] * B[t][k],   t = (n, p) over the block's
//   frames, B = im2col(X) (Appendix A.12), block tile 128 (g) x 128 (k),
//   each wave 64 x 64 (four 32x32 accumulators) as in conv_igemm2_kernel.
// The reduction walks the block's frames in chunks of bt <= 32 positions
// (P split evenly, so no k-step multiplies padding), and lane tl of every
// chunk always stands for the same position (p = bt*c + tl, or frame offset
// tl / P and p = tl % P when P <= 16).  Its map offset and its
// tap-validity mask are therefore computed once; per step only the frame
// base moves, and that lives in the (scalar) buffer descriptors, whose range
// also drops the frames past the split.  Per gathered X element: one add
// for the offset and two ops for the tap mask (padded maps only); per dY
// element one add.  Steps are double-buffered in LDS, one barrier each.
// Bias gradient: the k-tile-0 blocks also sum their dY values (fixed order).
// A last, partial filter tile reads rows past G (the next frame's values, or
// zeros past the descriptor's range): they only reach accumulator rows that
// are never stored.
// Partials go to ws[split][e] (e = g*Kdim + k, then G bias entries) and are
// reduced in a fixed order (kcnn_reduce_splits_wgrad): deterministic.
constexpr int W2_BG = 128, W2_BK = 128, W2_LD = 129;

template <int NCH, bool PADDED>
__global__ __launch_bounds__(256, 2) void conv_wgrad2_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dY,
    int dys, float *__restrict__ ws, int fps, int fpc, int bt, int ktiles, int nblocks) {
  __shared__ float As[2][32][W2_LD];  // dY tile [t][g]
  __shared__ float Bs[2][32][W2_LD];  // im2col tile [t][k]
  // XCD-aware order: hardware places block b on XCD b % 8; logical ids are
  // contiguous per XCD, so the tiles of one split (same frames) share an L2.
  const int nb8 = (nblocks + 7) >> 3;
  const int bid = (int)(blockIdx.x & 7) * nb8 + (int)(blockIdx.x >> 3);
  if (bid >= nblocks) return;
  const int ntiles = ktiles * ((g.G + W2_BG - 1) / W2_BG);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int k0 = (tile % ktiles) * W2_BK, g0 = (tile / ktiles) * W2_BG;
  const int nbeg = split * fps;
  const int nend = min(g.R, nbeg + fps);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = wave & 1, wk = wave >> 1;
  const int l = lane & 31, h = lane >> 5;
  const int tl = tid & 31, rs = tid >> 5;  // t-lane; row sub-index 0..7

  // This thread's im2col columns k = k0 + rs + 8j (fixed for the kernel).
  unsigned koff4[16];
  uint32_t tapj[PADDED ? 16 : 1];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int k = k0 + rs + 8 * j;
    uint32_t c = 0, r = 0, kx = 0, ky = 0;
    if (k < g.Kdim) {
      g.div_khkw.divmod((uint32_t)k, c, r);
      g.div_kh.divmod(r, kx, ky);
    }
    koff4[j] = k < g.Kdim ? (unsigned)(((int)c * g.HW + (int)kx * g.H + (int)ky) * 4)
                          : 0x40000000u;
    if (PADDED) tapj[j] = (kx << 8) | ky;
  }
  // This lane's position in each chunk; bad[c] bit j: column j's tap falls
  // outside the map at this position (padded maps).
  unsigned voffA[NCH], lpos4[NCH], bad[NCH];
#pragma unroll
  for (int c = 0; c < NCH; c++) {
    int fo = 0, p = bt * c + tl;
    if (fpc > 1) { fo = tl / g.P; p = tl - fo * g.P; }
    const bool valid = tl < bt && (fpc > 1 ? fo < fpc : p < g.P);
    uint32_t px = 0, py = 0;
    if (valid) g.div_oh.divmod((uint32_t)p, px, py);
    voffA[c] = valid ? (unsigned)((fo * dys + rs * g.P + p) * 4) : 0x80000000u;
    const int lp = fo * xs + ((int)px - g.pad_w) * g.H + (int)py - g.pad_h;
    lpos4[c] = valid ? (unsigned)(lp * 4) : 0x40000000u;
    unsigned b = 0;
    if (PADDED) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int xx = (int)px + (int)(tapj[j] >> 8) - g.pad_w;
        const int yy = (int)py + (int)(tapj[j] & 255) - g.pad_h;
        if ((unsigned)xx >= (unsigned)g.W || (unsigned)yy >= (unsigned)g.H) b |= 1u << j;
      }
    }
    bad[c] = b;
  }

  float areg[16], breg[16], bacc[16];
#pragma unroll
  for (int j = 0; j < 16; j++) bacc[j] = 0.0f;
  const bool do_bias = k0 == 0;
  // dY row offsets are wave-uniform: they go in soffset (valid lanes stay
  // inside the descriptor's range, masked lanes' voffset alone exceeds it).
  const unsigned gstep4 = (unsigned)(8 * g.P * 4), gbase4 = (unsigned)(g0 * g.P * 4);

  // All loads issue back to back; nothing reads them before store().
  auto load = [&](int n, int c) {
    const int nf = min(fpc, nend - n);
    const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dY + (int64_t)n * dys), (short)0, nf * dys * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + (int64_t)n * xs), (short)0, nf * xs * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < 16; j++)
      areg[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          ar, voffA[c], (int)(gbase4 + gstep4 * j), 0));  // row part: soffset
#pragma unroll
    for (int j = 0; j < 16; j++) {
      unsigned off = lpos4[c] + koff4[j];
      if (PADDED) off |= ((bad[c] >> j) & 1u) << 31;
      breg[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, off, 0, 0));
    }
  };
  auto store = [&](int b) {
#pragma unroll
    for (int j = 0; j < 16; j++) As[b][tl][rs + 8 * j] = areg[j];
#pragma unroll
    for (int j = 0; j < 16; j++) Bs[b][tl][rs + 8 * j] = breg[j];
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 16; j++) bacc[j] += areg[j];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[a][b][i] = 0.0f;

  load(nbeg, 0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int n = nbeg; n < nend; n += fpc) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const bool more = c + 1 < NCH || n + fpc < nend;
      if (more) load(c + 1 < NCH ? n : n + fpc, c + 1 < NCH ? c + 1 : 0);
#pragma unroll
      for (int s = 0; s < 16; s++) {
        if (2 * s >= bt) break;  // chunk length bt (uniform): no padded k-steps
        const float a0 = As[cur][2 * s + h][wg * 64 + l];
        const float a1 = As[cur][2 * s + h][wg * 64 + 32 + l];
        const float b0 = Bs[cur][2 * s + h][wk * 64 + l];
        const float b1 = Bs[cur][2 * s + h][wk * 64 + 32 + l];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
      if (more) store(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // Partials of this split: weights (lanes along k: 128-B runs), bias.
  const int64_t E = (int64_t)g.G * g.Kdim + g.G;
  float *wsp = ws + (int64_t)split * E;
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int kk = k0 + wk * 64 + 32 * b + l;
    if (kk >= g.Kdim) continue;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int gg = g0 + wg * 64 + 32 * a + kcnn::mfma32_row(r, lane);
        if (gg < g.G) wsp[(int64_t)gg * g.Kdim + kk] = acc[a][b][r];
      }
  }
  if (do_bias) {
    float *red = &As[0][0][0];  // [128][33]
#pragma unroll
    for (int j = 0; j < 16; j++) red[(rs + 8 * j) * 33 + tl] = bacc[j];
    __syncthreads();
    if (tid < W2_BG) {
      float s = 0.0f;
      for (int i = 0; i < 32; i++) s += red[tid * 33 + i];
      if (g0 + tid < g.G) wsp[(int64_t)g.G * g.Kdim + g0 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Data gradient, scatter form (maps much larger than the output: c5 C2/C4).
// The flipped-kernel gather (the reference's flip branch) multiplies every
// input position by every tap, valid or not: at c5 C2 only P*khkw of
// HW*khkw pairs (59 %) are real, at C4 19 %.  Here the contraction over the
// filters runs once per (output position, kernel row) -- a 1x1 convolution
// of dY with W^T on the implicit-GEMM kernel, Z[n][k*P + p] -- and
// conv_col2im_kernel adds the kh*kw taps of each input position:
//   dX[n][c*HW + x*H + y] = sum_{kx,ky valid} Z[n][(c*khkw + kx*kh + ky)*P
//                                                  + (x-kx+pad_w)*oh + (y-ky+pad_h)]
// (Appendix A.11's sum, grouped by tap).
__global__ __launch_bounds__(256) void conv_transpose_kernel(
    const float *__restrict__ in, int rows, int cols, int is,
    float *__restrict__ out, int os) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)rows * cols) return;
  const int r = (int)(e / cols), c = (int)(e - (int64_t)r * cols);
  out[(int64_t)c * os + r] = in[(int64_t)r * is + c];
}

__global__ __launch_bounds__(256) void conv_col2im_kernel(
    ConvGeom g, const float *__restrict__ Z, int zs, float *__restrict__ dX,
    int dxs) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)g.C * g.HW;
  if (e >= (int64_t)g.R * per) return;
  const int n = (int)(e / per);
  const uint32_t rem = (uint32_t)(e - (int64_t)n * per);
  uint32_t c, q, x, y;
  g.div_HW.divmod(rem, c, q);
  g.div_H.divmod(q, x, y);
  const float *zr = Z + (int64_t)n * zs + (int64_t)c * g.kh * g.kw * g.P;
  // only the taps whose output position exists: px = x + pad_w - kx in
  // [0, ow), py = y + pad_h - ky in [0, oh)
  const int tx = (int)x + g.pad_w, ty = (int)y + g.pad_h;
  const int kx0 = max(0, tx - g.ow + 1), kx1 = min(g.kw - 1, tx);
  const int ky0 = max(0, ty - g.oh + 1), ky1 = min(g.kh - 1, ty);
  float sum = 0.0f;
  for (int kx = kx0; kx <= kx1; kx++)
    for (int ky = ky0; ky <= ky1; ky++)
      sum += zr[(int64_t)(kx * g.kh + ky) * g.P + (tx - kx) * g.oh + (ty - ky)];
  dX[(int64_t)n * dxs + rem] = sum;
}

// col2im, one wave per (frame, input channel): the channel's kh*kw*P values
// of Z are one contiguous run (16-B coalesced into LDS), its H*W outputs
// another; the tap gathers happen in LDS.  Same sums, same order as
// conv_col2im_kernel.
__global__ __launch_bounds__(64) void conv_col2im_plane_kernel(
    ConvGeom g, const float *__restrict__ Z, int zs, float *__restrict__ dX, int dxs,
    int vec) {
  extern __shared__ __attribute__((aligned(16))) float zp[];
  const int lane = threadIdx.x;
  const int U = g.kh * g.kw * g.P;
  const int units = g.R * g.C;
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int n = u / g.C, c = u - n * g.C;
    const float *src = Z + (int64_t)n * zs + (int64_t)c * U;
    if (vec & 2) {  // streaming loads: Z was just written and is read once
      typedef float f4 __attribute__((ext_vector_type(4)));
      for (int i = lane; i < U / 4; i += 64)
        reinterpret_cast<f4 *>(zp)[i] =
            __builtin_nontemporal_load(reinterpret_cast<const f4 *>(src) + i);
    } else if (vec) {
      for (int i = lane; i < U / 4; i += 64)
        reinterpret_cast<float4 *>(zp)[i] = reinterpret_cast<const float4 *>(src)[i];
    } else {
      for (int i = lane; i < U; i += 64) zp[i] = src[i];
    }
    __syncthreads();
    float *dst = dX + (int64_t)n * dxs + (int64_t)c * g.HW;
    for (int qd = lane; qd < g.HW; qd += 64) {
      uint32_t x, y;
      g.div_H.divmod((uint32_t)qd, x, y);
      const int tx = (int)x + g.pad_w, ty = (int)y + g.pad_h;
      const int kx0 = max(0, tx - g.ow + 1), kx1 = min(g.kw - 1, tx);
      const int ky0 = max(0, ty - g.oh + 1), ky1 = min(g.kh - 1, ty);
      float sum = 0.0f;
      for (int kx = kx0; kx <= kx1; kx++)
        for (int ky = ky0; ky <= ky1; ky++)
          sum += zp[(kx * g.kh + ky) * g.P + (tx - kx) * g.oh + (ty - ky)];
      dst[qd] = sum;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Host-side planning.
struct IgemmPlan {
  int S, k_per_split;
  size_t ws_bytes;
};

IgemmPlan plan_igemm(const ConvGeom &g) {
  IgemmPlan pl;
  const int64_t tiles = ((g.M + IG_BM - 1) / IG_BM) * ((g.G + IG_BG - 1) / IG_BG);
  int S = 1;
  if (tiles < 1024 && g.Kdim > 8 * IG_BK) {
    int64_t want = (2048 + tiles - 1) / tiles;
    int64_t maxs = (g.Kdim + 4 * IG_BK - 1) / (4 * IG_BK);
    S = (int)(want < maxs ? want : maxs);
    if (S < 1) S = 1;
  }
  int kps = (g.Kdim + S - 1) / S;
  kps = (kps + IG_BK - 1) / IG_BK * IG_BK;
  S = (g.Kdim + kps - 1) / kps;
  pl.S = S;
  pl.k_per_split = kps;
  pl.ws_bytes = S > 1 ? (size_t)S * g.G * g.M * sizeof(float) +
                            kcnn_reduce_splits_ws(S, (int)(g.G * g.M))
                      : 0;
  return pl;
}

bool use_direct(const ConvGeom &g, int concat) { return concat && g.G <= 8; }

struct WgradPlan {
  int S;
  int64_t t_per_split;
  size_t ws_bytes;
};

WgradPlan plan_wgrad(const ConvGeom &g) {
  WgradPlan pl;
  const int64_t T = g.M;
  const int gk_tiles = ((g.G + WG_BG - 1) / WG_BG) * ((g.Kdim + WG_BK - 1) / WG_BK);
  int64_t tps = 1024;  // 32 t-steps per block: fp32 chain error ~ sqrt(1024) eps
  int64_t S = (T + tps - 1) / tps;
  const int64_t max_blocks = 16384;
  if (S * gk_tiles > max_blocks) {
    S = max_blocks / gk_tiles;
    if (S < 1) S = 1;
    tps = (T + S - 1) / S;
    tps = (tps + WG_BT - 1) / WG_BT * WG_BT;
    S = (T + tps - 1) / tps;
  }
  if (S < 1) S = 1;
  pl.S = (int)S;
  pl.t_per_split = tps;
  const size_t E = (size_t)g.G * g.Kdim + g.G;
  pl.ws_bytes = (size_t)S * E * sizeof(float) + kcnn_reduce_splits_ws((int)S, (int)E);
  return pl;
}

struct Wgrad2Plan {
  int S, fps, fpc, nch, bt, ktiles, nblocks;
  size_t ws_bytes;
};

// conv_wgrad2_kernel eligibility and split.  Splits are whole frame ranges;
// S keeps each accumulator chain <= ~8192 terms (fp32 chain error) and is
// picked so that the blocks fill whole rounds of 512 (2 per CU).
bool plan_wgrad2(const ConvGeom &g, int xs, int dys, Wgrad2Plan &pl) {
  static const int enabled = KCNN_KNOB("KCNN_WGRAD2", 1);
  if (!enabled || g.R <= 0 || g.G < 32 || g.P > 96 || g.Kdim < 32)
    return false;
  pl.fpc = g.P <= 16 ? 32 / g.P : 1;
  pl.nch = g.P <= 32 ? 1 : (g.P + 31) / 32;
  // positions per chunk: P split evenly (c5 P = 72 -> 3 x 24), even for the
  // MFMA's k-pairs; lanes past bt load nothing and feed no MFMA
  pl.bt = g.P <= 16 ? pl.fpc * g.P : (g.P + pl.nch - 1) / pl.nch;
  pl.bt = (pl.bt + 1) & ~1;
  if ((int64_t)pl.fpc * xs * 4 >= 0x3f000000 || (int64_t)pl.fpc * dys * 4 >= 0x7f000000 ||
      (int64_t)g.G * g.P * 4 >= 0x7f000000)
    return false;
  pl.ktiles = (g.Kdim + W2_BK - 1) / W2_BK;
  const int ntiles = pl.ktiles * ((g.G + W2_BG - 1) / W2_BG);
  const int64_t chain = (int64_t)g.R * g.P;
  int s0 = (int)((chain + 8191) / 8192);
  if (s0 < 1) s0 = 1;
  if (s0 * ntiles < 512) s0 = (512 + ntiles - 1) / ntiles;
  if (s0 > g.R) s0 = g.R;
  int best_s = -1, best_fps = 0;
  int64_t best_cost = 0;
  for (int s = s0; s <= 2 * s0 && s <= g.R; s++) {
    int fps = (g.R + s - 1) / s;
    fps = (fps + pl.fpc - 1) / pl.fpc * pl.fpc;  // whole chunks per split
    const int sa = (g.R + fps - 1) / fps;
    const int64_t rounds = ((int64_t)sa * ntiles + 511) / 512;
    const int64_t cost = rounds * ((fps + pl.fpc - 1) / pl.fpc);
    if (best_s < 0 || cost < best_cost) { best_s = sa; best_fps = fps; best_cost = cost; }
  }
  pl.S = best_s;
  pl.fps = best_fps;
  pl.nblocks = pl.S * ntiles;
  const size_t E = (size_t)g.G * g.Kdim + g.G;
  pl.ws_bytes = (size_t)pl.S * E * sizeof(float) + kcnn_reduce_splits_ws(pl.S, (int)E);
  return true;
}

int launch_wgrad2(const ConvGeom &g, const Wgrad2Plan &pl, const float *X, int xs,
                  const float *dY, int dys, float *ws, hipStream_t st) {
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
  const dim3 grid((unsigned)(8 * ((pl.nblocks + 7) / 8)));
#define KCNN_W2(N_, P_)                                                                    \
  hipLaunchKernelGGL((conv_wgrad2_kernel<N_, P_>), grid, dim3(256), 0, st, g, X, xs, dY, \
                     dys, ws, pl.fps, pl.fpc, pl.bt, pl.ktiles, pl.nblocks)
#define KCNN_W2P(N_) do { if (padded) KCNN_W2(N_, true); else KCNN_W2(N_, false); } while (0)
  switch (pl.nch) {
    case 1: KCNN_W2P(1); break;
    case 2: KCNN_W2P(2); break;
    case 3: KCNN_W2P(3); break;
    default: KCNN_W2P(3); break;
  }
#undef KCNN_W2P
#undef KCNN_W2
  return kcnn::launch_status();
}

// Scatter-form data gradient: worth it when the map has many more
// positions than the output (gather waste HW/P; nnet.config layer 1: 840 vs
// 18, a 47x waste for the flipped-kernel gather).
bool use_dgrad_scatter(const ConvGeom &g) {
  static const int enabled = KCNN_KNOB("KCNN_DGRAD_SCATTER", 1);
  return enabled && g.Kdim >= 32 && 4 * (int64_t)g.HW >= 5 * (int64_t)g.P && g.G >= 16;
}

size_t zbytes_pad(size_t b) { return (b + 255) & ~(size_t)255; }

size_t dgrad_scatter_ws(const ConvGeom &g) {
  if (!use_dgrad_scatter(g)) return 0;
  const int wts = (g.Kdim + 3) & ~3;
  const size_t wt = zbytes_pad((size_t)g.G * wts * 4);
  const size_t z = zbytes_pad((size_t)g.R * g.Kdim * g.P * 4);
  ConvGeom g1 = make_geom(g.R, g.oh, g.ow, g.G, 0, 0, 1, 1, g.Kdim);
  return wt + z + plan_igemm(g1).ws_bytes;
}

}  // namespace

extern "C" {
int hipF_conv2d(const float *in, MatrixDim in_dim, int in_height, int in_width,
                int in_channel, int pad_h, int pad_w, const float *kernel,
                MatrixDim kernel_dim, int kernel_height, int kernel_width,
                int group, const float *bias, float *out, MatrixDim out_dim,
                int concat, void *workspace, size_t workspace_bytes,
                kcnn_stream_t stream);
}

namespace {

int dgrad_scatter(const ConvGeom &g, const float *dY, MatrixDim dyd,
                  const float *W, MatrixDim wd, float *dX, MatrixDim dxd,
                  void *ws, size_t ws_bytes, kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  const int wts = (g.Kdim + 3) & ~3;
  float *wt = static_cast<float *>(ws);
  const size_t wt_b = zbytes_pad((size_t)g.G * wts * 4);
  float *z = reinterpret_cast<float *>(static_cast<char *>(ws) + wt_b);
  const size_t z_b = zbytes_pad((size_t)g.R * g.Kdim * g.P * 4);
  const int64_t nt = (int64_t)g.Kdim * g.G;
  hipLaunchKernelGGL(conv_transpose_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256),
                     0, st, W, g.Kdim, g.G, wd.stride, wt, wts);
  int rc = kcnn::launch_status();
  if (rc) return rc;
  MatrixDim wtd, zd;
  wtd.rows = g.G; wtd.cols = g.Kdim; wtd.stride = wts;
  zd.rows = g.R; zd.cols = g.Kdim * g.P; zd.stride = zd.cols;
  // Z[n][k*P + p] = sum_g dY[n][g*P + p] W[k][g]: a 1x1 convolution of the
  // (oh x ow x G) map dY into Kdim output maps.
  rc = hipF_conv2d(dY, dyd, g.oh, g.ow, g.G, 0, 0, wt, wtd, 1, 1, g.Kdim, nullptr, z,
                   zd, 1, static_cast<char *>(ws) + wt_b + z_b, ws_bytes - wt_b - z_b,
                   stream);
  if (rc) return rc;
  // one wave per (frame, channel) pays off for long runs only (c5 C2: 864
  // floats); short ones (nnet.config C5/C6: 12) go element-wise
  const size_t zlds = (size_t)g.kh * g.kw * g.P * 4;
  if (zlds >= 1024 && zlds <= 32768) {
    const int units = g.R * g.C;
    const bool vec = (g.kh * g.kw * g.P) % 4 == 0 && zd.stride % 4 == 0;
    static const int nt = KCNN_KNOB("KCNN_COL2IM_NT", 1);
    hipLaunchKernelGGL(conv_col2im_plane_kernel,
                       dim3((unsigned)(units < 256 * 24 ? units : 256 * 24)), dim3(64), zlds,
                       st, g, z, zd.stride, dX, dxd.stride, vec ? (nt ? 3 : 1) : 0);
    return kcnn::launch_status();
  }
  const int64_t ne = (int64_t)g.R * g.C * g.HW;
  hipLaunchKernelGGL(conv_col2im_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0,
                     st, g, z, zd.stride, dX, dxd.stride);
  return kcnn::launch_status();
}

}  // namespace

extern "C" {

size_t hipF_conv2d_workspace_bytes(MatrixDim in_dim, int in_height,
                                   int in_width, int in_channel, int pad_h,
                                   int pad_w, int kernel_height,
                                   int kernel_width, int group) {
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0) return 0;
  if (use_direct(g, 1)) return 0;  // caller decides concat; direct needs none
  return plan_igemm(g).ws_bytes;
}

// Conv2D(concat) + bias + channel-only Maxpool_prop in one pass (see
// include/cnsl-hip-kernels.h).  Returns -1 (nothing launched) when the
// geometry is not covered, so the caller runs the two components unfused.
int hipF_conv2d_maxpool(const float *in, MatrixDim in_dim, int in_height,
                        int in_width, int in_channel, int pad_h, int pad_w,
                        const float *kernel, MatrixDim kernel_dim,
                        int kernel_height, int kernel_width, int group,
                        const float *bias, float *out, MatrixDim out_dim,
                        float *pool, MatrixDim pool_dim, unsigned char *mask,
                        int mask_stride, int pool_channel_dim,
                        kcnn_stream_t stream) {
  return kcnn_conv2d_maxpool_stats(in, in_dim, in_height, in_width, in_channel, pad_h, pad_w,
                                   kernel, kernel_dim, kernel_height, kernel_width, group,
                                   bias, out, out_dim, pool, pool_dim, mask, mask_stride,
                                   pool_channel_dim, stream, nullptr);
}

// The scratch words for the pooled output's statistics (pool-stats.h) of
// hipF_conv2d_maxpool's geometry; 0 when the layer takes no frame kernel.
size_t kcnn_conv2d_maxpool_stats_words(int rows, int in_height, int in_width,
                                       int in_channel, int kernel_height, int kernel_width,
                                       int group, int pool_channel_dim) {
  ConvGeom g = make_geom(rows, in_height, in_width, in_channel, 0, 0, kernel_height,
                         kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || pool_channel_dim <= 0) return 0;
  return kcnn_pool_stats_partial_words(g, pool_channel_dim);
}

// hipF_conv2d_maxpool plus the pooled output's statistics when its kernel
// gives them (stats nullable; stats->produced tells)
int kcnn_conv2d_maxpool_stats(const float *in, MatrixDim in_dim, int in_height,
                              int in_width, int in_channel, int pad_h, int pad_w,
                              const float *kernel, MatrixDim kernel_dim,
                              int kernel_height, int kernel_width, int group,
                              const float *bias, float *out, MatrixDim out_dim,
                              float *pool, MatrixDim pool_dim, unsigned char *mask,
                              int mask_stride, int pool_channel_dim,
                              kcnn_stream_t stream, PoolStatsOut *stats) {
  if (stats) stats->produced = 0;
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group ||
      out_dim.rows != g.R || out_dim.cols != g.P * group ||
      pool_channel_dim <= 0 || pool_dim.rows != g.R ||
      pool_dim.cols * pool_channel_dim != out_dim.cols ||
      mask_stride < pool_dim.cols)
    return (int)hipErrorInvalidValue;
  if (g.R == 0) return 0;
  if (g.M >= ((int64_t)1 << 31)) return -1;
  return kcnn_conv_fwd_frame_pool(g, in, in_dim.stride, kernel, kernel_dim.stride,
                                  bias, out, out_dim.stride, pool, pool_dim.stride,
                                  mask, mask_stride, pool_channel_dim,
                                  kcnn::as_stream(stream), 1, 1, stats) == 0 ? 0 : -1;
}

int hipF_conv2d_maxpool3d(const float *in, MatrixDim in_dim, int in_height,
                          int in_width, int in_channel, int pad_h, int pad_w,
                          const float *kernel, MatrixDim kernel_dim,
                          int kernel_height, int kernel_width, int group,
                          const float *bias, float *out, MatrixDim out_dim,
                          float *pool, MatrixDim pool_dim, unsigned short *mask,
                          int mask_stride, int pool_height_dim, int pool_width_dim,
                          int pool_channel_dim, kcnn_stream_t stream) {
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  const int ph = pool_height_dim, pw = pool_width_dim, pc = pool_channel_dim;
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group ||
      out_dim.rows != g.R || out_dim.cols != g.P * group || ph <= 0 || pw <= 0 ||
      pc <= 0 || pool_dim.rows != g.R ||
      (int64_t)pool_dim.cols * ph * pw * pc != out_dim.cols || mask_stride < pool_dim.cols)
    return (int)hipErrorInvalidValue;
  if (g.R == 0) return 0;
  if (g.M >= ((int64_t)1 << 31)) return -1;
  hipStream_t st = kcnn::as_stream(stream);
  if (kcnn_conv_fwd_frame_pool(g, in, in_dim.stride, kernel, kernel_dim.stride, bias, out,
                               out_dim.stride, pool, pool_dim.stride,
                               reinterpret_cast<unsigned char *>(mask), mask_stride, pc, st,
                               ph, pw) == 0)
    return 0;
  // long kernels: the implicit GEMM with the pool in its epilogue, for the
  // shapes whose unfused convolution is that same kernel (conv2d_impl: not
  // in the frame kernels' range, not the small-filter direct kernel)
  // (KCNN_IGEMM_POOL=0: unfused)
  static const int igpool = KCNN_KNOB("KCNN_IGEMM_POOL", 1);
  if (!igpool || (g.Kdim <= 64 && g.P >= 16) || use_direct(g, 1)) return -1;
  return kcnn_conv_igemm_x6_pool(g, in, in_dim.stride, kernel, kernel_dim.stride, bias, out,
                                 out_dim.stride, pool, pool_dim.stride, mask, mask_stride, ph,
                                 pw, pc, st) == 0
             ? 0
             : -1;
}

// relu: the implicit-GEMM v2 path only (-1 for shapes that take another)
static int conv2d_impl(const float *in, MatrixDim in_dim, int in_height, int in_width,
                       int in_channel, int pad_h, int pad_w, const float *kernel,
                       MatrixDim kernel_dim, int kernel_height, int kernel_width,
                       int group, const float *bias, float *out, MatrixDim out_dim,
                       int concat, void *workspace, size_t workspace_bytes,
                       kcnn_stream_t stream, int relu) {
  hipStream_t st = kcnn::as_stream(stream);
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group)
    return (int)hipErrorInvalidValue;
  if (concat ? (out_dim.rows != g.R || out_dim.cols != g.P * group)
             : (out_dim.rows != g.M || out_dim.cols != group))
    return (int)hipErrorInvalidValue;
  if (g.M == 0) return 0;
  if (g.M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (!concat) bias = nullptr;

  // shapes in the frame kernels' range (kcnn_conv_fwd_frame) run unfused:
  // the fused result then comes from the same kernel as the unfused one
  if (relu && g.Kdim <= 64 && g.P >= 16) return -1;
  // likewise the small-filter-count shapes the direct kernel serves
  if (relu && use_direct(g, concat)) return -1;
  if (!relu && concat && kcnn_conv_fwd_frame(g, in, in_dim.stride, kernel,
                                             kernel_dim.stride, bias, out,
                                             out_dim.stride, st) == 0)
    return 0;
  if (!relu && use_direct(g, concat)) {
    const unsigned blocks = (unsigned)((g.M + 255) / 256);
#define KCNN_DIRECT(NG)                                                        \
  hipLaunchKernelGGL(conv_direct_smallg_kernel<NG>, dim3(blocks), dim3(256), 0, \
                     st, g, in, in_dim.stride, kernel, kernel_dim.stride, bias, \
                     out, out_dim.stride)
    if (g.G <= 1) KCNN_DIRECT(1);
    else if (g.G <= 2) KCNN_DIRECT(2);
    else if (g.G <= 4) KCNN_DIRECT(4);
    else KCNN_DIRECT(8);
#undef KCNN_DIRECT
    return kcnn::launch_status();
  }

  // the implicit GEMM on the bf16 MFMAs (exact three-way operand splits)
  if (concat && kcnn_conv_igemm_x6(g, in, in_dim.stride, kernel, kernel_dim.stride, bias,
                                   out, out_dim.stride, relu, st) == 0)
    return 0;
  // implicit GEMM v2 (fp32 MFMA): concat layout, X addressable with 32-bit
  // offsets, tap masks for padded maps need kh*kw <= 32
  static const int ig2 = KCNN_KNOB("KCNN_IGEMM2", 1);
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
  const int wgg = g.G > 64 ? 2 : 1;
  if (ig2 && concat && (int64_t)g.R * in_dim.stride * 4 < ((int64_t)1 << 31) &&
      (int64_t)g.Kdim * kernel_dim.stride * 4 < ((int64_t)1 << 31) &&
      g.G % 4 == 0 && kernel_dim.stride % 4 == 0 &&
      (uintptr_t)kernel % 16 == 0 && (!padded || g.kh * g.kw <= 32)) {
    const int bg = 64 * wgg, bm = 64 * (4 / wgg);
    dim3 grid2((unsigned)((g.M + bm - 1) / bm), (unsigned)((g.G + bg - 1) / bg));
    // timing experiments (operand loads / LDS stores / traffic switched off):
    // only in the phase-timing build (make timing), never in libkcnn.so
    static const int ig2timing = KCNN_KNOB("KCNN_IGEMM2_DEBUG", 0);
    const int ig2dbg = ig2timing | (relu ? kIg2Relu : 0);
    static const int ig2bk = KCNN_KNOB("KCNN_IGEMM2_BK", 16);
    static const int ig2tab = KCNN_KNOB("KCNN_IGEMM2_TAB", 1);
    const bool tab = ig2tab && (g.Kdim + 15) / 16 * 16 <= IG2_KTAB &&
                     (int64_t)g.HW * g.C < (1 << 28) && (!padded || g.kh * g.kw <= 31);
#define KCNN_IG2(W_, P_)                                                                  \
  do {                                                                                    \
    if (tab)                                                                              \
      hipLaunchKernelGGL((conv_igemm2_kernel<W_, P_, 16, true>), grid2, dim3(256), 0, st, g, \
                         in, in_dim.stride, kernel, kernel_dim.stride, bias, out,          \
                         out_dim.stride, ig2dbg);                                          \
    else if (ig2bk == 32)                                                                 \
      hipLaunchKernelGGL((conv_igemm2_kernel<W_, P_, 32, false>), grid2, dim3(256), 0, st, g, \
                         in, in_dim.stride, kernel, kernel_dim.stride, bias, out,          \
                         out_dim.stride, ig2dbg);                                          \
    else                                                                                  \
      hipLaunchKernelGGL((conv_igemm2_kernel<W_, P_, 16, false>), grid2, dim3(256), 0, st, g, \
                         in, in_dim.stride, kernel, kernel_dim.stride, bias, out,          \
                         out_dim.stride, ig2dbg);                                          \
  } while (0)
    if (wgg == 2) {
      if (padded) KCNN_IG2(2, true); else KCNN_IG2(2, false);
    } else {
      if (padded) KCNN_IG2(1, true); else KCNN_IG2(1, false);
    }
#undef KCNN_IG2
    return kcnn::launch_status();
  }
  if (relu) return -1;

  IgemmPlan pl = plan_igemm(g);
  if (pl.S > 1 && (workspace == nullptr || workspace_bytes < pl.ws_bytes)) {
    pl.S = 1;
    pl.k_per_split = (g.Kdim + IG_BK - 1) / IG_BK * IG_BK;
  }
  dim3 grid((unsigned)((g.M + IG_BM - 1) / IG_BM),
            (unsigned)((g.G + IG_BG - 1) / IG_BG), (unsigned)pl.S);
  if (pl.S > 1) {
    float *ws = static_cast<float *>(workspace);
    hipLaunchKernelGGL(conv_igemm_kernel<ST_PARTIAL>, grid, dim3(256), 0, st, g,
                       in, in_dim.stride, kernel, kernel_dim.stride, nullptr,
                       nullptr, 0, ws, pl.k_per_split);
    int rc = kcnn::launch_status();
    if (rc) return rc;
    // pass 1 (groups of 32 splits) into tmp, pass 2 = reduce + store epilogue
    const int E = (int)(g.G * g.M);
    const int Q = (pl.S + 31) / 32;
    float *tmp = ws + (size_t)pl.S * E;
    rc =kcnn_reduce_splits_pass1(ws, pl.S, E, tmp, st);
    if (rc) return rc;
    hipLaunchKernelGGL(conv_splitk_reduce_kernel,
                       dim3(kcnn::grid_for((int64_t)g.G * g.M)), dim3(256), 0,
                       st, g, tmp, Q, bias, out, out_dim.stride, concat);
  } else if (concat) {
    hipLaunchKernelGGL(conv_igemm_kernel<ST_CONCAT>, grid, dim3(256), 0, st, g,
                       in, in_dim.stride, kernel, kernel_dim.stride, bias, out,
                       out_dim.stride, nullptr, pl.k_per_split);
  } else {
    hipLaunchKernelGGL(conv_igemm_kernel<ST_PLAIN>, grid, dim3(256), 0, st, g,
                       in, in_dim.stride, kernel, kernel_dim.stride, nullptr,
                       out, out_dim.stride, nullptr, pl.k_per_split);
  }
  return kcnn::launch_status();
}

int hipF_conv2d(const float *in, MatrixDim in_dim, int in_height, int in_width,
                int in_channel, int pad_h, int pad_w, const float *kernel,
                MatrixDim kernel_dim, int kernel_height, int kernel_width,
                int group, const float *bias, float *out, MatrixDim out_dim,
                int concat, void *workspace, size_t workspace_bytes,
                kcnn_stream_t stream) {
  return conv2d_impl(in, in_dim, in_height, in_width, in_channel, pad_h, pad_w, kernel,
                     kernel_dim, kernel_height, kernel_width, group, bias, out, out_dim,
                     concat, workspace, workspace_bytes, stream, 0);
}

int hipF_conv2d_relu(const float *in, MatrixDim in_dim, int in_height, int in_width,
                     int in_channel, int pad_h, int pad_w, const float *kernel,
                     MatrixDim kernel_dim, int kernel_height, int kernel_width,
                     int group, const float *bias, float *out, MatrixDim out_dim,
                     kcnn_stream_t stream) {
  return conv2d_impl(in, in_dim, in_height, in_width, in_channel, pad_h, pad_w, kernel,
                     kernel_dim, kernel_height, kernel_width, group, bias, out, out_dim,
                     1, nullptr, 0, stream, 1);
}

size_t hipF_conv2d_wgrad_workspace_bytes(MatrixDim in_dim, int in_height,
                                         int in_width, int in_channel,
                                         int pad_h, int pad_w,
                                         int kernel_height, int kernel_width,
                                         int group) {
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0) return 0;
  size_t a = kcnn_conv_wgrad_frame_ws(g);
  const size_t b = plan_wgrad(g).ws_bytes, c = kcnn_conv_bwd_frame_ws(g);
  if (b > a) a = b;
  Wgrad2Plan p2;
  if (plan_wgrad2(g, in_dim.stride > 0 ? in_dim.stride : g.HW * in_channel,
                  g.P * group, p2) && p2.ws_bytes > a)
    a = p2.ws_bytes;
  int xS, xfps;
  size_t xb;
  if (kcnn_conv_wgrad_x6_plan(g, in_dim.stride > 0 ? in_dim.stride : g.HW * in_channel,
                              g.P * group, xS, xfps, xb) && xb > a)
    a = xb;
  return c > a ? c : a;
}

int hipF_conv2d_wgrad(const float *in, MatrixDim in_dim, int in_height,
                      int in_width, int in_channel, int pad_h, int pad_w,
                      const float *out_deriv, MatrixDim out_deriv_dim,
                      int kernel_height, int kernel_width, int group,
                      float *grad_W, MatrixDim grad_W_dim, float *grad_b,
                      void *workspace, size_t workspace_bytes,
                      kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      out_deriv_dim.rows != g.R || out_deriv_dim.cols != g.P * group ||
      grad_W_dim.rows != g.Kdim || grad_W_dim.cols != group)
    return (int)hipErrorInvalidValue;
  if (g.M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  // the fused backward's gradient-only pass (one stream of dY)
  if (g.M > 0 && kcnn_conv_bwd_frame(g, in, in_dim.stride, out_deriv,
                                     out_deriv_dim.stride, nullptr, 0, nullptr, 0,
                                     grad_W, grad_W_dim.stride, grad_b, workspace,
                                     workspace_bytes, st) == 0)
    return 0;
  if (g.M > 0 && kcnn_conv_wgrad_frame(g, in, in_dim.stride, out_deriv,
                                       out_deriv_dim.stride, grad_W,
                                       grad_W_dim.stride, grad_b, workspace,
                                       workspace_bytes, st) == 0)
    return 0;
  {
    // the long-kernel weight gradient on the bf16 MFMAs
    int xS, xfps;
    size_t xb;
    if (g.M > 0 &&
        kcnn_conv_wgrad_x6_plan(g, in_dim.stride, out_deriv_dim.stride, xS, xfps, xb) &&
        workspace != nullptr && workspace_bytes >= xb) {
      const int E = g.G * g.Kdim + g.G;
      float *part = static_cast<float *>(workspace);
      int rc = kcnn_conv_wgrad_x6(g, in, in_dim.stride, out_deriv, out_deriv_dim.stride,
                                  part, xS, xfps, st);
      if (rc) return rc;
      return kcnn_reduce_splits_wgrad(part, xS, E, part + (size_t)xS * E, g.G * g.Kdim,
                                      g.Kdim, grad_W, grad_W_dim.stride, grad_b, st);
    }
  }
  Wgrad2Plan p2;
  if (g.M > 0 && plan_wgrad2(g, in_dim.stride, out_deriv_dim.stride, p2) &&
      workspace != nullptr && workspace_bytes >= p2.ws_bytes) {
    const int E = g.G * g.Kdim + g.G;
    float *part = static_cast<float *>(workspace);
    int rc = launch_wgrad2(g, p2, in, in_dim.stride, out_deriv, out_deriv_dim.stride,
                           part, st);
    if (rc) return rc;
    return kcnn_reduce_splits_wgrad(part, p2.S, E, part + (size_t)p2.S * E,
                                    g.G * g.Kdim, g.Kdim, grad_W, grad_W_dim.stride,
                                    grad_b, st);
  }
  WgradPlan pl = plan_wgrad(g);
  if (workspace == nullptr || workspace_bytes < pl.ws_bytes)
    return (int)hipErrorInvalidValue;
  const int E = g.G * g.Kdim + g.G;
  float *ws_w = static_cast<float *>(workspace);
  float *ws_b = ws_w + (size_t)g.G * g.Kdim;
  float *tmp = ws_w + (size_t)pl.S * E;
  if (g.M == 0) {
    if (hipMemsetAsync(ws_w, 0, (size_t)pl.S * E * sizeof(float), st) != hipSuccess)
      return (int)hipErrorInvalidValue;
  } else {
    dim3 grid((unsigned)pl.S, (unsigned)((g.G + WG_BG - 1) / WG_BG),
              (unsigned)((g.Kdim + WG_BK - 1) / WG_BK));
    hipLaunchKernelGGL(conv_wgrad_kernel, grid, dim3(256), 0, st, g, in,
                       in_dim.stride, out_deriv, out_deriv_dim.stride, ws_w,
                       ws_b, pl.t_per_split);
  }
  int rc = kcnn::launch_status();
  if (rc) return rc;
  return kcnn_reduce_splits_wgrad(ws_w, pl.S, E, tmp, g.G * g.Kdim, g.Kdim,
                                  grad_W, grad_W_dim.stride, grad_b, st);
}

size_t hipF_conv2d_dgrad_workspace_bytes(MatrixDim out_deriv_dim, int in_height,
                                         int in_width, int in_channel,
                                         int pad_h, int pad_w,
                                         int kernel_height, int kernel_width,
                                         int group) {
  ConvGeom g = make_geom(out_deriv_dim.rows, in_height, in_width, in_channel,
                         pad_h, pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0) return 0;
  // fallback: flipped kernel + implicit GEMM over the virtually padded dY
  ConvGeom gt = make_geom(out_deriv_dim.rows, g.oh, g.ow, group,
                          kernel_height - 1 - pad_h, kernel_width - 1 - pad_w,
                          kernel_height, kernel_width, in_channel);
  const size_t flip_bytes = (size_t)kernel_height * kernel_width * group *
                            in_channel * sizeof(float);
  const size_t flip_pad = (flip_bytes + 255) & ~(size_t)255;
  const size_t a = flip_pad + (use_direct(gt, 1) ? 0 : plan_igemm(gt).ws_bytes);
  const size_t b = dgrad_scatter_ws(g);
  return b > a ? b : a;
}

int hipF_conv2d_dgrad(const float *out_deriv, MatrixDim out_deriv_dim,
                      int in_height, int in_width, int in_channel, int pad_h,
                      int pad_w, const float *kernel, MatrixDim kernel_dim,
                      int kernel_height, int kernel_width, int group,
                      float *in_deriv, MatrixDim in_deriv_dim, void *workspace,
                      size_t workspace_bytes, kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  ConvGeom g = make_geom(out_deriv_dim.rows, in_height, in_width, in_channel,
                         pad_h, pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || out_deriv_dim.cols != g.P * group ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group ||
      in_deriv_dim.rows != g.R || in_deriv_dim.cols != g.HW * in_channel ||
      pad_h > kernel_height - 1 || pad_w > kernel_width - 1)
    return (int)hipErrorInvalidValue;
  if (g.R == 0) return 0;
  if (g.M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  // the fused backward's data-gradient-only pass
  if (kcnn_conv_bwd_frame(g, nullptr, 0, out_deriv, out_deriv_dim.stride, kernel,
                          kernel_dim.stride, in_deriv, in_deriv_dim.stride, nullptr,
                          0, nullptr, nullptr, 0, st) == 0)
    return 0;
  if (kcnn_conv_dgrad_frame(g, out_deriv, out_deriv_dim.stride, kernel,
                            kernel_dim.stride, in_deriv, in_deriv_dim.stride,
                            st) == 0)
    return 0;
  if (use_dgrad_scatter(g) && workspace != nullptr &&
      workspace_bytes >= dgrad_scatter_ws(g))
    return dgrad_scatter(g, out_deriv, out_deriv_dim, kernel, kernel_dim, in_deriv,
                         in_deriv_dim, workspace, workspace_bytes, stream);
  // General shapes: dX = Conv2D(virtually padded dY, FlipMat(W)) -- the
  // reference's flip branch (nnet-component-nnet0.cc:529-540) in gather form.
  const size_t flip_bytes = (size_t)kernel_height * kernel_width * group *
                            in_channel * sizeof(float);
  const size_t flip_pad = (flip_bytes + 255) & ~(size_t)255;
  const size_t need = hipF_conv2d_dgrad_workspace_bytes(
      out_deriv_dim, in_height, in_width, in_channel, pad_h, pad_w,
      kernel_height, kernel_width, group);
  if (workspace == nullptr || workspace_bytes < need)
    return (int)hipErrorInvalidValue;
  float *flip = static_cast<float *>(workspace);
  MatrixDim fd;
  fd.rows = kernel_height * kernel_width * group;
  fd.cols = in_channel;
  fd.stride = in_channel;
  int rc = hipF_flip_mat(kernel, kernel_dim, kernel_height, kernel_width, group,
                         flip, fd, stream);
  if (rc) return rc;
  return hipF_conv2d(out_deriv, out_deriv_dim, g.oh, g.ow, group,
                     kernel_height - 1 - pad_h, kernel_width - 1 - pad_w, flip,
                     fd, kernel_height, kernel_width, in_channel, nullptr,
                     in_deriv, in_deriv_dim, 1,
                     static_cast<char *>(workspace) + flip_pad,
                     workspace_bytes - flip_pad, stream);
}

size_t hipF_conv2d_backward_workspace_bytes(MatrixDim in_dim, int in_height,
                                            int in_width, int in_channel,
                                            int pad_h, int pad_w,
                                            int kernel_height, int kernel_width,
                                            int group) {
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0) return 0;
  MatrixDim od;
  od.rows = in_dim.rows;
  od.cols = g.P * group;
  od.stride = od.cols;
  size_t a = kcnn_conv_bwd_frame_ws(g);
  const size_t b = hipF_conv2d_dgrad_workspace_bytes(
      od, in_height, in_width, in_channel, pad_h, pad_w, kernel_height,
      kernel_width, group);
  const size_t c = hipF_conv2d_wgrad_workspace_bytes(
      in_dim, in_height, in_width, in_channel, pad_h, pad_w, kernel_height,
      kernel_width, group);
  if (b > a) a = b;
  return c > a ? c : a;
}

// The pooled backward of a ph x 1 x pc window (ph == 1: channel-only, 1-byte
// mask; else a 2-byte mask), mask_bytes = the mask's row pitch in bytes.
static int conv2d_backward_pooled(const float *in, MatrixDim in_dim, int in_height,
                                  int in_width, int in_channel, int pad_h, int pad_w,
                                  const unsigned char *mask, int64_t mask_pitch,
                                  int64_t mask_cols, const float *pool_deriv,
                                  MatrixDim pool_deriv_dim, int ph, int pc,
                                  const float *kernel, MatrixDim kernel_dim,
                                  int kernel_height, int kernel_width, int group,
                                  float *in_deriv, MatrixDim in_deriv_dim, float *grad_W,
                                  MatrixDim grad_W_dim, float *grad_b, void *workspace,
                                  size_t workspace_bytes, hipStream_t st) {
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      !(pc == 2 || pc == 4 || pc == 8) || group % pc != 0 ||  // pc = 2: declined below
      ph < 1 || g.oh % ph != 0 ||
      pool_deriv_dim.rows != g.R ||
      (int64_t)pool_deriv_dim.cols * pc * ph != (int64_t)g.P * group ||
      mask == nullptr || mask_cols < pool_deriv_dim.cols ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group ||
      (grad_W == nullptr && in_deriv == nullptr) ||
      (grad_W != nullptr && (grad_W_dim.rows != g.Kdim || grad_W_dim.cols != group)))
    return (int)hipErrorInvalidValue;
  if (in_deriv != nullptr &&
      (in_deriv_dim.rows != g.R || in_deriv_dim.cols != g.HW * in_channel ||
       pad_h > kernel_height - 1 || pad_w > kernel_width - 1))
    return (int)hipErrorInvalidValue;
  if (g.M >= ((int64_t)1 << 31) || mask_pitch >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  if (g.R == 0) return 0;
  return kcnn_conv_bwd_frame(g, in, in_dim.stride, pool_deriv, pool_deriv_dim.stride,
                             kernel, kernel_dim.stride, in_deriv,
                             in_deriv ? in_deriv_dim.stride : 0, grad_W,
                             grad_W ? grad_W_dim.stride : 0, grad_b, workspace,
                             workspace_bytes, st, mask, (int)mask_pitch, pc,
                             ph);  // -1: declined, > 0: HIP error
}

int hipF_conv2d_backward_pooled(const float *in, MatrixDim in_dim, int in_height,
                                int in_width, int in_channel, int pad_h, int pad_w,
                                const unsigned char *mask, int mask_stride,
                                const float *pool_deriv, MatrixDim pool_deriv_dim,
                                int pool_channel_dim, const float *kernel,
                                MatrixDim kernel_dim, int kernel_height,
                                int kernel_width, int group, float *in_deriv,
                                MatrixDim in_deriv_dim, float *grad_W,
                                MatrixDim grad_W_dim, float *grad_b, void *workspace,
                                size_t workspace_bytes, kcnn_stream_t stream) {
  return conv2d_backward_pooled(in, in_dim, in_height, in_width, in_channel, pad_h, pad_w,
                                mask, mask_stride, mask_stride, pool_deriv, pool_deriv_dim,
                                1, pool_channel_dim, kernel, kernel_dim, kernel_height,
                                kernel_width, group, in_deriv, in_deriv_dim, grad_W,
                                grad_W_dim, grad_b, workspace, workspace_bytes,
                                kcnn::as_stream(stream));
}

int hipF_conv2d_backward_pooled3d(const float *in, MatrixDim in_dim, int in_height,
                                  int in_width, int in_channel, int pad_h, int pad_w,
                                  const unsigned short *mask, int mask_stride,
                                  const float *pool_deriv, MatrixDim pool_deriv_dim,
                                  int pool_height_dim, int pool_width_dim,
                                  int pool_channel_dim, const float *kernel,
                                  MatrixDim kernel_dim, int kernel_height,
                                  int kernel_width, int group, float *in_deriv,
                                  MatrixDim in_deriv_dim, float *grad_W,
                                  MatrixDim grad_W_dim, float *grad_b, void *workspace,
                                  size_t workspace_bytes, kcnn_stream_t stream) {
  if (pool_width_dim != 1 || pool_height_dim < 2) return -1;  // not covered
  return conv2d_backward_pooled(in, in_dim, in_height, in_width, in_channel, pad_h, pad_w,
                                reinterpret_cast<const unsigned char *>(mask),
                                (int64_t)mask_stride * 2, mask_stride, pool_deriv,
                                pool_deriv_dim, pool_height_dim, pool_channel_dim, kernel,
                                kernel_dim, kernel_height, kernel_width, group, in_deriv,
                                in_deriv_dim, grad_W, grad_W_dim, grad_b, workspace,
                                workspace_bytes, kcnn::as_stream(stream));
}

int hipF_conv2d_backward(const float *in, MatrixDim in_dim, int in_height,
                         int in_width, int in_channel, int pad_h, int pad_w,
                         const float *out_deriv, MatrixDim out_deriv_dim,
                         const float *kernel, MatrixDim kernel_dim,
                         int kernel_height, int kernel_width, int group,
                         float *in_deriv, MatrixDim in_deriv_dim, float *grad_W,
                         MatrixDim grad_W_dim, float *grad_b, void *workspace,
                         size_t workspace_bytes, kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  ConvGeom g = make_geom(in_dim.rows, in_height, in_width, in_channel, pad_h,
                         pad_w, kernel_height, kernel_width, group);
  if (g.oh <= 0 || g.ow <= 0 || in_dim.cols != g.HW * in_channel ||
      out_deriv_dim.rows != g.R || out_deriv_dim.cols != g.P * group ||
      kernel_dim.rows != g.Kdim || kernel_dim.cols != group ||
      grad_W_dim.rows != g.Kdim || grad_W_dim.cols != group || grad_W == nullptr)
    return (int)hipErrorInvalidValue;
  if (in_deriv != nullptr &&
      (in_deriv_dim.rows != g.R || in_deriv_dim.cols != g.HW * in_channel ||
       pad_h > kernel_height - 1 || pad_w > kernel_width - 1))
    return (int)hipErrorInvalidValue;
  if (g.M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (g.R > 0 &&
      kcnn_conv_bwd_frame(g, in, in_dim.stride, out_deriv, out_deriv_dim.stride,
                          kernel, kernel_dim.stride, in_deriv,
                          in_deriv ? in_deriv_dim.stride : 0, grad_W,
                          grad_W_dim.stride, grad_b, workspace, workspace_bytes,
                          st) == 0)
    return 0;
  if (in_deriv != nullptr) {
    const int rc = hipF_conv2d_dgrad(out_deriv, out_deriv_dim, in_height,
                                     in_width, in_channel, pad_h, pad_w, kernel,
                                     kernel_dim, kernel_height, kernel_width,
                                     group, in_deriv, in_deriv_dim, workspace,
                                     workspace_bytes, stream);
    if (rc) return rc;
  }
  return hipF_conv2d_wgrad(in, in_dim, in_height, in_width, in_channel, pad_h,
                           pad_w, out_deriv, out_deriv_dim, kernel_height,
                           kernel_width, group, grad_W, grad_W_dim, grad_b,
                           workspace, workspace_bytes, stream);
}

}  // extern "C"
