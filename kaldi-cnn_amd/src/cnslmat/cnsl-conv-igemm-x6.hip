// cnslmat/cnsl-conv-igemm-x6.hip -- the implicit-GEMM convolution of the
// long-kernel layers (BASELINE c5 C2-C4, every conv of the reference's
// egs/exp/nnet/nnet.config, and the flipped-kernel / 1x1 data gradients) on
// the bf16 matrix cores, with every fp32 operand split exactly into three
// bf16 parts and the six leading cross products kept (x6-util.h), or, for
// the large shapes (F16 below, igemm_x6 family 2 / 3), on the f16 matrix
// cores with two f16 parts under a power-of-two scale per filter and per
// frame and three products (f16-split.h), checked at the store and fixed up
// in fp32 where the scale cannot hold a product to the per-element bar.
//
// Reference: CuMatrixBase::Conv2D (conv2D.cc:43-201) = im2col span (:105,
// _span_row_to_convmat) + cuBLAS GEMM (:138-139) + _convmat_to_out (:181) +
// AddMatRepVec bias (nnet-component-nnet0.cc:443).  Here, with no span
// matrix:  out[n][g*P + p] = sum_k W[k][g] im2col(X)[k][n*P + p] + b[g],
// a GEMM with rows g (A = W^T) and columns m = n*P + p (B = im2col(X)).
//
// 512 threads, a BG x BN tile of [g x m] (BG + BN = 384: 256 x 128 for wide
// layers, 128 x 256 for G <= 128), 8 waves of 64 x 64 (2 x 2 accumulators of
// 32 x 32), K steps of 32.  Per step each thread loads its share of the next
// step's operands as fp32 into registers (A: W rows, lanes along g, 256-B
// runs; B: im2col gathered straight from X: a wave's k rows are uniform, so
// the tap offset of each k is a scalar stepped on the SALU and an element
// costs one vector add, plus a tap-mask test on padded maps), then splits
// them into three bf16 planes of the
// [row][k] LDS images (64-B rows, 16-B chunks XOR-swizzled), double
// buffered (2 x 72 KB), one barrier per step.  Out-of-range k rows, columns
// past M and taps outside a padded map read 0 through the buffer range.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>

#include "conv-geom.h"
#include "f16-split.h"
#include "x6-util.h"
#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/cu-kernels-lite.h"

using namespace kcnn;

namespace {

constexpr int NT = 512, BK = 32, ROWB = BK * 2;
constexpr unsigned kOob = 0x7ffffff0u;  // an offset past every buffer range used

// the implicit GEMM's images: 16-B chunk c of row r XOR ((r >> 1) ^ (r >> 2))
// & 3, conflict-free for both its ds_write_b128 (8 consecutive rows, banks
// mod 32) and its ds_read_b128 fragments (lane groups {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31}, banks mod 64; MI355X_MICROARCH.md LDS table); swz's
// (r >> 2) & 3 put two rows of every write group on one slot (the f16x3
// C3 forward: 27 % of its LDS cycles were bank conflicts)
__device__ __forceinline__ int swzi(int r, int c) {
  return r * ROWB + ((c ^ (((r >> 1) ^ (r >> 2)) & 3)) << 4);
}
__device__ __forceinline__ int swz(int r, int c) {
  return r * ROWB + ((c ^ ((r >> 2) & 3)) << 4);
}

// eight fp32 -> one 16-B chunk of each plane
__device__ __forceinline__ void put8(char *img, int pl_bytes, int off, const float *v) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) x6::split2(v[2 * i], v[2 * i + 1], h[i], m[i], l[i]);
  *reinterpret_cast<uint4 *>(img + off) = make_uint4(h[0], h[1], h[2], h[3]);
  *reinterpret_cast<uint4 *>(img + pl_bytes + off) = make_uint4(m[0], m[1], m[2], m[3]);
  *reinterpret_cast<uint4 *>(img + 2 * pl_bytes + off) = make_uint4(l[0], l[1], l[2], l[3]);
}

// eight fp32 under the scale 2^e -> one 16-B chunk of each f16 plane (f16x3)
__device__ __forceinline__ void put8h(char *img, int pl_bytes, int off, const float *v, int e,
                                      float m1) {
  f16x3::f16x8 hh, ll;
  f16x3::split8h(v, e, hh, ll, m1);
  *reinterpret_cast<f16x3::f16x8 *>(img + off) = hh;
  *reinterpret_cast<f16x3::f16x8 *>(img + pl_bytes + off) = ll;
}

// One output element (filter gg, column mm = (frame, position)) by a whole
// wave as an fp32 dot product over k in a fixed lane order (lane sums of k =
// lane + 64 i, then a butterfly: every lane ends with the same bits), the
// fixup kernel's element.  Taps outside a padded map are 0.
__device__ __forceinline__ float conv_dot(const ConvGeom &g, const float *__restrict__ X, int xs,
                                          const float *__restrict__ Kw, int ks, int gg, int64_t mm,
                                          int lane) {
  uint32_t n, p, px, py;
  g.div_P.divmod((uint32_t)mm, n, p);
  g.div_oh.divmod(p, px, py);
  const float *xf = X + (int64_t)n * xs;
  float s = 0.0f;
  constexpr int B = 8;  // loads in flight per lane
  for (int k0 = lane; k0 < g.Kdim; k0 += 64 * B) {
    float a[B], x[B];
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int k = k0 + 64 * b;
      a[b] = 0.0f;
      x[b] = 0.0f;
      if (k < g.Kdim) {
        uint32_t c, r, kx, ky;
        g.div_khkw.divmod((uint32_t)k, c, r);
        g.div_kh.divmod(r, kx, ky);
        const int xx = (int)px + (int)kx - g.pad_w, yy = (int)py + (int)ky - g.pad_h;
        if ((unsigned)xx < (unsigned)g.W && (unsigned)yy < (unsigned)g.H) {
          a[b] = Kw[(int64_t)k * ks + gg];
          x[b] = xf[(int64_t)c * g.HW + xx * g.H + yy];
        }
      }
    }
#pragma unroll
    for (int b = 0; b < B; b++) s = fmaf(a[b], x[b], s);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  return s;
}

// The Maxpool that follows the convolution, pooled in the epilogue (POOL >
// 0): a window of 2 consecutive map positions (ph x pw = 2 x 1 with oh even,
// or 1 x 2 with oh = 1: positions p, p + 1 with p even, the columns m, m + 1
// of lanes l, l ^ 1) by PC consecutive filters (rows 4k .. 4k + 3 of an
// accumulator are 4 consecutive registers of one lane).  pool[n][j*P/2 +
// p/2] and the 16-bit routing mask (bit c*2 + d for map PC*j + c at
// position p + d) as hipF_conv2d_maxpool3d writes them; out (Y) nullable.
struct PoolOut {
  float *pool;
  int ps;
  unsigned short *mask;
  int ms;
};

// The f16x3 form (F16, igemm_x6 family value 2; f16-split.h): two f16 planes
// per operand under a power-of-two scale per group, three products per pair.
// The groups: A's rows are W's columns (one filter over every k), B's columns
// take the scale of their frame (every tap of an im2col column reads one
// frame of X, so a frame's max covers them).  Statistics blocks [max, min,
// cnt] (kl_absmax_cols of W, kl_absmax_rows of X: f16-split.h spread /
// spread_weight).  A tile with an Inf / NaN group, or an element the store
// check (the GEMM's tile_epilogue rule: |acc| >= the two groups' spread
// weights) cannot clear, is recomputed in fp32 (conv_dot: a fixed-order dot
// product, IEEE Inf / NaN like the reference's sgemm):
//  - a rejected element is stored (or pooled) as computed and listed with
//    its pool window's values (elist: EW words per entry);
//    conv_igemm_efix_kernel recomputes it and stores it, or re-pools the
//    window, over the epilogue's result;
//  - a tile with an Inf / NaN group, or with a wave of more than REJ_MAX
//    rejections (a pathological spread), stores nothing and lists its id;
//    conv_igemm_fixup_kernel computes every element of it.
constexpr int REJ_MAX = 8;  // listed rejections per wave (more: the whole tile)
constexpr int EW = 12;      // words per element entry: g, m, mask, 8 window values
struct F16Aux {
  const uint32_t *wst;   // [max G][min G][cnt G] of W's columns
  const uint32_t *xst;   // [max R][min R][cnt R] of X's rows (frames)
  unsigned *list;        // [tile count, element count, tile ids (one per tile)]
  unsigned *elist;       // element entries (8 waves x REJ_MAX per tile)
  const uint32_t *wsplit;  // W split once per call: [Kdim][ks] of (lo << 16 | hi)
};

// W's f16x3 parts, once per call (conv_w_presplit_kernel): element (k, g)
// under its filter's scale (the tile kernel's exponent of row g of A = W^T),
// hi in the low half and lo in the high half of a word, the bits split8h
// gives; the tiles then only repack them (two v_perm per element pair)
// instead of splitting every tile's copy of W (each tile re-reads all of W)
__global__ __launch_bounds__(256) void conv_w_presplit_kernel(const float *__restrict__ Kw,
                                                              int ks, int Kdim, int G,
                                                              const uint32_t *__restrict__ wst,
                                                              uint32_t *__restrict__ out) {
  const float m1 = f16x3::opaque_m1();
  const int64_t n = (int64_t)Kdim * G;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i / G), gg = (int)(i - (int64_t)k * G);
    const int e0 = f16x3::scale_exp(wst[gg]);
    const int e = e0 == f16x3::SKIP ? 0 : e0;
    const float x = Kw[(int64_t)k * ks + gg];
    uint32_t h, l;
    f16x3::split2h(x, x, e, e, h, l, m1);
    out[(int64_t)k * ks + gg] = (l << 16) | (h & 0xffffu);
  }
}
constexpr int kAuxBytes = 384 * 8;  // F16: scale exponents and weights of a tile's groups

template <int BG, bool PADDED, bool STG, bool TAB, int POOL, bool F16>
__global__ __launch_bounds__(NT, 1) void conv_igemm_x6_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ Kw, int ks,
    const float *__restrict__ bias, float *__restrict__ out, int os, int relu, PoolOut po,
    F16Aux fx) {
  constexpr int BN = 384 - BG;
  constexpr int APT = BG * BK / NT, BPT = BN * BK / NT;  // values per thread per step
  constexpr int NPL = F16 ? 2 : 3;                       // planes per operand
  constexpr int PLA = BG * ROWB, PLB = BN * ROWB, BUF = NPL * (PLA + PLB);
  constexpr int WN = BN / 64;                            // waves along m
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int l = lane & 31, h = lane >> 5;

  // XCD-aware order: consecutive logical ids on one XCD (blocks are dealt
  // round-robin over the 8 XCDs), g tiles fastest (they share the X columns)
  const int tiles_g = (g.G + BG - 1) / BG;
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rr = nb & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int g0 = (lid % tiles_g) * BG;
  const int64_t m0 = (int64_t)(lid / tiles_g) * BN;
  const int T = (g.Kdim + BK - 1) / BK;

  // A = W^T: thread row g0 + a_row, k = kt*32 + a_kc*APT + j (a_kc uniform)
  const int a_row = tid % BG;
  const int a_kc = __builtin_amdgcn_readfirstlane(tid / BG);
  // (F16: W's parts, split once per call; the same range)
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      F16 ? (void *)fx.wsplit : (void *)Kw, (short)0, g.Kdim * ks * 4, 0x00020000);
  const unsigned a_voff = (unsigned)(g0 + a_row) * 4u;
  // B = im2col(X): thread column m0 + b_row, k = kt*32 + b_kc*BPT + e
  const int b_row = tid % BN;
  const int b_kc = __builtin_amdgcn_readfirstlane(tid / BN);
  const int64_t mcol = m0 + b_row;
  const bool mvalid = mcol < g.M;
  // byte offset of tap (0, 0) of this column (unpadded: in [0, range); a
  // column past M: kOob, so that kOob + any tap offset stays past the range
  // without wrapping; padded: may wrap below 0, the tap mask guards it)
  unsigned xoff4 = kOob;
  unsigned nmask = 0;  // PADDED: bit tap set = tap outside the map
  {
    uint32_t n = 0, p = 0, px = 0, py = 0;
    if (mvalid) {
      g.div_P.divmod((uint32_t)mcol, n, p);
      g.div_oh.divmod(p, px, py);
      xoff4 = (unsigned)((int)n * xs + ((int)px - g.pad_w) * g.H + (int)py - g.pad_h) * 4u;
    }
    if (PADDED) {
      nmask = 0xffffffffu;
      if (mvalid)
        for (int kx = 0; kx < g.kw; kx++)
          for (int ky = 0; ky < g.kh; ky++) {
            const int xx = (int)px + kx - g.pad_w, yy = (int)py + ky - g.pad_h;
            if ((unsigned)xx < (unsigned)g.W && (unsigned)yy < (unsigned)g.H)
              nmask &= ~(1u << (kx * g.kh + ky));
          }
    }
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)X, (short)0, (int)((int64_t)g.R * xs * 4), 0x00020000);

  // TAB: per k row the byte offset of its tap in a map (kOob past Kdim: out
  // of range; tap index 31 for padded maps, which no lane's mask admits)
  const int KT = T * BK;
  unsigned *ktab = reinterpret_cast<unsigned *>(lds + 2 * BUF);
  unsigned char *ttab = reinterpret_cast<unsigned char *>(ktab + (TAB ? KT : 0));

  // F16: the tile's group scales (sexp) and check weights (sw): entries
  // [0, BG) its rows g, [BG, 384) its columns m; groups past G / M: scale 0,
  // weight -inf (never checked).  A tile with an Inf / NaN group is flagged.
  int *sexp = reinterpret_cast<int *>(lds + 2 * BUF + (TAB ? KT * 4 + (PADDED ? KT : 0) : 0));
  float *sw = reinterpret_cast<float *>(sexp + 384);
  int ea = 0, eb = 0;
  if constexpr (F16) {
    bool bad = false;
    if (tid < 384) {
      uint32_t mx = 0, cnt = 0;
      bool in = false;
      if (tid < BG) {
        const int gg = g0 + tid;
        if (gg < g.G) {
          in = true;
          mx = fx.wst[gg];
          cnt = fx.wst[2 * (size_t)g.G + gg];
        }
      } else {
        const int64_t mm = m0 + (tid - BG);
        if (mm < g.M) {
          uint32_t n, p;
          g.div_P.divmod((uint32_t)mm, n, p);
          in = true;
          mx = fx.xst[n];
          cnt = fx.xst[2 * (size_t)g.R + n];
        }
      }
      const int e = in ? f16x3::scale_exp(mx) : 0;
      bad = e == f16x3::SKIP;
      sexp[tid] = bad ? 0 : e;
      sw[tid] = in && mx != 0 ? f16x3::spread_weight(cnt) : -__builtin_inff();
    }
    if (__syncthreads_or(bad)) {
      if (tid == 0) fx.list[2 + atomicAdd(fx.list, 1u)] = (unsigned)lid;
      return;
    }
    ea = sexp[a_row];
    eb = sexp[BG + b_row];
  }
  if constexpr (TAB) {
    for (int k = tid; k < KT; k += NT) {
      uint32_t c = 0, r = 0, kx = 0, ky = 0;
      if (k < g.Kdim) {
        g.div_khkw.divmod((uint32_t)k, c, r);
        g.div_kh.divmod(r, kx, ky);
      }
      ktab[k] = k < g.Kdim ? (unsigned)((int)c * g.HW + (int)kx * g.H + (int)ky) * 4u : kOob;
      if (PADDED) ttab[k] = (unsigned char)(k < g.Kdim ? kx * g.kh + ky : 31);
    }
    __syncthreads();
  }
  float av[APT], bv[BPT];
  auto load = [&](int kt) {
#pragma unroll
    for (int j = 0; j < APT; j++) {
      // k uniform; the whole offset goes in voffset, which the range check
      // covers (rows past Kdim and columns past the last row read 0)
      const int k = kt * BK + a_kc * APT + j;
      av[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          wr, a_voff + (unsigned)k * (unsigned)ks * 4u, 0, 0));
    }
    const int kb = kt * BK + b_kc * BPT;
    if constexpr (TAB) {
      // the wave's k rows from the LDS table (uniform address: broadcast)
      const int kq = min(kb, KT - BPT);  // a step past T re-reads the last
      unsigned ko[BPT];
#pragma unroll
      for (int q4 = 0; q4 < BPT / 4; q4++) {
        const uint4 v = *reinterpret_cast<const uint4 *>(ktab + kq + 4 * q4);
        ko[4 * q4] = v.x; ko[4 * q4 + 1] = v.y; ko[4 * q4 + 2] = v.z; ko[4 * q4 + 3] = v.w;
      }
      uint32_t tt[PADDED ? BPT / 4 : 1];
      if (PADDED) {
#pragma unroll
        for (int q4 = 0; q4 < BPT / 8; q4++) {
          const uint2 v = *reinterpret_cast<const uint2 *>(ttab + kq + 8 * q4);
          tt[2 * q4] = v.x; tt[2 * q4 + 1] = v.y;
        }
      }
#pragma unroll
      for (int e = 0; e < BPT; e++) {
        unsigned off = xoff4 + ko[e];
        if (PADDED) {
          const unsigned tap = (tt[e >> 2] >> (8 * (e & 3))) & 31u;
          off |= ((nmask >> tap) & 1u) << 31;  // tap 31 (k past Kdim): never inside
        }
        bv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
      }
      return;
    }
    // the k rows of this wave: (c, kx, ky) of the first by division, then
    // stepped (all scalar)
    uint32_t c, r, kx, ky;
    g.div_khkw.divmod((uint32_t)(kb < g.Kdim ? kb : 0), c, r);
    g.div_kh.divmod(r, kx, ky);
#pragma unroll
    for (int e = 0; e < BPT; e++) {
      const int k = kb + e;
      const unsigned ko =
          k < g.Kdim ? (unsigned)((int)c * g.HW + (int)kx * g.H + (int)ky) * 4u : kOob;
      // the whole offset in voffset (range-checked); a tap outside a padded
      // map, a column past M or a row past Kdim lands past the range
      unsigned off = xoff4 + ko;
      if (PADDED) {
        const unsigned tap = kx * (uint32_t)g.kh + ky;
        off = k < g.Kdim ? off | (((nmask >> tap) & 1u) << 31) : kOob;
      }
      bv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
      if (++ky == (uint32_t)g.kh) {
        ky = 0;
        if (++kx == (uint32_t)g.kw) { kx = 0; ++c; }
      }
    }
  };
  const float m1 = F16 ? f16x3::opaque_m1() : -1.0f;
  auto store = [&](char *buf) {
    if constexpr (F16) {
      // A: the pre-split words repacked, hi halves to plane 0, lo to plane 1
#pragma unroll
      for (int cc = 0; cc < APT / 8; cc++) {
        uint32_t hh[4], ll[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t w0 = __float_as_uint(av[8 * cc + 2 * i]);
          const uint32_t w1 = __float_as_uint(av[8 * cc + 2 * i + 1]);
          hh[i] = __builtin_amdgcn_perm(w1, w0, 0x05040100u);
          ll[i] = __builtin_amdgcn_perm(w1, w0, 0x07060302u);
        }
        const int off = swzi(a_row, a_kc * (APT / 8) + cc);
        *reinterpret_cast<uint4 *>(buf + off) = make_uint4(hh[0], hh[1], hh[2], hh[3]);
        *reinterpret_cast<uint4 *>(buf + PLA + off) = make_uint4(ll[0], ll[1], ll[2], ll[3]);
      }
      (void)ea;
#pragma unroll
      for (int cc = 0; cc < BPT / 8; cc++)
        put8h(buf + 2 * PLA, PLB, swzi(b_row, b_kc * (BPT / 8) + cc), &bv[8 * cc], eb, m1);
    } else {
#pragma unroll
      for (int cc = 0; cc < APT / 8; cc++)
        put8(buf, PLA, swzi(a_row, a_kc * (APT / 8) + cc), &av[8 * cc]);
#pragma unroll
      for (int cc = 0; cc < BPT / 8; cc++)
        put8(buf + 3 * PLA, PLB, swzi(b_row, b_kc * (BPT / 8) + cc), &bv[8 * cc]);
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = x6::zero16();

  if (T > 0) {
    load(0);
    store(lds);
    __syncthreads();
    if (T > 1) load(1);
  }
  const int ar = wm * 64 + l, br = wn * 64 + l;
  // one k16 half of a step: 12 fragment reads, 24 MFMAs
  auto half_step = [&](const char *bufA, int s) {
    const int c = 2 * s + h;
    if constexpr (F16) {  // 8 fragment reads, 12 MFMAs
      const char *bufB = bufA + 2 * PLA;
      f16x3::f16x8 a[2][2], bb[2][2];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int pl = 0; pl < 2; pl++) {
          a[i][pl] = *reinterpret_cast<const f16x3::f16x8 *>(bufA + pl * PLA + swzi(ar + 32 * i, c));
          bb[i][pl] = *reinterpret_cast<const f16x3::f16x8 *>(bufB + pl * PLB + swzi(br + 32 * i, c));
        }
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          acc[i][j] = f16x3::mfma3(a[i][0], a[i][1], bb[j][0], bb[j][1], acc[i][j]);
      return;
    }
    const char *bufB = bufA + 3 * PLA;
    x6::bf16x8 a[2][3], bb[2][3];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int pl = 0; pl < 3; pl++) {
        a[i][pl] = *reinterpret_cast<const x6::bf16x8 *>(bufA + pl * PLA + swzi(ar + 32 * i, c));
        bb[i][pl] = *reinterpret_cast<const x6::bf16x8 *>(bufB + pl * PLB + swzi(br + 32 * i, c));
      }
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = x6::mfma6(a[i], bb[j], acc[i][j]);
  };
  // STG: waves 4-7 split the next step's operands between their two MFMA
  // halves, waves 0-3 after both, so the two waves of a SIMD (w, w + 4)
  // alternate their vector and matrix phases instead of running them at once
  const bool late = !STG || wave < 4;
  for (int t = 0; t < T; t++) {
    const char *buf = lds + (t & 1) * BUF;
    half_step(buf, 0);
    if (!late && t + 1 < T) store(lds + ((t + 1) & 1) * BUF);
    half_step(buf, 1);
    if (late && t + 1 < T) store(lds + ((t + 1) & 1) * BUF);
    if (t + 2 < T) load(t + 2);
    __syncthreads();
  }

  // epilogue: accumulator r of lane (l, h) is row g0 + wm*64 + 32i +
  // mfma32_row(r), column m0 + wn*64 + 32j + l; concat layout + bias (+ReLU)
  uint64_t rej = 0;  // F16: rejected elements, bit 16 (2i + j) + r
  if constexpr (F16) {
    // the store check (f16-split.h: a scaled sum of at least the groups'
    // spread weights keeps its small elements' error under 2^-19 of itself),
    // then the exact unscale
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int cl = BG + wn * 64 + 32 * j + l;
      const int ec = sexp[cl];
      const float wc = sw[cl];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int rl = wm * 64 + 32 * i + mfma32_row(r, lane);
          const float v = acc[i][j][r];
          if (fabsf(v) < sw[rl] + wc) rej |= 1ull << (16 * (2 * i + j) + r);
          acc[i][j][r] = __builtin_amdgcn_ldexpf(v, -(sexp[rl] + ec));
        }
    }
    int nrej = __builtin_popcountll(rej);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nrej += __shfl_xor(nrej, d);
    if (__syncthreads_or(nrej > REJ_MAX)) {
      if (tid == 0) fx.list[2 + atomicAdd(fx.list, 1u)] = (unsigned)lid;
      return;
    }
  }
  if constexpr (POOL > 0) {
    constexpr int PC = POOL == 1 ? 4 : POOL == 2 ? 1 : 2;
    const int Q = g.P >> 1;  // pooled positions per map
    const int d = l & 1;     // this lane's position in its window
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int64_t mm = m0 + wn * 64 + 32 * j + l;
      const bool mv = mm < g.M;  // both lanes of a window alike (P even)
      uint32_t on = 0, op = 0;
      if (mv) g.div_P.divmod((uint32_t)mm, on, op);
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += PC) {
          const int gg0 = g0 + wm * 64 + 32 * i + mfma32_row(r0, lane);
          const bool gv = gg0 < g.G;  // G % PC == 0: a group is all in or all out
          float v[PC], w[PC];
#pragma unroll
          for (int c = 0; c < PC; c++) {
            float x = acc[i][j][r0 + c];
            if (bias && gv) x = x + bias[gg0 + c];
            v[c] = x;
          }
#pragma unroll
          for (int c = 0; c < PC; c++) w[c] = __shfl_xor(v[c], 1);
          if (out && mv && gv) {
#pragma unroll
            for (int c = 0; c < PC; c++) out[(int64_t)on * os + (int64_t)(gg0 + c) * g.P + op] = v[c];
          }
          // A.8's order and compare: maps c, then the window's two
          // positions; the mask bit of each element equal to the max
          float mx = -1e20f;
#pragma unroll
          for (int c = 0; c < PC; c++) {
            const float e0 = d ? w[c] : v[c], e1 = d ? v[c] : w[c];
            if (mx < e0) mx = e0;
            if (mx < e1) mx = e1;
          }
          unsigned mk = 0;
#pragma unroll
          for (int c = 0; c < PC; c++) {
            const float e0 = d ? w[c] : v[c], e1 = d ? v[c] : w[c];
            mk |= (e0 == mx ? 1u : 0u) << (2 * c);
            mk |= (e1 == mx ? 1u : 0u) << (2 * c + 1);
          }
          if (d == 0 && mv && gv) {
            const int64_t q = (int64_t)(gg0 / PC) * Q + (op >> 1);
            po.pool[(int64_t)on * po.ps + q] = mx;
            po.mask[(int64_t)on * po.ms + q] = (unsigned short)mk;
          }
          if constexpr (F16) {  // a window holding a rejected element: listed
            const unsigned rm = (unsigned)(rej >> (16 * (2 * i + j) + r0)) & ((1u << PC) - 1u);
            const unsigned rp = (unsigned)__shfl_xor((int)rm, 1);
            if (d == 0 && mv && gv && (rm | rp)) {
              unsigned bits = 0;
#pragma unroll
              for (int c = 0; c < PC; c++)
                bits |= ((rm >> c) & 1u) << (2 * c) | ((rp >> c) & 1u) << (2 * c + 1);
              unsigned *e = fx.elist + (size_t)EW * atomicAdd(fx.list + 1, 1u);
              e[0] = (unsigned)gg0;
              e[1] = (unsigned)mm;
              e[2] = bits;
#pragma unroll
              for (int c = 0; c < PC; c++) {
                e[3 + 2 * c] = __float_as_uint(v[c]);
                e[4 + 2 * c] = __float_as_uint(w[c]);
              }
            }
          }
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int64_t mm = m0 + wn * 64 + 32 * j + l;
    if (mm >= g.M) continue;
    uint32_t on, op;
    g.div_P.divmod((uint32_t)mm, on, op);
    float *orow = out + (int64_t)on * os + op;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int gg = g0 + wm * 64 + 32 * i + mfma32_row(r, lane);
        if (gg >= g.G) continue;
        float v = acc[i][j][r];
        if (bias) v = v + bias[gg];
        if (relu) v = v < 0.0f ? 0.0f : v;  // RectifiedLinear: ApplyFloor(0)
        orow[(int64_t)gg * g.P] = v;
      }
  }
  if constexpr (F16) {
    while (rej) {  // (rare) this lane's rejected elements, listed
      const int b = __builtin_ctzll(rej);
      rej &= rej - 1;
      const int i = b >> 5, j = (b >> 4) & 1, r = b & 15;
      const int gg = g0 + wm * 64 + 32 * i + mfma32_row(r, lane);
      const int64_t mm = m0 + wn * 64 + 32 * j + l;
      if (gg >= g.G || mm >= g.M) continue;
      unsigned *e = fx.elist + (size_t)EW * atomicAdd(fx.list + 1, 1u);
      e[0] = (unsigned)gg;
      e[1] = (unsigned)mm;
      e[2] = 1u;
    }
  }
}

// The listed tiles of the f16x3 form in fp32 (F16Aux): work item it = (the
// list's tile it / 256, chunk it % 256), a chunk being 8 rows g x 16
// columns m of a BG x BN tile (BG = 256: 32 x 8 chunks; 128: 16 x 16), so
// it holds whole pool windows (PC | 8 consecutive filters, column pairs m, m
// + 1 with m even).  Each of the 4 waves computes 32 of its elements
// (conv_dot) into LDS, then they are stored (+ bias, ReLU) or pooled with
// the epilogue's order and compares.  A grid of at most 256 blocks walks
// the items; with an empty list every block leaves at once.
template <int BG, int POOL>
__global__ __launch_bounds__(256) void conv_igemm_fixup_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ Kw, int ks,
    const float *__restrict__ bias, float *__restrict__ out, int os, int relu, PoolOut po,
    const unsigned *__restrict__ list) {
  constexpr int BN = 384 - BG, CC = BN / 16;  // column chunks per tile
  __shared__ float val[8][17];
  const unsigned nitems = list[0] * 256u;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_g = (g.G + BG - 1) / BG;
  for (unsigned it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int lid = (int)list[2 + it / 256], ch = (int)(it % 256);
    const int g0 = (lid % tiles_g) * BG + (ch / CC) * 8;
    const int64_t m0 = (int64_t)(lid / tiles_g) * BN + (int64_t)(ch % CC) * 16;
    for (int e = wave; e < 128; e += 4) {
      const int gg = g0 + (e >> 4);
      const int64_t mm = m0 + (e & 15);
      float v = 0.0f;
      if (gg < g.G && mm < g.M) v = conv_dot(g, X, xs, Kw, ks, gg, mm, lane);
      if (lane == 0) val[e >> 4][e & 15] = v;
    }
    __syncthreads();
    if constexpr (POOL > 0) {
      constexpr int PC = POOL == 1 ? 4 : POOL == 2 ? 1 : 2;
      const int Q = g.P >> 1;
      if (tid < 64) {  // window (8 / PC filter groups) x (8 column pairs)
        const int wg = tid >> 3, wp = tid & 7;
        const int gg0 = g0 + wg * PC;
        const int64_t mm = m0 + 2 * wp;
        if (wg < 8 / PC && gg0 < g.G && mm < g.M) {
          uint32_t on, op;
          g.div_P.divmod((uint32_t)mm, on, op);
          float e0[PC], e1[PC];
#pragma unroll
          for (int c = 0; c < PC; c++) {
            e0[c] = val[wg * PC + c][2 * wp];
            e1[c] = val[wg * PC + c][2 * wp + 1];
            if (bias) {
              e0[c] = e0[c] + bias[gg0 + c];
              e1[c] = e1[c] + bias[gg0 + c];
            }
            if (out) {
              out[(int64_t)on * os + (int64_t)(gg0 + c) * g.P + op] = e0[c];
              out[(int64_t)on * os + (int64_t)(gg0 + c) * g.P + op + 1] = e1[c];
            }
          }
          float mx = -1e20f;
#pragma unroll
          for (int c = 0; c < PC; c++) {
            if (mx < e0[c]) mx = e0[c];
            if (mx < e1[c]) mx = e1[c];
          }
          unsigned mk = 0;
#pragma unroll
          for (int c = 0; c < PC; c++) {
            mk |= (e0[c] == mx ? 1u : 0u) << (2 * c);
            mk |= (e1[c] == mx ? 1u : 0u) << (2 * c + 1);
          }
          const int64_t q = (int64_t)(gg0 / PC) * Q + (op >> 1);
          po.pool[(int64_t)on * po.ps + q] = mx;
          po.mask[(int64_t)on * po.ms + q] = (unsigned short)mk;
        }
      }
    } else if (tid < 128) {
      const int gg = g0 + (tid >> 4);
      const int64_t mm = m0 + (tid & 15);
      if (gg < g.G && mm < g.M) {
        uint32_t on, op;
        g.div_P.divmod((uint32_t)mm, on, op);
        float v = val[tid >> 4][tid & 15];
        if (bias) v = v + bias[gg];
        if (relu) v = v < 0.0f ? 0.0f : v;
        out[(int64_t)on * os + (int64_t)gg * g.P + op] = v;
      }
    }
    __syncthreads();  // val is rewritten by the next item
  }
}

// The listed elements of the f16x3 form (F16Aux elist), one entry per wave:
// the rejected element recomputed (conv_dot) and stored (+ bias, ReLU), or,
// for the pooled epilogue, the window's rejected elements recomputed (+ bias)
// and the window pooled again with the epilogue's order and compares.
// Cumulative fix-up counts of the f16x3 form since the last reset (listed
// tiles, listed elements), read by kcnn_conv_fix_counts: the tests' evidence
// that a full-size call took the fix-up paths (one atomic pair per call).
__device__ unsigned long long g_igemm_fix_counts[2];

template <int POOL>
__global__ __launch_bounds__(256) void conv_igemm_efix_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ Kw, int ks,
    const float *__restrict__ bias, float *__restrict__ out, int os, int relu, PoolOut po,
    const unsigned *__restrict__ list, const unsigned *__restrict__ elist) {
  const unsigned n = list[1];
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&g_igemm_fix_counts[0], (unsigned long long)list[0]);
    atomicAdd(&g_igemm_fix_counts[1], (unsigned long long)n);
  }
  const unsigned w0 = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (unsigned en = w0; en < n; en += nw) {
    const unsigned *e = elist + (size_t)EW * en;
    const int gg0 = (int)e[0];
    const int64_t mm = (int64_t)e[1];
    const unsigned bits = e[2];
    uint32_t on, op;
    g.div_P.divmod((uint32_t)mm, on, op);
    if constexpr (POOL > 0) {
      constexpr int PC = POOL == 1 ? 4 : POOL == 2 ? 1 : 2;
      const int Q = g.P >> 1;
      float v[2 * PC];
#pragma unroll
      for (int b = 0; b < 2 * PC; b++) {
        v[b] = __uint_as_float(e[3 + b]);
        if ((bits >> b) & 1u) {  // wave-uniform
          const int gg = gg0 + (b >> 1);
          float x = conv_dot(g, X, xs, Kw, ks, gg, mm + (b & 1), lane);
          if (bias) x = x + bias[gg];
          v[b] = x;
          if (out && lane == 0) out[(int64_t)on * os + (int64_t)gg * g.P + op + (b & 1)] = x;
        }
      }
      float mx = -1e20f;
#pragma unroll
      for (int c = 0; c < PC; c++) {
        if (mx < v[2 * c]) mx = v[2 * c];
        if (mx < v[2 * c + 1]) mx = v[2 * c + 1];
      }
      unsigned mk = 0;
#pragma unroll
      for (int c = 0; c < PC; c++) {
        mk |= (v[2 * c] == mx ? 1u : 0u) << (2 * c);
        mk |= (v[2 * c + 1] == mx ? 1u : 0u) << (2 * c + 1);
      }
      if (lane == 0) {
        const int64_t q = (int64_t)(gg0 / PC) * Q + (op >> 1);
        po.pool[(int64_t)on * po.ps + q] = mx;
        po.mask[(int64_t)on * po.ms + q] = (unsigned short)mk;
      }
    } else {
      float x = conv_dot(g, X, xs, Kw, ks, gg0, mm, lane);
      if (bias) x = x + bias[gg0];
      if (relu) x = x < 0.0f ? 0.0f : x;
      if (lane == 0) out[(int64_t)on * os + (int64_t)gg0 * g.P + op] = x;
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient (ConvolutionComponent::Update's TpBlock(X) conv
// TpInsideBlock(dY) + ModPermuteRow, nnet-component-nnet0.cc:738-765,
// Appendix A.12) on the bf16 MFMAs:
//   gW[g][k] = sum_t dY[n][g*P + p] im2col(X)[t][k],  gb[g] = sum_t dY[n][g*P + p]
// over t = n*P + p of a split's frames: C[g][k] = A[g][t] B[k][t], rows g in
// a tile of 256, columns k in a tile of 128, the reduction t flattened over
// the split's frames in steps of 32 (no padding of P to a chunk length).
// Thread (tp, r) = (tid % 16, tid / 16) loads the t pair 2tp, 2tp + 1 of A
// rows r + 32j (j < 8) and B rows r + 32j (j < 4): lanes along t, so a wave
// reads 128-B runs of dY and of the X map; each pair splits into one packed
// bf16 pair per plane (a 4-B LDS write).  The split's frame range is the
// range of the two buffer descriptors, so t past the split reads 0.  The
// k-tile-0 blocks also sum dY for the bias gradient (fixed order).  Partials
// go to ws[split][g*Kdim + k] (then the G bias entries), reduced in a fixed
// order by kcnn_reduce_splits_wgrad: deterministic.
template <bool PADDED, bool STG>
__global__ __launch_bounds__(NT, 1) void conv_wgrad_x6_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dY, int dys,
    float *__restrict__ ws, int fps, int ktiles, int nblocks) {
  constexpr int BG = 256, BN = 128;
  constexpr int PLA = BG * ROWB, PLB = BN * ROWB, BUF = 3 * (PLA + PLB);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // XCD-aware order: logical ids contiguous per XCD, so the tiles of one
  // split (the same frames) share an L2
  const int nb8 = (nblocks + 7) >> 3;
  const int bid = (int)(blockIdx.x & 7) * nb8 + (int)(blockIdx.x >> 3);
  if (bid >= nblocks) return;  // whole workgroup: no barrier is skipped
  const int ntiles = ktiles * ((g.G + BG - 1) / BG);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int k0 = (tile % ktiles) * BN, g0 = (tile / ktiles) * BG;
  const int nbeg = split * fps;
  const int nf = min(g.R, nbeg + fps) - nbeg;  // frames of this split (>= 1)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int l = lane & 31, h = lane >> 5;
  const int tp = tid & 15, r = tid >> 4;

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(dY + (int64_t)nbeg * dys), (short)0, nf * dys * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(X + (int64_t)nbeg * xs), (short)0, nf * xs * 4, 0x00020000);
  // this thread's B rows k = k0 + r + 32j: map offset of the tap, its
  // (kx, ky) for padded maps; rows past Kdim read 0
  unsigned koff4[4];
  int tkx[PADDED ? 4 : 1], tky[PADDED ? 4 : 1];
  bool kval[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = k0 + r + 32 * j;
    uint32_t c = 0, rr = 0, kx = 0, ky = 0;
    kval[j] = k < g.Kdim;
    if (kval[j]) {
      g.div_khkw.divmod((uint32_t)k, c, rr);
      g.div_kh.divmod(rr, kx, ky);
    }
    koff4[j] = (unsigned)((int)c * g.HW + (int)kx * g.H + (int)ky) * 4u;
    if (PADDED) { tkx[j] = (int)kx - g.pad_w; tky[j] = (int)ky - g.pad_h; }
  }
  const int nsteps = (nf * g.P + BK - 1) / BK;

  float av[8][2], bv[4][2], bsum[8];
#pragma unroll
  for (int j = 0; j < 8; j++) bsum[j] = 0.0f;
  const bool do_bias = k0 == 0;
  auto load = [&](int st) {
    // t pair (t0, t0 + 1) -> (n, p) and map position (px, py) of each
    const uint32_t t0 = (uint32_t)(st * BK + 2 * tp);
    uint32_t n0, p0, px0, py0;
    g.div_P.divmod(t0, n0, p0);
    g.div_oh.divmod(p0, px0, py0);
    uint32_t n1 = n0, p1 = p0 + 1, px1 = px0, py1 = py0 + 1;
    if (py1 == (uint32_t)g.oh) { py1 = 0; ++px1; }
    if (p1 == (uint32_t)g.P) { p1 = 0; px1 = 0; py1 = 0; ++n1; }
    const uint32_t nn[2] = {n0, n1}, pp[2] = {p0, p1}, pxs[2] = {px0, px1}, pys[2] = {py0, py1};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      // past the split: n >= nf, every offset lands past the range
      const unsigned a4 = (nn[e] * (unsigned)dys + pp[e]) * 4u;
#pragma unroll
      for (int j = 0; j < 8; j++)
        av[j][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            ar, a4 + (unsigned)((g0 + r + 32 * j) * g.P) * 4u, 0, 0));
      const int xo = (int)(nn[e] * (unsigned)xs) + ((int)pxs[e] - g.pad_w) * g.H +
                     (int)pys[e] - g.pad_h;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        unsigned off = (unsigned)xo * 4u + koff4[j];
        if (PADDED) {
          const bool in = (unsigned)((int)pxs[e] + tkx[j]) < (unsigned)g.W &&
                          (unsigned)((int)pys[e] + tky[j]) < (unsigned)g.H;
          off = in ? off : kOob;
        }
        off = kval[j] ? off : kOob;
        bv[j][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, off, 0, 0));
      }
    }
  };
  auto store = [&](char *buf) {
    // pair (t0, t0 + 1) of row q: bytes 2*(t0 % 8) of chunk t0 / 8
    const int tc = (2 * tp) >> 3, tb = ((2 * tp) & 7) * 2;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t hh, mm, ll;
      x6::split2(av[j][0], av[j][1], hh, mm, ll);
      const int o = swz(r + 32 * j, tc) + tb;
      *reinterpret_cast<uint32_t *>(buf + o) = hh;
      *reinterpret_cast<uint32_t *>(buf + PLA + o) = mm;
      *reinterpret_cast<uint32_t *>(buf + 2 * PLA + o) = ll;
      if (do_bias) bsum[j] += av[j][0] + av[j][1];
    }
    char *bb = buf + 3 * PLA;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t hh, mm, ll;
      x6::split2(bv[j][0], bv[j][1], hh, mm, ll);
      const int o = swz(r + 32 * j, tc) + tb;
      *reinterpret_cast<uint32_t *>(bb + o) = hh;
      *reinterpret_cast<uint32_t *>(bb + PLB + o) = mm;
      *reinterpret_cast<uint32_t *>(bb + 2 * PLB + o) = ll;
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = x6::zero16();
  load(0);
  store(lds);
  __syncthreads();
  if (nsteps > 1) load(1);
  const int arow = wm * 64 + l, brow = wn * 64 + l;
  auto half_step = [&](const char *bufA, int s) {
    const char *bufB = bufA + 3 * PLA;
    x6::bf16x8 a[2][3], bb[2][3];
    const int c = 2 * s + h;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int pl = 0; pl < 3; pl++) {
        a[i][pl] = *reinterpret_cast<const x6::bf16x8 *>(bufA + pl * PLA + swz(arow + 32 * i, c));
        bb[i][pl] = *reinterpret_cast<const x6::bf16x8 *>(bufB + pl * PLB + swz(brow + 32 * i, c));
      }
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[i][j] = x6::mfma6(a[i], bb[j], acc[i][j]);
  };
  const bool late = !STG || wave < 4;  // as in conv_igemm_x6_kernel
  for (int t = 0; t < nsteps; t++) {
    const char *buf = lds + (t & 1) * BUF;
    half_step(buf, 0);
    if (!late && t + 1 < nsteps) store(lds + ((t + 1) & 1) * BUF);
    half_step(buf, 1);
    if (late && t + 1 < nsteps) store(lds + ((t + 1) & 1) * BUF);
    if (t + 2 < nsteps) load(t + 2);
    __syncthreads();
  }

  // partials of this split: gW (lanes along k: 128-B runs), then the bias
  const int64_t E = (int64_t)g.G * g.Kdim + g.G;
  float *wsp = ws + (int64_t)split * E;
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int kk = k0 + wn * 64 + 32 * j + l;
    if (kk >= g.Kdim) continue;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int gg = g0 + wm * 64 + 32 * i + mfma32_row(q, lane);
        if (gg < g.G) wsp[(int64_t)gg * g.Kdim + kk] = acc[i][j][q];
      }
  }
  if (do_bias) {
    // row r + 32j's 16 t-lane sums, added in lane order through LDS (the
    // last barrier of the loop ended every read of the images)
    float *red = reinterpret_cast<float *>(lds);  // [256][17]
#pragma unroll
    for (int j = 0; j < 8; j++) red[(r + 32 * j) * 17 + tp] = bsum[j];
    __syncthreads();
    if (tid < BG && g0 + tid < g.G) {
      float sum = 0.0f;
      for (int i = 0; i < 16; i++) sum += red[tid * 17 + i];
      wsp[(int64_t)g.G * g.Kdim + g0 + tid] = sum;
    }
  }
}

// Weight gradient, wide tiles: 256 (g) x 256 (k) per workgroup and t steps
// of 16, so each dY value a workgroup loads and splits feeds twice the MFMAs
// of conv_wgrad_x6_kernel (the split's vector work per MFMA drops by a
// third).  Images of 32-B rows (16 t), the two 16-B chunks of a row swapped
// on rows 8-15 of every 16 (conflict-free fragment reads), 2 x 48 KB.  Waves
// 4 (g) x 2 (k), each 64 x 128: 2 x 4 accumulators.  Thread (tp, r) = (tid %
// 8, tid / 8) loads the t pair (2tp, 2tp + 1) of A and B rows r + 64j.
// Same split plan, partial layout, bias sums and fixed-order reduction as
// conv_wgrad_x6_kernel.
constexpr int WROW = 32;  // bytes per image row (16 bf16)
__device__ __forceinline__ int swz32(int r, int c) {
  return r * WROW + ((c ^ ((r >> 3) & 1)) << 4);
}

// The f16x3 form of the wide weight gradient (F16, wgrad_x6 family 3; not
// the default: on c5 it measured slower than the bf16x6 form): scale groups over the whole batch -- a filter g
// (dY's columns g*P .. g*P + P - 1 of every frame) and an input channel c (X's
// columns c*HW .. c*HW + HW - 1 of every frame, a superset of every tap of
// that channel) -- from wgrad_group_stats_kernel.  A split's partial of
// (g, k) is checked like the implicit GEMM's store; a rejected one is listed
// (elist: split, g, k) and recomputed over the split's frames in fp32
// (conv_wgrad_efix_kernel); a block with an Inf / NaN group or a wave of
// more than REJ_MAX rejections flags itself (flags[bid]) and the bf16x6 form
// then recomputes exactly the flagged blocks (redo).
struct WF16 {
  const uint32_t *gst;   // [max G][min G][cnt G] of dY's filter groups
  const uint32_t *cst;   // [max C][min C][cnt C] of X's channel groups
  unsigned *flags;       // F16: per block, 1 = recompute on bf16x6
  const unsigned *redo;  // bf16x6 form: non-null = only the flagged blocks
  unsigned *list;        // [element count]
  unsigned *elist;       // entries (split, g, k)
};

template <bool PADDED, bool F16>
__global__ __launch_bounds__(NT, 1) void conv_wgrad_x6w_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dY, int dys,
    float *__restrict__ ws, int fps, int ktiles, int nblocks, WF16 wf) {
  constexpr int BG = 256, BN = 256, BT = 16;
  constexpr int NPL = F16 ? 2 : 3;
  constexpr int PLA = BG * WROW, PLB = BN * WROW, BUF = NPL * (PLA + PLB);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int nb8 = (nblocks + 7) >> 3;
  const int bid = (int)(blockIdx.x & 7) * nb8 + (int)(blockIdx.x >> 3);
  if (bid >= nblocks) return;  // whole workgroup: no barrier is skipped
  if constexpr (!F16) {
    if (wf.redo && wf.redo[bid] == 0) return;  // (uniform) the f16x3 partial stands
  }
  const int ntiles = ktiles * ((g.G + BG - 1) / BG);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int k0 = (tile % ktiles) * BN, g0 = (tile / ktiles) * BG;
  const int nbeg = split * fps;
  const int nf = min(g.R, nbeg + fps) - nbeg;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int l = lane & 31, h = lane >> 5;
  const int tp = tid & 7, r = tid >> 3;

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(dY + (int64_t)nbeg * dys), (short)0, nf * dys * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(X + (int64_t)nbeg * xs), (short)0, nf * xs * 4, 0x00020000);
  unsigned koff4[4];
  int tkx[PADDED ? 4 : 1], tky[PADDED ? 4 : 1];
  bool kval[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = k0 + r + 64 * j;
    uint32_t c = 0, rr = 0, kx = 0, ky = 0;
    kval[j] = k < g.Kdim;
    if (kval[j]) {
      g.div_khkw.divmod((uint32_t)k, c, rr);
      g.div_kh.divmod(rr, kx, ky);
    }
    koff4[j] = (unsigned)((int)c * g.HW + (int)kx * g.H + (int)ky) * 4u;
    if (PADDED) { tkx[j] = (int)kx - g.pad_w; tky[j] = (int)ky - g.pad_h; }
  }
  const int nsteps = (nf * g.P + BT - 1) / BT;

  // F16: scale exponents / check weights of the block's 256 filters (sx[0,
  // 256)) and 256 k columns (sx[256, 512), by their channel) in LDS past the
  // images; a block with an Inf / NaN group is flagged for the bf16x6 form
  int *sx = reinterpret_cast<int *>(lds + 2 * BUF);
  float *swt = reinterpret_cast<float *>(sx + 512);
  int ea[4] = {0, 0, 0, 0}, eb[4] = {0, 0, 0, 0};
  if constexpr (F16) {
    uint32_t mx = 0, cnt = 0;
    bool in = false;
    if (tid < 256) {
      const int gg = g0 + tid;
      if (gg < g.G) { in = true; mx = wf.gst[gg]; cnt = wf.gst[2 * g.G + gg]; }
    } else {
      const int k = k0 + tid - 256;
      if (k < g.Kdim) {
        uint32_t c, rr;
        g.div_khkw.divmod((uint32_t)k, c, rr);
        in = true;
        mx = wf.cst[c];
        cnt = wf.cst[2 * g.C + c];
      }
    }
    const int e = in ? f16x3::scale_exp(mx) : 0;
    const bool bad = e == f16x3::SKIP;
    sx[tid] = bad ? 0 : e;
    swt[tid] = in && mx != 0 ? f16x3::spread_weight(cnt) : -__builtin_inff();
    if (__syncthreads_or(bad)) {
      if (tid == 0) wf.flags[bid] = 1u;
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      ea[j] = sx[r + 64 * j];
      eb[j] = sx[256 + r + 64 * j];
    }
  }

  float av[4][2], bv[4][2], bsum[4];
#pragma unroll
  for (int j = 0; j < 4; j++) bsum[j] = 0.0f;
  const bool do_bias = k0 == 0;
  auto load = [&](int st) {
    const uint32_t t0 = (uint32_t)(st * BT + 2 * tp);
    uint32_t n0, p0, px0, py0;
    g.div_P.divmod(t0, n0, p0);
    g.div_oh.divmod(p0, px0, py0);
    uint32_t n1 = n0, p1 = p0 + 1, px1 = px0, py1 = py0 + 1;
    if (py1 == (uint32_t)g.oh) { py1 = 0; ++px1; }
    if (p1 == (uint32_t)g.P) { p1 = 0; px1 = 0; py1 = 0; ++n1; }
    const uint32_t nn[2] = {n0, n1}, pp[2] = {p0, p1}, pxs[2] = {px0, px1}, pys[2] = {py0, py1};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const unsigned a4 = (nn[e] * (unsigned)dys + pp[e]) * 4u;
#pragma unroll
      for (int j = 0; j < 4; j++)
        av[j][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            ar, a4 + (unsigned)((g0 + r + 64 * j) * g.P) * 4u, 0, 0));
      const int xo = (int)(nn[e] * (unsigned)xs) + ((int)pxs[e] - g.pad_w) * g.H +
                     (int)pys[e] - g.pad_h;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        unsigned off = (unsigned)xo * 4u + koff4[j];
        if (PADDED) {
          const bool in = (unsigned)((int)pxs[e] + tkx[j]) < (unsigned)g.W &&
                          (unsigned)((int)pys[e] + tky[j]) < (unsigned)g.H;
          off = in ? off : kOob;
        }
        off = kval[j] ? off : kOob;
        bv[j][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, off, 0, 0));
      }
    }
  };
  const int tc = tp >> 2, tb = (tp & 3) * 4;  // pair (2tp, 2tp+1): chunk, byte
  const float m1 = F16 ? f16x3::opaque_m1() : -1.0f;
  auto store = [&](char *buf) {
    if constexpr (F16) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t hh, ll;
        f16x3::split2h(av[j][0], av[j][1], ea[j], ea[j], hh, ll, m1);
        const int o = swz32(r + 64 * j, tc) + tb;
        *reinterpret_cast<uint32_t *>(buf + o) = hh;
        *reinterpret_cast<uint32_t *>(buf + PLA + o) = ll;
        if (do_bias) bsum[j] += av[j][0] + av[j][1];
      }
      char *bb = buf + 2 * PLA;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t hh, ll;
        f16x3::split2h(bv[j][0], bv[j][1], eb[j], eb[j], hh, ll, m1);
        const int o = swz32(r + 64 * j, tc) + tb;
        *reinterpret_cast<uint32_t *>(bb + o) = hh;
        *reinterpret_cast<uint32_t *>(bb + PLB + o) = ll;
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t hh, mm, ll;
      x6::split2(av[j][0], av[j][1], hh, mm, ll);
      const int o = swz32(r + 64 * j, tc) + tb;
      *reinterpret_cast<uint32_t *>(buf + o) = hh;
      *reinterpret_cast<uint32_t *>(buf + PLA + o) = mm;
      *reinterpret_cast<uint32_t *>(buf + 2 * PLA + o) = ll;
      if (do_bias) bsum[j] += av[j][0] + av[j][1];
    }
    char *bb = buf + 3 * PLA;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t hh, mm, ll;
      x6::split2(bv[j][0], bv[j][1], hh, mm, ll);
      const int o = swz32(r + 64 * j, tc) + tb;
      *reinterpret_cast<uint32_t *>(bb + o) = hh;
      *reinterpret_cast<uint32_t *>(bb + PLB + o) = mm;
      *reinterpret_cast<uint32_t *>(bb + 2 * PLB + o) = ll;
    }
  };

  floatx16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = x6::zero16();
  load(0);
  store(lds);
  __syncthreads();
  if (nsteps > 1) load(1);
  const int arow = wm * 64 + l, brow = wn * 128 + l;
  for (int t = 0; t < nsteps; t++) {
    if constexpr (F16) {
      const char *bufA = lds + (t & 1) * BUF;
      const char *bufB = bufA + 2 * PLA;
      f16x3::f16x8 a[2][2];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int pl = 0; pl < 2; pl++)
          a[i][pl] = *reinterpret_cast<const f16x3::f16x8 *>(bufA + pl * PLA + swz32(arow + 32 * i, h));
#pragma unroll
      for (int j = 0; j < 4; j++) {
        f16x3::f16x8 bb[2];
#pragma unroll
        for (int pl = 0; pl < 2; pl++)
          bb[pl] = *reinterpret_cast<const f16x3::f16x8 *>(bufB + pl * PLB + swz32(brow + 32 * j, h));
#pragma unroll
        for (int i = 0; i < 2; i++) acc[i][j] = f16x3::mfma3(a[i][0], a[i][1], bb[0], bb[1], acc[i][j]);
      }
      if (t + 1 < nsteps) {
        store(lds + ((t + 1) & 1) * BUF);
        if (t + 2 < nsteps) load(t + 2);
      }
      __syncthreads();
      continue;
    }
    const char *bufA = lds + (t & 1) * BUF;
    const char *bufB = bufA + 3 * PLA;
    x6::bf16x8 a[2][3];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int pl = 0; pl < 3; pl++)
        a[i][pl] = *reinterpret_cast<const x6::bf16x8 *>(bufA + pl * PLA + swz32(arow + 32 * i, h));
#pragma unroll
    for (int j = 0; j < 4; j++) {
      x6::bf16x8 bb[3];
#pragma unroll
      for (int pl = 0; pl < 3; pl++)
        bb[pl] = *reinterpret_cast<const x6::bf16x8 *>(bufB + pl * PLB + swz32(brow + 32 * j, h));
#pragma unroll
      for (int i = 0; i < 2; i++) acc[i][j] = x6::mfma6(a[i], bb, acc[i][j]);
    }
    if (t + 1 < nsteps) {
      store(lds + ((t + 1) & 1) * BUF);
      if (t + 2 < nsteps) load(t + 2);
    }
    __syncthreads();
  }

  const int64_t E = (int64_t)g.G * g.Kdim + g.G;
  float *wsp = ws + (int64_t)split * E;
  uint64_t rej[2] = {0, 0};  // F16: bit 16 j + q of word i
  if constexpr (F16) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int kl = 256 + wn * 128 + 32 * j + l;
      const int ec = sx[kl];
      const float wc = swt[kl];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int gl = wm * 64 + 32 * i + mfma32_row(q, lane);
          const float v = acc[i][j][q];
          if (fabsf(v) < swt[gl] + wc) rej[i] |= 1ull << (16 * j + q);
          acc[i][j][q] = __builtin_amdgcn_ldexpf(v, -(sx[gl] + ec));
        }
    }
    int nrej = __builtin_popcountll(rej[0]) + __builtin_popcountll(rej[1]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nrej += __shfl_xor(nrej, d);
    const int f = __syncthreads_or(nrej > REJ_MAX);
    if (tid == 0) wf.flags[bid] = f ? 1u : 0u;
    if (f) return;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int kk = k0 + wn * 128 + 32 * j + l;
    if (kk >= g.Kdim) continue;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int gg = g0 + wm * 64 + 32 * i + mfma32_row(q, lane);
        if (gg < g.G) wsp[(int64_t)gg * g.Kdim + kk] = acc[i][j][q];
      }
  }
  if constexpr (F16) {
#pragma unroll
    for (int i = 0; i < 2; i++)
      while (rej[i]) {  // (rare) this lane's rejected partials, listed
        const int b = __builtin_ctzll(rej[i]);
        rej[i] &= rej[i] - 1;
        const int j = b >> 4, q = b & 15;
        const int gg = g0 + wm * 64 + 32 * i + mfma32_row(q, lane);
        const int kk = k0 + wn * 128 + 32 * j + l;
        if (gg >= g.G || kk >= g.Kdim) continue;
        unsigned *e = wf.elist + 3 * (size_t)atomicAdd(wf.list, 1u);
        e[0] = (unsigned)split;
        e[1] = (unsigned)gg;
        e[2] = (unsigned)kk;
      }
  }
  if (do_bias) {
    float *red = reinterpret_cast<float *>(lds);  // [256][9]
#pragma unroll
    for (int j = 0; j < 4; j++) red[(r + 64 * j) * 9 + tp] = bsum[j];
    __syncthreads();
    if (tid < BG && g0 + tid < g.G) {
      float sum = 0.0f;
      for (int i = 0; i < 8; i++) sum += red[tid * 9 + i];
      wsp[(int64_t)g.G * g.Kdim + g0 + tid] = sum;
    }
  }
}

// Scale-group statistics of the f16x3 weight gradient: op 0 = dY's filter
// groups (gw = P contiguous columns per group, G groups), op 1 = X's channel
// groups (gw = HW, C groups), every frame.  Block (group, row chunk);
// pass 0: max |x| and min nonzero |x| (bit patterns, atomicMax / atomicMin:
// order-independent), pass 1: for a spread group (f16-split.h) the count of
// its nonzero elements under small_bound (integer atomics).  out: [max n]
// [min n (0xffffffff: none)][cnt n]; wgrad_group_init_kernel sets them (and
// the element list's counter) first.
struct GStatOp {
  const float *A;
  int rows, ld, gw, n, rchunks;
  uint32_t *out;
};
__global__ __launch_bounds__(256) void wgrad_group_init_kernel(GStatOp a, GStatOp b,
                                                               unsigned *counter) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) *counter = 0u;
  for (const GStatOp *o : {&a, &b})
    if (i < o->n) {
      o->out[i] = 0u;
      o->out[o->n + i] = 0xffffffffu;
      o->out[2 * o->n + i] = 0u;
    }
}
__global__ __launch_bounds__(256) void wgrad_group_stats_kernel(GStatOp a, GStatOp b, int pass) {
  __shared__ uint32_t red[2][4];
  const int na = a.n * a.rchunks;
  const bool isa = (int)blockIdx.x < na;
  const GStatOp &o = isa ? a : b;
  const int blk = isa ? blockIdx.x : blockIdx.x - na;
  const int grp = blk % o.n, rc = blk / o.n;
  const int rb = (o.rows + o.rchunks - 1) / o.rchunks;
  const int r0 = rc * rb, r1 = min(o.rows, r0 + rb);
  if (r0 >= r1) return;
  const int cnt_e = (r1 - r0) * o.gw;
  const float *base = o.A + (int64_t)r0 * o.ld + (int64_t)grp * o.gw;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (pass == 0) {
    uint32_t m = 0, n = 0xffffffffu;
    for (int e = threadIdx.x; e < cnt_e; e += 256) {
      const int rr = e / o.gw, cc = e - rr * o.gw;
      const uint32_t x = __float_as_uint(base[(int64_t)rr * o.ld + cc]) & 0x7fffffffu;
      m = max(m, x);
      n = min(n, x - 1u);  // 0 - 1 wraps: a zero never wins
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      m = max(m, (uint32_t)__shfl_xor((int)m, d));
      n = min(n, (uint32_t)__shfl_xor((int)n, d));
    }
    if (lane == 0) { red[0][wave] = m; red[1][wave] = n; }
    __syncthreads();
    if (threadIdx.x == 0) {
      m = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
      n = min(min(red[1][0], red[1][1]), min(red[1][2], red[1][3]));
      atomicMax(o.out + grp, m);
      if (n != 0xffffffffu) atomicMin(o.out + o.n + grp, n + 1u);
    }
    return;
  }
  const uint32_t mx = o.out[grp], mn = o.out[o.n + grp];
  if (!f16x3::spread(mx, mn == 0xffffffffu ? 0u : mn)) return;  // (uniform)
  const float bound = f16x3::small_bound(mx);
  uint32_t c = 0;
  for (int e = threadIdx.x; e < cnt_e; e += 256) {
    const int rr = e / o.gw, cc = e - rr * o.gw;
    const float x = fabsf(base[(int64_t)rr * o.ld + cc]);
    c += (x < bound && x != 0.0f) ? 1u : 0u;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d);
  if (lane == 0 && c) atomicAdd(o.out + 2 * o.n + grp, c);
}

// A listed partial of the f16x3 weight gradient (entry: split, g, k), one
// wave per entry: the split's sum over t = n*P + p in fp32 (lane sums of t =
// lane + 64 i, then a butterfly), stored over the partial.
__global__ __launch_bounds__(256) void conv_wgrad_efix_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dY, int dys,
    float *__restrict__ ws, int fps, const unsigned *__restrict__ list,
    const unsigned *__restrict__ elist) {
  const unsigned cnt = list[0];
  const int lane = threadIdx.x & 63;
  const unsigned w0 = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int64_t E = (int64_t)g.G * g.Kdim + g.G;
  for (unsigned en = w0; en < cnt; en += nw) {
    const unsigned *e = elist + 3 * (size_t)en;
    const int split = (int)e[0], gg = (int)e[1], kk = (int)e[2];
    const int nbeg = split * fps, nf = min(g.R, nbeg + fps) - nbeg;
    uint32_t c, rr, kx, ky;
    g.div_khkw.divmod((uint32_t)kk, c, rr);
    g.div_kh.divmod(rr, kx, ky);
    const int T = nf * g.P;
    float s = 0.0f;
    for (int t = lane; t < T; t += 64) {
      uint32_t n, p, px, py;
      g.div_P.divmod((uint32_t)t, n, p);
      g.div_oh.divmod(p, px, py);
      const int xx = (int)px + (int)kx - g.pad_w, yy = (int)py + (int)ky - g.pad_h;
      const int64_t fr = nbeg + (int64_t)n;
      if ((unsigned)xx < (unsigned)g.W && (unsigned)yy < (unsigned)g.H)
        s = fmaf(dY[fr * dys + (int64_t)gg * g.P + p],
                 X[fr * xs + (int64_t)c * g.HW + xx * g.H + yy], s);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if (lane == 0) ws[(int64_t)split * E + (int64_t)gg * g.Kdim + kk] = s;
  }
}

// KCNN_CONV_X6_STAGGER=1: the wave-pair stagger (STG).  It gained 4 % on
// c5 while the split subtractions were packed into v_pk_add_f32; built
// without SLP vectorization (Makefile) the kernels measure the same or
// 0.6 % slower with it, so it is off by default.
int stagger() {
  static const int v = KCNN_KNOB("KCNN_CONV_X6_STAGGER", 0);
  return v;
}

constexpr int kLdsMax = 160 * 1024;
constexpr int img_bytes(bool f16) { return 2 * (f16 ? 2 : 3) * 384 * ROWB; }  // double-buffered planes

// LDS of the tap table for Kdim (0: it does not fit beside the images)
int tab_bytes(const ConvGeom &g, bool padded) {
  static const int use = KCNN_KNOB("KCNN_IGX6_TAB", 1);
  const int KT = (g.Kdim + BK - 1) / BK * BK;
  const int b = KT * 4 + (padded ? KT : 0);
  return use && img_bytes(false) + b <= kLdsMax ? b : 0;
}

template <int BG, bool PADDED, bool STG, bool TAB, int POOL, bool F16>
void launch_t(const ConvGeom &g, unsigned blocks, const float *X, int xs, const float *K,
              int ks, const float *bias, float *out, int os, int relu, hipStream_t st,
              PoolOut po, F16Aux fx) {
  const int lds = img_bytes(F16) + (TAB ? tab_bytes(g, PADDED) : 0) + (F16 ? kAuxBytes : 0);
  static bool attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&conv_igemm_x6_kernel<BG, PADDED, STG, TAB, POOL, F16>),
      hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL((conv_igemm_x6_kernel<BG, PADDED, STG, TAB, POOL, F16>), dim3(blocks),
                     dim3(NT), lds, st, g, X, xs, K, ks, bias, out, os, relu, po, fx);
}
// f16x3 implicit-GEMM calls since the last reset (kcnn_conv_fix_counts)
std::atomic<unsigned long long> g_igemm_f16_calls{0};
// the bf16x6 form, or the f16x3 form and the fp32 fixup of its listed tiles
template <int BG, bool PADDED, bool TAB, int POOL>
void launch_pair(const ConvGeom &g, unsigned blocks, const float *X, int xs, const float *K,
                 int ks, const float *bias, float *out, int os, int relu, hipStream_t st,
                 PoolOut po, F16Aux fx) {
  if (!fx.list) {
    launch_t<BG, PADDED, false, TAB, POOL, false>(g, blocks, X, xs, K, ks, bias, out, os, relu,
                                                  st, po, fx);
    return;
  }
  launch_t<BG, PADDED, false, TAB, POOL, true>(g, blocks, X, xs, K, ks, bias, out, os, relu,
                                               st, po, fx);
  g_igemm_f16_calls.fetch_add(1, std::memory_order_relaxed);
  hipLaunchKernelGGL((conv_igemm_fixup_kernel<BG, POOL>), dim3(std::min(blocks, 256u)),
                     dim3(256), 0, st, g, X, xs, K, ks, bias, out, os, relu, po,
                     (const unsigned *)fx.list);
  hipLaunchKernelGGL((conv_igemm_efix_kernel<POOL>), dim3(64), dim3(256), 0, st, g, X, xs, K,
                     ks, bias, out, os, relu, po, (const unsigned *)fx.list,
                     (const unsigned *)fx.elist);
}
// pooled epilogue (POOL > 0): no stagger (the host declines it)
template <int BG, bool PADDED, int POOL>
void launch_pool(const ConvGeom &g, unsigned blocks, const float *X, int xs, const float *K,
                 int ks, const float *bias, float *out, int os, PoolOut po, F16Aux fx,
                 hipStream_t st) {
  if (tab_bytes(g, PADDED))
    launch_pair<BG, PADDED, true, POOL>(g, blocks, X, xs, K, ks, bias, out, os, 0, st, po, fx);
  else
    launch_pair<BG, PADDED, false, POOL>(g, blocks, X, xs, K, ks, bias, out, os, 0, st, po, fx);
}
template <int BG, bool PADDED>
void launch(const ConvGeom &g, unsigned blocks, const float *X, int xs, const float *K, int ks,
            const float *bias, float *out, int os, int relu, F16Aux fx, hipStream_t st) {
  const bool tb = tab_bytes(g, PADDED) != 0;
  if (stagger() && !fx.list) {
    if (tb) launch_t<BG, PADDED, true, true, 0, false>(g, blocks, X, xs, K, ks, bias, out, os, relu, st, PoolOut{}, fx);
    else launch_t<BG, PADDED, true, false, 0, false>(g, blocks, X, xs, K, ks, bias, out, os, relu, st, PoolOut{}, fx);
    return;
  }
  if (tb) launch_pair<BG, PADDED, true, 0>(g, blocks, X, xs, K, ks, bias, out, os, relu, st, PoolOut{}, fx);
  else launch_pair<BG, PADDED, false, 0>(g, blocks, X, xs, K, ks, bias, out, os, relu, st, PoolOut{}, fx);
}

// The f16x3 form's statistics and tile flags (igemm_x6 family 2) in per-call
// scratch from the device allocator (kaldi-lite/cu-device.h CuScratch: the
// block is reused only by work ordered after this call's kernels): W's column
// and X's row statistics (f16-split.h), one flag per tile.  Returns 0, or
// the error of a statistics launch.
struct F16Setup {
  kaldi::CuScratch ws;
  F16Aux fx{};
  int rc = 0;
  F16Setup(bool on, const ConvGeom &g, const float *X, int xs, const float *K, int ks,
           unsigned blocks, hipStream_t st)
      : ws(on ? words(g, blocks, ks) * 4 : 0) {
    if (!on) return;
    uint32_t *w = static_cast<uint32_t *>(ws.p);
    uint32_t *wst = w, *xst = wst + 3 * (size_t)g.G, *list = xst + 3 * (size_t)g.R,
             *elist = list + 2 + blocks, *part = elist + elist_words(blocks);
    rc = kl_absmax_rows_cols(X, g.R, g.HW * g.C, xs, xst, K, g.Kdim, g.G, ks, wst, part, list,
                             reinterpret_cast<kcnn_stream_t>(st));
    if (rc) return;
    uint32_t *wsplit = part + kl_absmax_cols_words(g.Kdim, g.G);
    const int64_t nw = (int64_t)g.Kdim * g.G;
    hipLaunchKernelGGL(conv_w_presplit_kernel,
                       dim3((unsigned)std::min<int64_t>((nw + 255) / 256, 1024)), dim3(256), 0,
                       st, K, ks, g.Kdim, g.G, (const uint32_t *)wst, wsplit);
    rc = (int)hipGetLastError();
    fx.wst = wst;
    fx.xst = xst;
    fx.list = list;
    fx.elist = elist;
    fx.wsplit = wsplit;
  }
  static size_t elist_words(unsigned blocks) { return (size_t)blocks * 8 * REJ_MAX * EW; }
  static size_t words(const ConvGeom &g, unsigned blocks, int ks) {
    return 3 * (size_t)g.G + 3 * (size_t)g.R + 2 + blocks + elist_words(blocks) +
           kl_absmax_cols_words(g.Kdim, g.G) + (size_t)g.Kdim * ks;
  }
};
// f16x3 for the large convolutions (2 M G Kdim >= 2^34 flop: c5's C2 / C3
// forward, C3 data gradient and C2's 1x1 data gradient); the others keep
// bf16x6.  nnet.config's layers (<= 8.6 Gflop): the statistics pass over X
// and the few tiles do not repay it (its convolutions 2.06 -> 2.20 ms per
// step with f16x3)
// (family value 3: f16x3 for every shape, the tests' setting)
bool use_f16(const ConvGeom &g) {
  static const int lg = KCNN_KNOB("KCNN_IGF16_LOG2FLOP", 34);
  const int f = family(kFamIgemmX6);
  return g.R > 0 && (f == 3 || (f == 2 && 2.0 * (double)g.M * g.G * g.Kdim >=
                                              (double)(1ull << lg)));
}
// experiment build: KCNN_IGF16_DEBUG=1 prints each call's recomputed tiles
void report_flags(const F16Aux &fx, unsigned nb, const ConvGeom &g, hipStream_t st) {
  static const int dbg = KCNN_KNOB("KCNN_IGF16_DEBUG", 0);
  if (!dbg || !fx.list) return;
  unsigned n[2] = {0, 0};
  if (hipMemcpyAsync(n, fx.list, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return;
  fprintf(stderr, "igemm f16x3: G %d Kdim %d M %lld: %u of %u tiles, %u elements recomputed\n",
          g.G, g.Kdim, (long long)g.M, n[0], nb, n[1]);
}

}  // namespace

// The f16x3 implicit GEMM's cumulative counts (kcnn.h): out[0] its calls,
// out[1] the tiles and out[2] the elements its fix-up kernels recomputed in
// fp32; reset != 0 zeroes them afterwards.  Synchronises the device.
extern "C" int kcnn_conv_fix_counts(unsigned long long *out, int reset) {
  unsigned long long d[2] = {0, 0};
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(d, HIP_SYMBOL(g_igemm_fix_counts), sizeof d) != hipSuccess)
    return 1;
  if (out) {
    out[0] = g_igemm_f16_calls.load();
    out[1] = d[0];
    out[2] = d[1];
  }
  if (reset) {
    const unsigned long long z[2] = {0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_igemm_fix_counts), z, sizeof z) != hipSuccess) return 1;
    g_igemm_f16_calls.store(0);
  }
  return 0;
}

// Conv2D(concat) + bias (+ ReLU) on the f16 (family igemm_x6 = 2, with the
// bf16x6 form for flagged tiles) or bf16 (1) MFMAs; -1 (nothing launched)
// for shapes outside its addressing limits.  KCNN_IGEMM_X6=0 disables it
// (the fp32-MFMA conv_igemm2_kernel then runs).
// Blocks of kcnn_conv_igemm_x6 for g, 0 when the shape is outside its limits.
static unsigned igemm_x6_blocks(const ConvGeom &g, int xs, int ks) {
  if (!family(kFamIgemmX6) || g.M <= 0 || g.G <= 0 || g.Kdim <= 0) return 0;
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
  if (padded && g.kh * g.kw > 31) return 0;
  if ((int64_t)g.R * xs * 4 >= (int64_t)kOob || (int64_t)g.C * g.HW * 4 >= (int64_t)kOob)
    return 0;
  if ((int64_t)(g.Kdim + BK) * ks * 4 >= (int64_t)kOob || g.M >= ((int64_t)1 << 31) ||
      (int64_t)g.G * g.P >= ((int64_t)1 << 31))
    return 0;
  const int BG = g.G <= 128 ? 128 : 256;
  const int64_t tiles = (int64_t)((g.G + BG - 1) / BG) * ((g.M + (384 - BG) - 1) / (384 - BG));
  if (tiles >= ((int64_t)1 << 31)) return 0;
  return (unsigned)tiles;
}

int kcnn_conv_igemm_x6(const ConvGeom &g, const float *X, int xs, const float *K, int ks,
                       const float *bias, float *out, int os, int relu, hipStream_t st) {
  const unsigned nb = igemm_x6_blocks(g, xs, ks);
  if (nb == 0) return -1;
  const bool f16 = use_f16(g);
  F16Setup fs(f16, g, X, xs, K, ks, nb, st);
  if (fs.rc) return fs.rc;
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
  if (g.G <= 128) {
    if (padded) launch<128, true>(g, nb, X, xs, K, ks, bias, out, os, relu, fs.fx, st);
    else launch<128, false>(g, nb, X, xs, K, ks, bias, out, os, relu, fs.fx, st);
  } else {
    if (padded) launch<256, true>(g, nb, X, xs, K, ks, bias, out, os, relu, fs.fx, st);
    else launch<256, false>(g, nb, X, xs, K, ks, bias, out, os, relu, fs.fx, st);
  }
  report_flags(fs.fx, nb, g, st);
  if (!f16 && KCNN_KNOB("KCNN_IGF16_DEBUG", 0))
    fprintf(stderr, "igemm bf16x6: G %d Kdim %d M %lld relu %d\n", g.G, g.Kdim, (long long)g.M, relu);
  return (int)hipGetLastError();
}

// The same convolution (bit for bit: the same kernel, tiles and K order) with
// the following ph x pw x pc Maxpool in its epilogue, for windows of two
// consecutive map positions: ph x pw = 2 x 1 (oh even) or 1 x 2 (oh = 1, ow
// even), pc in {1, 2, 4} dividing G.  out (Y) nullable; mask 16-bit, ms in
// elements.  -1 (nothing launched) otherwise.
int kcnn_conv_igemm_x6_pool(const ConvGeom &g, const float *X, int xs, const float *K,
                            int ks, const float *bias, float *out, int os, float *pool,
                            int ps, unsigned short *mask, int ms, int ph, int pw, int pc,
                            hipStream_t st) {
  const bool win = (ph == 2 && pw == 1 && g.oh % 2 == 0) ||
                   (ph == 1 && pw == 2 && g.oh == 1 && g.ow % 2 == 0);
  if (!win || !(pc == 1 || pc == 2 || pc == 4) || g.G % pc != 0 || stagger()) return -1;
  const unsigned nb = igemm_x6_blocks(g, xs, ks);
  if (nb == 0) return -1;
  const bool f16 = use_f16(g);
  F16Setup fs(f16, g, X, xs, K, ks, nb, st);
  if (fs.rc) return fs.rc;
  const PoolOut po{pool, ps, mask, ms};
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
#define KCNN_IGP(BG_, PAD_)                                                                 \
  do {                                                                                      \
    if (pc == 4) launch_pool<BG_, PAD_, 1>(g, nb, X, xs, K, ks, bias, out, os, po, fs.fx, st);     \
    else if (pc == 1) launch_pool<BG_, PAD_, 2>(g, nb, X, xs, K, ks, bias, out, os, po, fs.fx, st); \
    else launch_pool<BG_, PAD_, 3>(g, nb, X, xs, K, ks, bias, out, os, po, fs.fx, st);             \
  } while (0)
  if (g.G <= 128) {
    if (padded) KCNN_IGP(128, true);
    else KCNN_IGP(128, false);
  } else {
    if (padded) KCNN_IGP(256, true);
    else KCNN_IGP(256, false);
  }
#undef KCNN_IGP
  report_flags(fs.fx, nb, g, st);
  return (int)hipGetLastError();
}

// Weight gradient plan: S frame-range splits, each a whole number of frames,
// sized so the S x tiles blocks fill whole rounds of 256 (one per CU) and an
// accumulation chain stays within ~16k terms.
// KCNN_WGRAD_X6: 0 off, 1 the 128-wide k tiles, 2 the wide (256) k tiles
static int wgrad_x6_mode() { return family(kFamWgradX6); }
static int wgrad_kwidth() { return wgrad_x6_mode() >= 2 ? 256 : 128; }
// the f16x3 form of the wide kernel: family 3 (not the default: measured
// slower on c5, DESIGN 3 Long kernels)
static bool wgrad_f16(const ConvGeom &) { return wgrad_x6_mode() == 3; }

bool kcnn_conv_wgrad_x6_plan(const ConvGeom &g, int xs, int dys, int &S, int &fps,
                             size_t &ws_bytes) {
  const int use = wgrad_x6_mode();
  if (!use || g.R <= 0 || g.G < 32 || g.Kdim < 32) return false;
  if ((int64_t)g.C * g.HW * 4 >= (int64_t)kOob || (int64_t)g.G * g.P * 4 >= (int64_t)kOob)
    return false;
  const int ktiles = (g.Kdim + wgrad_kwidth() - 1) / wgrad_kwidth();
  const int ntiles = ktiles * ((g.G + 255) / 256);
  const int64_t chain = (int64_t)g.R * g.P;
  int s0 = (int)((chain + 16383) / 16384);
  if (s0 < 1) s0 = 1;
  if ((int64_t)s0 * ntiles < 256) s0 = (256 + ntiles - 1) / ntiles;
  if (s0 > g.R) s0 = g.R;
  int best_s = -1, best_fps = 0;
  double best_cost = 0;
  for (int s = s0; s <= 2 * s0 && s <= g.R; s++) {
    const int f = (g.R + s - 1) / s;
    const int sa = (g.R + f - 1) / f;
    const int64_t rounds = ((int64_t)sa * ntiles + 255) / 256;
    const double cost = (double)rounds * f;
    if (best_s < 0 || cost < best_cost) { best_s = sa; best_fps = f; best_cost = cost; }
  }
  if ((int64_t)best_fps * dys * 4 >= (int64_t)kOob || (int64_t)best_fps * xs * 4 >= (int64_t)kOob)
    return false;
  S = best_s;
  fps = best_fps;
  const size_t E = (size_t)g.G * g.Kdim + g.G;
  ws_bytes = (size_t)S * E * sizeof(float) + kcnn_reduce_splits_ws(S, (int)E);
  return true;
}

// Partials [S][G*Kdim + G] into ws (kcnn_conv_wgrad_x6_plan's S and fps).
int kcnn_conv_wgrad_x6(const ConvGeom &g, const float *X, int xs, const float *dY, int dys,
                       float *ws, int S, int fps, hipStream_t st) {
  const bool padded = g.pad_h > 0 || g.pad_w > 0;
  const int ktiles = (g.Kdim + wgrad_kwidth() - 1) / wgrad_kwidth();
  const int nblocks = S * ktiles * ((g.G + 255) / 256);
  const dim3 grid((unsigned)(8 * ((nblocks + 7) / 8)));
  if (wgrad_kwidth() == 256) {
    constexpr int wl = 2 * 3 * 512 * WROW;
    constexpr int wl16 = 2 * 2 * 512 * WROW + 512 * 8;  // + the groups' scales / weights
    const bool f16 = wgrad_f16(g);
    WF16 wf{};
    kaldi::CuScratch sc(f16 ? (3 * (size_t)(g.G + g.C) + 1 + (size_t)nblocks +
                               3 * (size_t)nblocks * 8 * REJ_MAX) * 4
                            : 0);
    if (f16) {
      uint32_t *w = static_cast<uint32_t *>(sc.p);
      uint32_t *gst = w, *cst = gst + 3 * (size_t)g.G, *list = cst + 3 * (size_t)g.C;
      wf.gst = gst;
      wf.cst = cst;
      wf.list = list;
      wf.flags = list + 1;
      wf.elist = wf.flags + nblocks;
      const int rch = std::max(1, std::min(64, g.R / 64));
      const GStatOp ga{dY, g.R, dys, g.P, g.G, rch, gst};
      const GStatOp gc{X, g.R, xs, g.HW, g.C, rch, cst};
      hipLaunchKernelGGL(wgrad_group_init_kernel, dim3((std::max(g.G, g.C) + 255) / 256),
                         dim3(256), 0, st, ga, gc, list);
      for (int pass = 0; pass < 2; pass++)
        hipLaunchKernelGGL(wgrad_group_stats_kernel, dim3((g.G + g.C) * rch), dim3(256), 0, st,
                           ga, gc, pass);
    }
#define KCNN_WX6W(P_, F_, L_)                                                               \
  do {                                                                                      \
    static bool attr = hipFuncSetAttribute(                                                 \
        reinterpret_cast<const void *>(&conv_wgrad_x6w_kernel<P_, F_>),                     \
        hipFuncAttributeMaxDynamicSharedMemorySize, L_) == hipSuccess;                       \
    (void)attr;                                                                             \
    hipLaunchKernelGGL((conv_wgrad_x6w_kernel<P_, F_>), grid, dim3(NT), L_, st, g, X, xs,  \
                       dY, dys, ws, fps, ktiles, nblocks, wf);                              \
  } while (0)
    if (f16) {
      if (padded) KCNN_WX6W(true, true, wl16);
      else KCNN_WX6W(false, true, wl16);
      hipLaunchKernelGGL(conv_wgrad_efix_kernel, dim3(64), dim3(256), 0, st, g, X, xs, dY, dys,
                         ws, fps, (const unsigned *)wf.list, (const unsigned *)wf.elist);
      wf.redo = wf.flags;
    }
    if (padded) KCNN_WX6W(true, false, wl);
    else KCNN_WX6W(false, false, wl);
#undef KCNN_WX6W
    return (int)hipGetLastError();
  }
  constexpr int lds = 2 * 3 * 384 * ROWB;
#define KCNN_WX6(P_, S_)                                                                  \
  do {                                                                                    \
    static bool attr = hipFuncSetAttribute(                                               \
        reinterpret_cast<const void *>(&conv_wgrad_x6_kernel<P_, S_>),                    \
        hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;                    \
    (void)attr;                                                                           \
    hipLaunchKernelGGL((conv_wgrad_x6_kernel<P_, S_>), grid, dim3(NT), lds, st, g, X, xs, \
                       dY, dys, ws, fps, ktiles, nblocks);                                \
  } while (0)
  if (padded) {
    if (stagger()) KCNN_WX6(true, true); else KCNN_WX6(true, false);
  } else {
    if (stagger()) KCNN_WX6(false, true); else KCNN_WX6(false, false);
  }
#undef KCNN_WX6
  return (int)hipGetLastError();
}
