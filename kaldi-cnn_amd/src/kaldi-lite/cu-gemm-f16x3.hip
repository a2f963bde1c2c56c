// kaldi-lite/cu-gemm-f16x3.hip -- fp32 GEMM on the f16 matrix cores from a
// two-part f16 split of each operand under a power-of-two scale per output
// row and column (the "f16x3" scheme, AddMatMat's default engine).
//
// Upstream Kaldi's CuMatrixBase::AddMatMat is cuBLAS sgemm; the reference
// calls it for the FullyConnectedComponent forward, data gradient and update
// (nnet-component.cc:1225-1227, :1247; nnet-component-nnet0.cc:1137-1142).
// The bf16x6 kernel (cu-gemm-x6.hip) reaches fp32 accuracy with six bf16
// products per fp32 product.  f16 carries 11 significant bits to bf16's 8,
// so two parts suffice once the operands are scaled into f16's range:
//
//   x' = x * 2^s   (s per row of op(A) / column of op(B): the row's largest
//                   |x'| lies in [2^14, 2^15))
//   hi = f16(x'),  lo = f16(x' - hi)        (x' - hi is exact in fp32)
//
// x' = hi + lo to within 2^-22 |x'| while |x'| >= 2^-3; below that lo is an
// f16 subnormal and the error is under 2^-25 absolute, 2^-39 of the row's
// largest element.  With every f16 product exact in fp32,
//
//   a'b' = hi.hi + (hi.lo + lo.hi) + lo.lo
//
// and the kernel keeps the first three (one v_mfma_f32_32x32x16_f16 each,
// smallest first, accumulated in fp32), then C = acc * 2^-(s_a + s_b) by an
// exact ldexp.  The bound is therefore per group, not per product: for two
// groups that are not "spread" (no element more than 20 binades under the
// group's max, f16-split.h) every element is held to 2^-19, and a product is
// within (2 * 2^-19 + 2^-22) S of exact; a product touching a spread group
// is checked at its store against the count of the group's small elements
// and recomputed in fp32 when the check cannot clear it (tile_epilogue,
// gemm_f16x3_reduce_kernel).  So every finite C element meets the 1e-5 * S
// parity bar whatever the operands' range; the scale puts a
// whole row near FLT_MAX or of fp32 subnormals into f16's range like any
// other (the bf16x6 split loses bits there).  The f16 MFMA runs at the bf16
// rate: half the matrix-core work of bf16x6 for the same split VALU.
//
// The scales come from per-row / per-column max |x| (kl_absmax_rows /
// kl_absmax_cols: the bit patterns of |x|, whose unsigned order is the
// magnitude order).  A row of
// op(A) or a column of op(B) holding Inf or NaN has no scale; every C
// element in it is Inf or NaN in IEEE arithmetic.  The main loop leaves
// those elements alone and the tile's split-0 workgroup computes them as
// plain fp32 dot products (tile_epilogue), which gives sgemm's IEEE pattern
// (+Inf, -Inf or NaN).
//
// Structure: gemm_x6d_kernel's (cu-gemm-x6.hip): 512 threads, a 256 x 128
// tile of C per workgroup (8 waves of 2 x 2 accumulators of 32 x 32), K steps
// of 32, operands loaded as fp32 by branch-free buffer loads two steps ahead,
// split in registers into two f16 planes of swizzled [row][k] LDS images
// (double-buffered, 2 x 48 KB), one barrier per step.  Thin outputs split K
// over workgroups into partial slabs, which gemm_f16x3_reduce_kernel sums in
// a fixed order.
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "cnslmat/f16-split.h"
#include "cnslmat/hip-util.h"
#include "cnslmat/momentum-step.h"
#include "cnslmat/pool-stats-dev.h"
#include "cnslmat/pool-stats.h"
#include "kaldi-lite/cu-kernels-lite.h"

namespace {

using kcnn::COLMAX_ROWS;
using kcnn::PoolCountSmem;
using kcnn::pool_colmax_block;
using kcnn::pool_count_block;
using kcnn::f16x3::f16x8;
using kcnn::f16x3::f32x16;
using kcnn::f16x3::NONFINITE;
using kcnn::f16x3::SKIP;
using kcnn::f16x3::scale_exp;
using kcnn::f16x3::split2h;
using kcnn::f16x3::mfma;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 128, BK = 32, NT = 512;
constexpr int ROWB = BK * 2;                  // bytes per LDS row of one plane
constexpr int A_PLANE = BM * ROWB;            // 16 KB
constexpr int B_PLANE = BN * ROWB;            // 8 KB
constexpr int BUF = 2 * (A_PLANE + B_PLANE);  // 48 KB
constexpr int LDS_BYTES = 2 * BUF + (BM + BN) * 8;  // + sexp, sw

struct GemmF16Args {
  const float *A, *B;
  float *C;                      // the output
  float *part;                   // ksplit > 1: the partial slabs [ksplit][M][N]
  uint32_t *rflag;               // ksplit > 1: per 64 quads of C, 1 when the reduce left
                                 // its rejections to gemm_f16x3_fixup_kernel; after
                                 // them one word, gen when any group was flagged
  uint32_t gen;                  // this call's number (host counter, never 0)
  const uint32_t *amax, *bmax;   // max |x| bits per row of op(A), per column of op(B)
  const uint32_t *amin, *bmin;   // min nonzero |x| bits (0: none), the same groups
  const uint32_t *acnt, *bcnt;   // spread groups: their elements below 2^-3 after the scale
  const float *bias;             // nullable: C += bias[col] on every row (after alpha, beta)
  int M, N, K, lda, ldb, ldc;
  int bvec;                      // bmax, bcnt 16-B aligned and N % 4 == 0 (the reduce's loads)
  MomentumEpi mom;               // mom.W: C is a weight gradient applied in the store (emit)
  int dbg;                       // KCNN_EXPERIMENTS builds: A/B switches
  int kps, ksplit, tiles_m, tiles_n;
  int nwhole;                    // ksplit > 1: the first nwhole tiles (a multiple of 256) whole
  int fix_local;                 // ksplit > 1: no fix-up launch; the reduce recomputes every rejection
  uint32_t *fix_report;          // nullable (host memory): set to 1 when a group would be deferred
  float alpha, beta;
};

// Tile t of the order -> (tile row, tile column).  The tiles go in groups of
// GM tile rows, column-major inside a group, so the 32 workgroups an XCD runs
// at once (consecutive logical ids, block_tile) cover about 32 / GM tile
// columns of GM tile rows, sharing GM row panels of op(A) and a few column
// panels of op(B) in that XCD's L2, instead of one row panel and 32 column
// panels (c2's data gradient: an XCD wave then reads 8 MB of operand panels
// instead of 17)
#ifndef KCNN_GEMM_GM
#define KCNN_GEMM_GM 4
#endif
__device__ __forceinline__ void tile_rc(const GemmF16Args &p, int t, int &tm, int &tn) {
  const int gsz = KCNN_GEMM_GM * p.tiles_n;
  const int g = t / gsz, r = t - g * gsz;
  const int m0 = g * KCNN_GEMM_GM;
  const int gm = min(p.tiles_m - m0, KCNN_GEMM_GM);
  tm = m0 + r % gm;
  tn = r / gm;
}
// ... and back: the order's index of tile (tm, tn)
__device__ __forceinline__ int tile_index(const GemmF16Args &p, int tm, int tn) {
  const int g = tm / KCNN_GEMM_GM, m0 = g * KCNN_GEMM_GM;
  const int gm = min(p.tiles_m - m0, KCNN_GEMM_GM);
  return g * KCNN_GEMM_GM * p.tiles_n + tn * gm + (tm - m0);
}
// This workgroup's (split, tile row, tile column); true for a whole tile.
// Blocks [0, nwhole) take tiles [0, nwhole) over all of K, the others the
// ksplit splits of the remaining tiles (consecutive logical ids: the splits
// of one tile).  Each part in the XCD-aware order (gemm_x6_kernel): block b
// runs on XCD b & 7, and consecutive logical ids go to one XCD (nwhole is a
// multiple of 256, so both parts keep that phase and every XCD gets an
// eighth of each).  nwhole 0: the plain split grid.
__device__ __forceinline__ bool block_tile(const GemmF16Args &p, int &split, int &tm, int &tn) {
  const bool whole = (int)blockIdx.x < p.nwhole;
  const int b = whole ? (int)blockIdx.x : (int)blockIdx.x - p.nwhole;
  const int nb = whole ? p.nwhole : (int)gridDim.x - p.nwhole;
  const int ks = whole ? 1 : p.ksplit;
  const int xcd = b & 7, q = nb >> 3, rr = nb & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  split = lid % ks;
  tile_rc(p, (whole ? 0 : p.nwhole) + lid / ks, tm, tn);
  return whole;
}
// C element (r, c) is a split tile's (its value from the partial slabs)
__device__ __forceinline__ bool in_split_tile(const GemmF16Args &p, int r, int c) {
  return p.nwhole == 0 || tile_index(p, r / BM, c / BN) >= p.nwhole;
}

__device__ __forceinline__ int swz(int r, int c) {
  return r * ROWB + ((c ^ ((r >> 2) & 3)) << 4);
}
// offset of (k, col) in a [k][R] image of 16-bit values, 16-B chunks XOR-
// swizzled by (k & 3) << 2 so the four k-rows of one transposed read hit
// four disjoint 16-bank groups (cu-gemm-x6.hip's fast kernel)
template <int R>
__device__ __forceinline__ int tswz(int k, int col) {
  return k * (R * 2) + ((((col >> 3) ^ ((k & 3) << 2))) << 4) + ((col & 7) << 1);
}

// Operand tile loaders (R rows of C's side x BK per K step), loads two steps
// ahead by branch-free buffer loads (gemm_x6d_kernel's TileLoaderD), split in
// registers into the hi / lo planes.  Three source layouts:
//   LK  K-contiguous (element (row, k) at src[row * ld + k]): unit = (row,
//       8-k chunk), two 16-B loads; [row][k] image (swz), fragments by
//       ds_read_b128;
//   LR  row-contiguous ([k][row]) with one dword per lane: unit = (row, KPT
//       consecutive k), lanes along the row; [row][k] image;
//   LT  row-contiguous with 16-B loads along the rows (ld % 4 == 0, 16-B
//       base, the row count a multiple of 4): unit = (4 rows, KQ k); [k][row]
//       image (tswz), fragments by ds_read_b64_tr_b16.
// Every row of a unit has its own scale exponent (e[]).
enum { LK = 0, LR = 1, LT = 2 };

template <int R, int MODE>
struct Loader {
  static constexpr int KPT = MODE == LK ? 8 : MODE == LR ? R * BK / NT : R * BK / (NT * 4);
  static constexpr int UNITS = MODE == LK ? R * 4 : MODE == LR ? R * BK / KPT : NT;
  static constexpr int UPT = (UNITS + NT - 1) / NT;
  static constexpr int NE = MODE == LT ? 4 : UPT;  // exponents per thread
  static_assert(UNITS % NT == 0, "tile shape");
  static_assert(MODE != LR || KPT % 8 == 0, "tile shape");
  static_assert(MODE != LT || (R / 4) * (BK / KPT) == NT, "tile shape");
  static constexpr int NV = MODE == LT ? 4 * KPT : KPT;  // values per unit
  float v[UPT][NV];
  int e[NE];

  // first row of exponent i
  __device__ static __forceinline__ int row_of(int i, int tid) {
    if constexpr (MODE == LT) return 4 * (tid % (R / 4)) + i;
    const int unit = tid + i * NT;
    return MODE == LK ? unit >> 2 : unit % R;
  }
  __device__ __forceinline__ void init_exp(const int *sexp, int tid) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int s = sexp[row_of(i, tid)];
      e[i] = s == SKIP ? 0 : s;
    }
  }

  // base: LK, the tile's first row (src + row0 * ld); LR / LT, the split's
  // first k and the tile's first column (src + kbeg * ld + row0).  Rows past
  // the matrix read past the buffer's range (0).
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int ld, int vrows, int kk,
                                       int tid) {
    constexpr unsigned OOB = 0x80000000u;
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      if constexpr (MODE == LK) {
        const int r = unit >> 2, k = kk + (unit & 3) * 8;
        const unsigned off = r < vrows ? (unsigned)(r * ld + k) * 4u : OOB;
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[u][j] = __uint_as_float(a[j]);
          v[u][4 + j] = __uint_as_float(b[j]);
        }
      } else if constexpr (MODE == LR) {
        const int r = unit % R, k = kk + (unit / R) * KPT;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
          const unsigned off = r < vrows ? (unsigned)((k + j) * ld + r) * 4u : OOB;
          v[u][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      } else {
        const int rq = unit % (R / 4), k = kk + (unit / (R / 4)) * KPT;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
          const unsigned off = 4 * rq < vrows ? (unsigned)((k + j) * ld + 4 * rq) * 4u : OOB;
          const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[u][4 * j + i] = __uint_as_float(a[i]);
        }
      }
    }
  }

  // split and write the two planes (plane stride PL bytes); kv < BK: the
  // tile is the last, partial one and its k >= kv are zeroed (they are the
  // next row's values or a pitch's padding)
  // (RAG: K is not a whole number of BK steps, so the last tile can be
  // partial; without it no masking code is emitted -- the compiler turns
  // the uniform kv test into per-element selects)
  template <int PL, bool RAG>
  __device__ __forceinline__ void store(char *lds, int tid, int kv, float m1) const {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      float x[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) x[j] = v[u][j];
      if constexpr (MODE == LT) {
        const int rq = unit % (R / 4), kq = unit / (R / 4);
        if (RAG && kv < BK) {
#pragma unroll
          for (int j = 0; j < KPT; ++j)
            if (kq * KPT + j >= kv)
#pragma unroll
              for (int i = 0; i < 4; ++i) x[4 * j + i] = 0.0f;
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
          uint32_t h0, l0, h1, l1;
          split2h(x[4 * j], x[4 * j + 1], e[0], e[1], h0, l0, m1);
          split2h(x[4 * j + 2], x[4 * j + 3], e[2], e[3], h1, l1, m1);
          const int o = tswz<R>(kq * KPT + j, 4 * rq);
          *reinterpret_cast<uint2 *>(lds + o) = make_uint2(h0, h1);
          *reinterpret_cast<uint2 *>(lds + PL + o) = make_uint2(l0, l1);
        }
      } else {
        int r, c0, kb;
        if constexpr (MODE == LK) {
          r = unit >> 2;
          c0 = unit & 3;
          kb = c0 * 8;
        } else {
          r = unit % R;
          c0 = (unit / R) * (KPT / 8);
          kb = (unit / R) * KPT;
        }
        if (RAG && kv < BK) {
#pragma unroll
          for (int j = 0; j < KPT; ++j)
            if (kb + j >= kv) x[j] = 0.0f;
        }
#pragma unroll
        for (int cc = 0; cc < KPT / 8; ++cc) {
          uint32_t h[4], l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            split2h(x[cc * 8 + 2 * i], x[cc * 8 + 2 * i + 1], e[u], e[u], h[i], l[i], m1);
          const int off = swz(r, c0 + cc);
          *reinterpret_cast<uint4 *>(lds + off) = make_uint4(h[0], h[1], h[2], h[3]);
          *reinterpret_cast<uint4 *>(lds + PL + off) = make_uint4(l[0], l[1], l[2], l[3]);
        }
      }
    }
  }

  // The split of store() in NPIECE pieces of one pair each, for the fast
  // kernel's interleaving with MFMAs: piece pc splits one pair into the
  // caller's temporaries; a unit's (LK, LR) or a k-row's (LT) plane writes go
  // with its last piece
  static constexpr int NPIECE = MODE == LT ? 2 * KPT : UPT * (KPT / 2);
  template <int PL, bool RAG>
  __device__ __forceinline__ void piece(char *lds, int tid, int pc, int kv, uint32_t (&ph)[4],
                                        uint32_t (&pl)[4], float m1) const {
    if constexpr (MODE == LT) {
      const int j = pc >> 1, hf = pc & 1;
      const int unit = tid;
      const int rq = unit % (R / 4), kq = unit / (R / 4);
      float x0 = v[0][4 * j + 2 * hf], x1 = v[0][4 * j + 2 * hf + 1];
      if (RAG && kv < BK) {
        asm volatile("");  // a branch: not per-element selects in every K step
        if (kq * KPT + j >= kv) x0 = x1 = 0.0f;
      }
#ifdef KCNN_GEMM_XNOSPLIT
      ph[hf] = __float_as_uint(x0);
      pl[hf] = __float_as_uint(x1);
#else
      split2h(x0, x1, e[2 * hf], e[2 * hf + 1], ph[hf], pl[hf], m1);
#endif
      if (hf == 1) {
        const int o = tswz<R>(kq * KPT + j, 4 * rq);
        *reinterpret_cast<uint2 *>(lds + o) = make_uint2(ph[0], ph[1]);
        *reinterpret_cast<uint2 *>(lds + PL + o) = make_uint2(pl[0], pl[1]);
      }
    } else {
      constexpr int PPU = KPT / 2;  // pieces per unit
      const int u = pc / PPU, q = pc % PPU;
      const int unit = tid + u * NT;
      int r, c0, kb;
      if constexpr (MODE == LK) {
        r = unit >> 2;
        c0 = unit & 3;
        kb = c0 * 8;
      } else {
        r = unit % R;
        c0 = (unit / R) * (KPT / 8);
        kb = (unit / R) * KPT;
      }
      float x0 = v[u][2 * q], x1 = v[u][2 * q + 1];
      if (RAG && kv < BK) {
        asm volatile("");  // a branch: not per-element selects in every K step
        if (kb + 2 * q >= kv) x0 = 0.0f;
        if (kb + 2 * q + 1 >= kv) x1 = 0.0f;
      }
#ifdef KCNN_GEMM_XNOSPLIT  // experiment build: timing without the split
      ph[q & 3] = __float_as_uint(x0);
      pl[q & 3] = __float_as_uint(x1);
#else
      split2h(x0, x1, e[u], e[u], ph[q & 3], pl[q & 3], m1);
#endif
      if ((q & 3) == 3) {
        const int off = swz(r, c0 + (q >> 2));
        *reinterpret_cast<uint4 *>(lds + off) = make_uint4(ph[0], ph[1], ph[2], ph[3]);
        *reinterpret_cast<uint4 *>(lds + PL + off) = make_uint4(pl[0], pl[1], pl[2], pl[3]);
      }
    }
  }
  // fragment reads per MFMA fragment (LT: two transposed 8-B reads)
  static constexpr int NRD = MODE == LT ? 2 : 1;

  // MFMA fragment: 32 rows from rb, k16 half s (lane l: row l & 31, k 8 (l >> 5) + 0..7)
  __device__ static __forceinline__ f16x8 frag(const char *plane, int rb, int s, int lane) {
    if constexpr (MODE != LT) {
      return *reinterpret_cast<const f16x8 *>(plane + swz(rb + (lane & 31), 2 * s + (lane >> 5)));
    } else {
      const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
      const int k = 16 * s + 8 * (g >> 1) + q;
      const int col = rb + 16 * (g & 1) + 4 * pp;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4 *)(plane + tswz<R>(k, col)));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4 *)(plane + tswz<R>(k + 4, col)));
      const s16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(f16x8, c);
    }
  }
};


// The scale exponents of the tile's rows and columns into sexp, and each
// one's spread weight into sw (f16-split.h spread_weight: 0 unless the group
// is spread; -inf for an all-zero group, whose products are exactly 0: the
// threshold sum is then -inf, i.e. no check).  Returns bit 0: one of them is
// an Inf / NaN row or column; bit 1: one of them is spread (both for the
// whole block).
__device__ __forceinline__ int tile_scales(const GemmF16Args &p, int *sexp, float *sw, int row0,
                                           int col0, int tid) {
#ifdef KCNN_EXPERIMENTS  // KCNN_GEMM_DEBUG & 4: no statistics loads (scale 0; timing only)
  if (p.dbg & 64) {
    for (int i = tid; i < BM + BN; i += NT) {
      sexp[i] = 0;
      sw[i] = 0.0f;
    }
    __syncthreads();
    return 0;
  }
#endif
  int skip = 0, spr = 0;
  for (int i = tid; i < BM + BN; i += NT) {
    int s = 0;
    float w = 0.0f;
    if (i < BM) {
      if (row0 + i < p.M) {
        const uint32_t m = p.amax[row0 + i];
        s = scale_exp(m);
        w = m == 0 ? -__builtin_inff() : kcnn::f16x3::spread_weight(p.acnt[row0 + i]);
      }
    } else if (col0 + i - BM < p.N) {
      const uint32_t m = p.bmax[col0 + i - BM];
      s = scale_exp(m);
      w = m == 0 ? -__builtin_inff() : kcnn::f16x3::spread_weight(p.bcnt[col0 + i - BM]);
    }
    sexp[i] = s;
    sw[i] = w;
    skip |= s == SKIP;
    spr |= w > 0.0f;
  }
  const int any_skip = __syncthreads_or(skip) != 0;
  return any_skip | (__syncthreads_or(spr) != 0 ? 2 : 0);
}

// One C element by a whole wave, for the store's check (called with the same
// row and column in every lane): fp32 products of op(A) row i and op(B)
// column j in a fixed order per lane, then a butterfly over the lanes (every
// lane ends with the same bits: deterministic)
__device__ __forceinline__ float wave_dot(const GemmF16Args &p, bool a_kc, bool b_kc, int row,
                                          int col, int lane) {
  // element k of the row of op(A) / column of op(B): qa[k * sa], qb[k * sb]
  // (wave-uniform strides; the pointers step, no per-load index products)
  const int64_t sa = a_kc ? 1 : p.lda, sb = b_kc ? 1 : p.ldb;
  const float *qa = (a_kc ? p.A + (int64_t)row * p.lda : p.A + row) + lane * sa;
  const float *qb = (b_kc ? p.B + (int64_t)col * p.ldb : p.B + col) + lane * sb;
  const int64_t da = 64 * sa, db = 64 * sb;
  // four partial sums (k = lane + 64 (4 i + j) into sum j): eight loads in
  // flight per lane instead of one
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int k = lane;
#pragma unroll 1
  for (; k + 192 < p.K; k += 256) {
    float x[4], y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = qa[j * da];
      y[j] = qb[j * db];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = fmaf(x[j], y[j], s[j]);
    qa += 4 * da;
    qb += 4 * db;
  }
#pragma unroll 1
  for (; k < p.K; k += 64) {
    s[0] = fmaf(*qa, *qb, s[0]);
    qa += da;
    qb += db;
  }
  float t = (s[0] + s[1]) + (s[2] + s[3]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
  return t;
}
__device__ __forceinline__ float store_value(const GemmF16Args &p, float v, float *o, int col) {
  float r = p.beta == 0.0f ? p.alpha * v : p.alpha * v + p.beta * *o;
  if (p.bias) r += p.bias[col];
  return r;
}
// C[row][col] from the product's value v; with p.mom.W the element is instead
// the gradient of the momentum update (momentum-step.h: alpha * v, beta 0, no
// bias), applied to W and prev in place of storing C
__device__ __forceinline__ void emit(const GemmF16Args &p, int row, int col, float v) {
  if (p.mom.W) {
    float *w = p.mom.W + (int64_t)row * p.mom.ldw + col;
    float *q = p.mom.prev + (int64_t)row * p.mom.ldp + col;
    float wv = *w, pv = *q;
    kcnn::momentum_step(p.alpha * v, pv, wv, p.mom.momentum, p.mom.a_wd, p.mom.a_g);
    *q = pv;
    *w = wv;
    return;
  }
  float *o = p.C + (int64_t)row * p.ldc + col;
  *o = store_value(p, v, o, col);
}
// The elements a lane's check rejected (bit n of `mine` its n-th candidate,
// decode(lane, n) -> (row, col)), each recomputed by the whole wave
// (wave_dot) and handed to put(l, n, row, col, v) on lane 0: a wave-uniform
// loop over the wave's rejections
template <typename Decode, typename Put>
__device__ __forceinline__ void fix_rejected(const GemmF16Args &p, bool a_kc, bool b_kc,
                                             uint64_t mine, int lane, Decode decode, Put put) {
  for (;;) {
    const uint64_t who = __ballot(mine != 0);
    if (who == 0) break;
    const int l = __builtin_ctzll(who);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mine, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(mine >> 32), l);
    const uint64_t bits = ((uint64_t)hi << 32) | lo;
    const int n = __builtin_ctzll(bits);
    int row, col;
    decode(l, n, row, col);
    const float v = wave_dot(p, a_kc, b_kc, row, col, lane);
    if (lane == 0) put(l, n, row, col, v);
    if (lane == l) mine &= mine - 1;
  }
}
template <typename Decode>
__device__ __forceinline__ void fix_rejected(const GemmF16Args &p, bool a_kc, bool b_kc,
                                             uint64_t mine, int lane, Decode decode) {
  fix_rejected(p, a_kc, b_kc, mine, lane, decode,
               [&](int, int, int row, int col, float v) { emit(p, row, col, v); });
}

// The tile's results.  C/D map of 32x32x16: register g of lane l holds row
// (g & 3) + 8 (g >> 2) + 4 (l >> 5), column l & 31.  Each value is unscaled
// by 2^-(s_row + s_col) (exact).
//  - One split (or a whole tile of a split grid, block_tile): C = alpha * v
//    + beta * C.
//  - ksplit > 1: the split's values go to its partial slab, which
//    gemm_f16x3_reduce_kernel adds in increasing split order.  (Adding them
//    in the tile's last-arriving workgroup instead needs a device-scope
//    release fence per workgroup, which on gfx950 writes back the XCD's L2:
//    the c2 FC forward went 330 -> 436 us and the weight gradient 368 ->
//    654 us with it.)
//  - Elements of an Inf / NaN row or column are skipped above; split 0's
//    workgroup computes them here as fp32 dot products in increasing k
//    (IEEE Inf / NaN, the reference sgemm's pattern).
template <bool A_KC, bool B_KC>
__device__ __forceinline__ void tile_epilogue(const GemmF16Args &p, const int *sexp,
                                              const float *sw, const f32x16 (&acc)[2][2],
                                              int split, bool whole, int row0, int col0,
                                              int flags, int tid, char *lds) {
  const int lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int half2 = lane >> 5;
  const bool partial = p.ksplit > 1 && !whole;
  const bool skip = flags & 1;
  // the spread check (f16-split.h): with a spread row or column in the tile
  // and one split, an element whose |acc| is below its threshold is
  // recomputed in fp32 (fix_rejected) instead of stored; split K checks the
  // summed value in gemm_f16x3_reduce_kernel
  const bool check = (flags & 2) && !partial;
  const int np4 = (p.N + 3) & ~3;  // partial slab pitch (16-B rows)
  float *slab = partial ? p.part + (int64_t)split * p.M * np4 : p.C;
  const int ldo = partial ? np4 : p.ldc;
  uint64_t rej = 0;  // bit (2 i + j) * 16 + g: that element is rejected
  auto fix = [&]() {
    fix_rejected(p, A_KC, B_KC, rej, lane, [&](int l, int n, int &row, int &col) {
      const int i = n >> 5, j = (n >> 4) & 1, g = n & 15;
      row = row0 + wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * (l >> 5);
      col = col0 + wn * 64 + j * 32 + (l & 31);
    });
  };
  // A whole tile without Inf / NaN rows or columns (block-uniform): each
  // wave's 64 x 64 block through LDS in two 32-row halves (the main loop's
  // plane buffers, free after a barrier), then 16-B stores of whole rows:
  // a quarter of the store instructions of the per-register stores below
  // (c2's data gradient: 400 -> 388 us at K 1024).  An element the check
  // rejects is recomputed by its wave (fix_rejected) into its staging slot
  // before the half is stored, so alpha, beta * C and the bias are applied
  // to it once, by the same 16-B store as its neighbours (a
  // second store_value after the staged store read back the new C).
  // (the momentum update's W and prev have 16-B aligned rows: host check)
  const bool staged = row0 + BM <= p.M && col0 + BN <= p.N && !skip &&
                      (partial || p.mom.W || ((ldo & 3) | ((uintptr_t)slab & 15)) == 0)
#ifdef KCNN_EXPERIMENTS  // KCNN_GEMM_DEBUG & 8: the per-register stores only
                      && !(p.dbg & 128)
#endif
      ;
  if (staged) {
    __syncthreads();  // every wave past its last read of the plane buffers
    constexpr int SR = 68;  // staging row pitch (floats): 16-B rows, rows 4 apart on other banks
    float *st = reinterpret_cast<float *>(lds) + wave * 32 * SR;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cl = wn * 64 + j * 32 + (lane & 31);
        const int ec = sexp[BM + cl];
        const float wc = check ? sw[BM + cl] : 0.0f;
        const bool bcheck =
            check && (__ballot(wc > 0.0f || sw[wm * 64 + i * 32 + (lane & 31)] > 0.0f) != 0);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int rr = (g & 3) + 8 * (g >> 2) + 4 * half2;
          const int rl = wm * 64 + i * 32 + rr;
          if (bcheck) {
            const float thr = wc + sw[rl];
            if (thr != 0.0f && !(fabsf(acc[i][j][g]) >= thr))
              rej |= (uint64_t)1 << ((2 * i + j) * 16 + g);
          }
          st[rr * SR + j * 32 + (lane & 31)] =
              __builtin_amdgcn_ldexpf(acc[i][j][g], -(sexp[rl] + ec));
        }
      }
      if (check) {
        // this half's rejections (bits 32 i .. 32 i + 31) into their slots
        // (lane 0 writes after every lane's staging write: one wave, LDS in order)
        const uint64_t mine = (rej >> (32 * i)) & 0xffffffffull;
        fix_rejected(
            p, A_KC, B_KC, mine, lane,
            [&](int l, int n, int &row, int &col) {
              const int j = (n >> 4) & 1, g = n & 15;
              row = row0 + wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * (l >> 5);
              col = col0 + wn * 64 + j * 32 + (l & 31);
            },
            [&](int l, int n, int, int, float v) {
              const int j = (n >> 4) & 1, g = n & 15;
              const int rr = (g & 3) + 8 * (g >> 2) + 4 * (l >> 5);
              st[rr * SR + j * 32 + (l & 31)] = v;
            });
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int f = lane + 64 * k, rr = f >> 4, c4 = f & 15;
        const float4 v = *reinterpret_cast<const float4 *>(st + rr * SR + 4 * c4);
        const int row = row0 + wm * 64 + i * 32 + rr, col = col0 + wn * 64 + 4 * c4;
        if (!partial && p.mom.W) {  // emit's momentum step, four elements per access
          float4 *wq = reinterpret_cast<float4 *>(p.mom.W + (int64_t)row * p.mom.ldw + col);
          float4 *pq = reinterpret_cast<float4 *>(p.mom.prev + (int64_t)row * p.mom.ldp + col);
          float4 w4 = *wq, q4 = *pq;
          const MomentumEpi &m = p.mom;
          kcnn::momentum_step(p.alpha * v.x, q4.x, w4.x, m.momentum, m.a_wd, m.a_g);
          kcnn::momentum_step(p.alpha * v.y, q4.y, w4.y, m.momentum, m.a_wd, m.a_g);
          kcnn::momentum_step(p.alpha * v.z, q4.z, w4.z, m.momentum, m.a_wd, m.a_g);
          kcnn::momentum_step(p.alpha * v.w, q4.w, w4.w, m.momentum, m.a_wd, m.a_g);
          *pq = q4;
          *wq = w4;
          continue;
        }
        float4 *o = reinterpret_cast<float4 *>(slab + (int64_t)row * ldo + col);
        if (partial) {
          *o = v;
          continue;
        }
        float4 w = make_float4(p.alpha * v.x, p.alpha * v.y, p.alpha * v.z, p.alpha * v.w);
        if (p.beta != 0.0f) {
          const float4 c = *o;
          w = make_float4(p.alpha * v.x + p.beta * c.x, p.alpha * v.y + p.beta * c.y,
                          p.alpha * v.z + p.beta * c.z, p.alpha * v.w + p.beta * c.w);
        }
        if (p.bias) {
          w.x += p.bias[col];
          w.y += p.bias[col + 1];
          w.z += p.bias[col + 2];
          w.w += p.bias[col + 3];
        }
        *o = w;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = wn * 64 + j * 32 + (lane & 31);
      const int col = col0 + cl;
      const int ec = sexp[BM + cl];
      if (col >= p.N || ec == SKIP) continue;
      const float wc = check ? sw[BM + cl] : 0.0f;
      // this 32 x 32 block's check: one of its columns or rows is spread
      // (wave-uniform; most blocks skip it)
      const bool bcheck =
          check && (__ballot(wc > 0.0f || sw[wm * 64 + i * 32 + (lane & 31)] > 0.0f) != 0);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rl = wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * half2;
        const int row = row0 + rl;
        const int er = sexp[rl];
        if (row >= p.M || er == SKIP) continue;
        if (bcheck) {
          const float thr = wc + sw[rl];
          if (thr != 0.0f && !(fabsf(acc[i][j][g]) >= thr)) {
            rej |= (uint64_t)1 << ((2 * i + j) * 16 + g);
            continue;
          }
        }
        const float v = __builtin_amdgcn_ldexpf(acc[i][j][g], -(er + ec));
#ifdef KCNN_EXPERIMENTS  // KCNN_GEMM_DEBUG & 1: no stores, & 2: nontemporal stores
        if (p.dbg & 16) continue;
        if (p.dbg & 32) {
          float *o = partial ? slab + (int64_t)row * ldo + col : p.C + (int64_t)row * p.ldc + col;
          __builtin_nontemporal_store(partial ? v : store_value(p, v, o, col), o);
          continue;
        }
#endif
        if (partial) slab[(int64_t)row * ldo + col] = v;
        else emit(p, row, col, v);
      }
    }
  if (check) fix();
  if (skip && split == 0) {
    for (int e = tid; e < BM * BN; e += NT) {
      const int rl = e / BN, cl = e - rl * BN;
      const int row = row0 + rl, col = col0 + cl;
      if (row >= p.M || col >= p.N) continue;
      if (sexp[rl] != SKIP && sexp[BM + cl] != SKIP) continue;
      float sum = 0.0f;
      for (int k = 0; k < p.K; ++k) {
        const float a = A_KC ? p.A[(int64_t)row * p.lda + k] : p.A[(int64_t)k * p.lda + row];
        const float b = B_KC ? p.B[(int64_t)col * p.ldb + k] : p.B[(int64_t)k * p.ldb + col];
        sum = fmaf(a, b, sum);
      }
      emit(p, row, col, sum);
    }
  }
}

template <int AM, int BMODE, bool RAG>
__global__ __launch_bounds__(NT, 1) void gemm_f16x3_kernel(GemmF16Args p) {
  constexpr bool A_KC = AM == LK, B_KC = BMODE == LK;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int *sexp = reinterpret_cast<int *>(lds + 2 * BUF);  // [BM] rows, then [BN] columns
  float *sw = reinterpret_cast<float *>(sexp + BM + BN);  // spread weights, the same order
  const int tid = threadIdx.x;
  const float m1 = kcnn::f16x3::opaque_m1();
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int split, tm, tn;
  const bool whole = block_tile(p, split, tm, tn);
  const int row0 = tm * BM, col0 = tn * BN;
  const int kbeg = whole ? 0 : split * p.kps;
  const int kend = whole ? p.K : min(p.K, kbeg + p.kps);
  const int T = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int klast = kend - kbeg - (T - 1) * BK;  // valid k of the last tile

  const int flags = tile_scales(p, sexp, sw, row0, col0, tid);

  // descriptors whose range ends at the operand's last element: a partial
  // last tile reads 0 past it (and the split zeroes the pitch's padding)
  const float *baseA = A_KC ? p.A + (int64_t)row0 * p.lda : p.A + (int64_t)kbeg * p.lda + row0;
  const float *baseB = B_KC ? p.B + (int64_t)col0 * p.ldb : p.B + (int64_t)kbeg * p.ldb + col0;
  const int vra = p.M - row0, vrb = p.N - col0;
  const int64_t endA = A_KC ? ((int64_t)(vra - 1) * p.lda + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.lda + vra) * 4;
  const int64_t endB = B_KC ? ((int64_t)(vrb - 1) * p.ldb + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.ldb + vrb) * 4;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseA, (short)0, (int)(endA < 0x7fffffff ? endA : 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseB, (short)0, (int)(endB < 0x7fffffff ? endB : 0x7fffffff), 0x00020000);
  // k of tile t relative to the base (clamped to the last tile: a re-read)
  auto kk = [&](int t, bool kc) { return (kc ? kbeg : 0) + min(t, T - 1) * BK; };

  using LA = Loader<BM, AM>;
  using LB = Loader<BN, BMODE>;
  LA la[2];
  LB lb[2];
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.0f;
  la[0].init_exp(sexp, tid);
  la[1].init_exp(sexp, tid);
  lb[0].init_exp(sexp + BM, tid);
  lb[1].init_exp(sexp + BM, tid);

  if (T > 0) {
    la[0].load(rsA, p.lda, vra, kk(0, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(0, B_KC), tid);
    la[0].template store<A_PLANE, RAG>(lds, tid, T == 1 ? klast : BK, m1);
    lb[0].template store<B_PLANE, RAG>(lds + 2 * A_PLANE, tid, T == 1 ? klast : BK, m1);
    // tiles 1, 2 into sets 1, 0 (as at every later loop entry)
    __builtin_amdgcn_sched_barrier(0);
    la[1].load(rsA, p.lda, vra, kk(1, A_KC), tid);
    lb[1].load(rsB, p.ldb, vrb, kk(1, B_KC), tid);
    __builtin_amdgcn_sched_barrier(0);
    la[0].load(rsA, p.lda, vra, kk(2, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(2, B_KC), tid);
    __syncthreads();

    const int ar = wm * 64, br = wn * 64;
    // one k16 half of a step: 8 fragments, 12 MFMAs
    auto half_step = [&](const char *bufA, int s) {
      const char *bufB = bufA + 2 * A_PLANE;
      f16x8 a[2][2], bb[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          a[i][pl] = LA::frag(bufA + pl * A_PLANE, ar + 32 * i, s, lane);
          bb[i][pl] = LB::frag(bufB + pl * B_PLANE, br + 32 * i, s, lane);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 x = acc[i][j];
          x = mfma(a[i][1], bb[j][0], x);  // lo hi
          x = mfma(a[i][0], bb[j][1], x);  // hi lo
          x = mfma(a[i][0], bb[j][0], x);  // hi hi
          acc[i][j] = x;
        }
    };
    // waves 4-7 split the next tile between their two MFMA halves, waves
    // 0-3 after both (gemm_x6_kernel's stagger)
    const bool late = wave < 4;
    // step t: tile t+1 is in set (t+1) & 1, which then takes tile t+3 (a
    // step past T issues its clamped loads too, so every path issues the
    // same loads and each split waits only for its own tile)
    auto step = [&](int t, LA &lan, LB &lbn) {
      if (t < T) {
        const char *buf = lds + (t & 1) * BUF;
        char *nA = lds + ((t + 1) & 1) * BUF;
        const int kv = t + 2 == T ? klast : BK;
        half_step(buf, 0);
        if (!late && t + 1 < T) {
          lan.template store<A_PLANE, RAG>(nA, tid, kv, m1);
          lbn.template store<B_PLANE, RAG>(nA + 2 * A_PLANE, tid, kv, m1);
        }
        half_step(buf, 1);
        if (late && t + 1 < T) {
          lan.template store<A_PLANE, RAG>(nA, tid, kv, m1);
          lbn.template store<B_PLANE, RAG>(nA + 2 * A_PLANE, tid, kv, m1);
        }
      }
      lan.load(rsA, p.lda, vra, kk(t + 3, A_KC), tid);
      lbn.load(rsB, p.ldb, vrb, kk(t + 3, B_KC), tid);
      __syncthreads();
    };
    for (int t = 0; t < T; t += 2) {
      step(t, la[1], lb[1]);
      step(t + 1, la[0], lb[0]);
    }
  }

  tile_epilogue<A_KC, B_KC>(p, sexp, sw, acc, split, whole, row0, col0, flags, tid, lds);
}

// ---------------------------------------------------------------------------
// gemm_f16x3_fast_kernel: gemm_f16x3_kernel's arithmetic (the same images,
// fragments and MFMA order into every accumulator: bitwise the same C) with
// one barrier per K step in its middle and the LDS traffic moved under the
// MFMAs.  K step t:
//   phase A: the 12 k16-half-0 MFMAs (fragments F0, read in the previous
//            phase B); beside them the split of tile t+1 into the other
//            buffer (one pair per MFMA) and the reads of the half-1
//            fragments F1;
//   barrier: tile t+1 written, buffer t & 1 read by every wave;
//   phase B: the 12 half-1 MFMAs; beside them the F0 reads of step t+1 (from
//            the other buffer) and the HBM loads of tile t+3.
// Each MFMA and the work placed after it are fenced (sched_barrier), so this
// is the issue order.  The bf16x6 kernel of this shape (cu-gemm-x6.hip
// gemm_x6_fast_kernel) measured no faster: its six products held the chip at
// its power limit.  f16x3's three leave the clock up, and the MFMA pipe idles
// on LDS latency instead (35-44 % busy at 2.1-2.3 GHz with the two-phase
// loop).
template <int AM, int BMODE, bool RAG>
__global__ __launch_bounds__(NT, 1) void gemm_f16x3_fast_kernel(GemmF16Args p) {
  constexpr bool A_KC = AM == LK, B_KC = BMODE == LK;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int *sexp = reinterpret_cast<int *>(lds + 2 * BUF);
  float *sw = reinterpret_cast<float *>(sexp + BM + BN);
  const int tid = threadIdx.x;
  const float m1 = kcnn::f16x3::opaque_m1();
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int split, tm, tn;
  const bool whole = block_tile(p, split, tm, tn);
  const int row0 = tm * BM, col0 = tn * BN;
  const int kbeg = whole ? 0 : split * p.kps;
  const int kend = whole ? p.K : min(p.K, kbeg + p.kps);
  const int T = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int klast = kend - kbeg - (T - 1) * BK;

  const float *baseA = A_KC ? p.A + (int64_t)row0 * p.lda : p.A + (int64_t)kbeg * p.lda + row0;
  const float *baseB = B_KC ? p.B + (int64_t)col0 * p.ldb : p.B + (int64_t)kbeg * p.ldb + col0;
  const int vra = p.M - row0, vrb = p.N - col0;
  const int64_t endA = A_KC ? ((int64_t)(vra - 1) * p.lda + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.lda + vra) * 4;
  const int64_t endB = B_KC ? ((int64_t)(vrb - 1) * p.ldb + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.ldb + vrb) * 4;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseA, (short)0, (int)(endA < 0x7fffffff ? endA : 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseB, (short)0, (int)(endB < 0x7fffffff ? endB : 0x7fffffff), 0x00020000);
  auto kk = [&](int t, bool kc) { return (kc ? kbeg : 0) + min(t, T - 1) * BK; };

  using LA = Loader<BM, AM>;
  using LB = Loader<BN, BMODE>;
  LA la[2];
  LB lb[2];
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.0f;

  const int ar = wm * 64, br = wn * 64;
  f16x8 fa0[2][2], fb0[2][2], fa1[2][2], fb1[2][2];
  // r-th fragment of half s: A fragments (i, plane) first, then B
  auto read_frag = [&](const char *buf, int s, int r, f16x8 (&fa)[2][2], f16x8 (&fb)[2][2]) {
    if (r < 4) {
      const int i = r >> 1, pl = r & 1;
      fa[i][pl] = LA::frag(buf + pl * A_PLANE, ar + 32 * i, s, lane);
    } else {
      const int i = (r - 4) >> 1, pl = (r - 4) & 1;
      fb[i][pl] = LB::frag(buf + 2 * A_PLANE + pl * B_PLANE, br + 32 * i, s, lane);
    }
  };
  // n-th MFMA of a half: accumulator (n / 6, (n / 3) % 2), lo.hi, hi.lo, hi.hi
  auto mfma_n = [&](int n, const f16x8 (&fa)[2][2], const f16x8 (&fb)[2][2]) {
    const int i = n / 6, j = (n / 3) & 1, pr = n % 3;
    constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#ifdef KCNN_GEMM_XNOMFMA  // experiment build: timing without the products
    asm volatile("" ::"v"(fa[i][PA[pr]]), "v"(fb[j][PB[pr]]));
#else
    acc[i][j] = mfma(fa[i][PA[pr]], fb[j][PB[pr]], acc[i][j]);
#endif
  };

  // waves 4-7 (each SIMD's second wave) at priority 1 for the whole kernel
  // (MI355X_MICROARCH.md, two waves per SIMD, item 4: the younger half loses
  // every VALU arbitration otherwise)
#ifndef KCNN_GEMM_PRIO
#define KCNN_GEMM_PRIO 1
#endif
  if (KCNN_GEMM_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  // the first two K tiles' loads go out before the tile's scales are read
  // (the split needs both; the scales' loads and barriers then pass under
  // the tiles' latency: c2's data gradient 400 -> 381 us at K 1024 without
  // the scales at all)
  if (T > 0) {
    la[0].load(rsA, p.lda, vra, kk(0, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(0, B_KC), tid);
    la[1].load(rsA, p.lda, vra, kk(1, A_KC), tid);
    lb[1].load(rsB, p.ldb, vrb, kk(1, B_KC), tid);
  }
  __builtin_amdgcn_sched_barrier(0);
  const int flags = tile_scales(p, sexp, sw, row0, col0, tid);
  la[0].init_exp(sexp, tid);
  la[1].init_exp(sexp, tid);
  lb[0].init_exp(sexp + BM, tid);
  lb[1].init_exp(sexp + BM, tid);
  if (T > 0) {
    la[0].template store<A_PLANE, RAG>(lds, tid, T == 1 ? klast : BK, m1);
    lb[0].template store<B_PLANE, RAG>(lds + 2 * A_PLANE, tid, T == 1 ? klast : BK, m1);
    __builtin_amdgcn_sched_barrier(0);
    la[0].load(rsA, p.lda, vra, kk(2, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(2, B_KC), tid);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) read_frag(lds, 0, r, fa0, fb0);

    // step t: tile t+1 is in set (t+1) & 1 (split in phase A), which then
    // takes tile t+3 (phase B; a step past T issues its clamped loads too)
    // (more_c: std::true_type where the step is known not to be the last,
    // so its split and next-fragment reads carry no branch; std::false_type
    // for the last step, which has neither)
    auto step = [&](int t, LA &lan, LB &lbn, auto more_c) {
      const char *buf = lds + (t & 1) * BUF;
      char *nbuf = lds + ((t + 1) & 1) * BUF;
      constexpr bool more = decltype(more_c)::value;
      const int kv = t + 2 == T ? klast : BK;
      uint32_t ph[4], pl[4];
      // phase A
#pragma unroll
      for (int n = 0; n < 12; ++n) {
        mfma_n(n, fa0, fb0);
        if (more) {
          if (n < LA::NPIECE)
            lan.template piece<A_PLANE, RAG>(nbuf, tid, n, kv, ph, pl, m1);
          else if (n - LA::NPIECE < LB::NPIECE)
            lbn.template piece<B_PLANE, RAG>(nbuf + 2 * A_PLANE, tid, n - LA::NPIECE, kv, ph, pl, m1);
        }
        if (n >= 2 && n < 10) read_frag(buf, 1, n - 2, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
      // phase B
#pragma unroll
      for (int n = 0; n < 12; ++n) {
        mfma_n(n, fa1, fb1);
#ifndef KCNN_GEMM_XNOLOAD  // experiment build: timing without the main loop's loads
        if (n == 1) lan.load(rsA, p.lda, vra, kk(t + 3, A_KC), tid);
        if (n == 3) lbn.load(rsB, p.ldb, vrb, kk(t + 3, B_KC), tid);
#endif
        if (more && n >= 2 && n < 10) read_frag(nbuf, 0, n - 2, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    int t = 0;
    // every step of the loop has a successor; the last one or two after it
    for (; t + 2 < T; t += 2) {
      step(t, la[1], lb[1], std::true_type{});
      step(t + 1, la[0], lb[0], std::true_type{});
    }
    if (t + 1 < T) {
      step(t, la[1], lb[1], std::true_type{});
      step(t + 1, la[0], lb[0], std::false_type{});
    } else {
      step(t, la[1], lb[1], std::false_type{});
    }
  }

  tile_epilogue<A_KC, B_KC>(p, sexp, sw, acc, split, whole, row0, col0, flags, tid, lds);
}

// Max |x| and min nonzero |x| per row or per column of a pitched fp32 matrix,
// as the bit patterns of |x| (unsigned order = magnitude order, Inf / NaN
// above every finite value; max and min are order-independent, so the
// results are deterministic), and for a spread group (f16-split.h: an
// element far enough below the max to lose low bits, which the GEMM's store
// then checks, tile_epilogue) the count of its elements held only to 2^-25
// (an integer: deterministic).  A group set's statistics block is
// [max[n], min[n], cnt[n]] (n groups): max[i] sets the group's f16x3 scale,
// min[i] (0: no nonzero element) says whether the group is spread, cnt[i]
// (0 unless spread here) sizes its check.  The check is sound for any count
// that covers the group's small elements (each is held to 2^-25, spread or
// not), so a producer may also count them in a group that is not spread
// (the pooled output's columns, pool-stats.h): that only adds checks.  The
// min is taken as min(|x| - 1) in wrapping unsigned arithmetic, so a zero
// (0 - 1 = 0xffffffff) never wins, then + 1.
// A GEMM needs op(A)'s rows and op(B)'s columns; both operands' statistics
// go in one launch (stats_kernel: blocks [0, a.blocks) for A, then B's) and
// one more (stats_finalize_kernel) when either is per column:
//  rows, cols >= 2048: a block per row (thread t reads float4 t + 256 i,
//    four in flight), a wave reduction and an LDS step;
//  rows, shorter rows: a wave per row;
//  columns: block (cb, rc) covers 1024 columns (4 per thread) of a chunk of
//    rows (8 in flight) and stores its column maxima and minima as partial
//    rc; the finalize takes the maxima / minima over the chunks (64 columns
//    x 4 chunk groups per block, combined through LDS).
struct StatOp {
  const float *X;
  uint32_t *out;   // the statistics block [max, min, cnt], per row (mode 0) or column (1)
  uint32_t *part;  // mode 1: [2][rbk][cols] partials (maxima, then minima - 1)
  int rows, cols, ld, mode, vec;
  int blocks;      // of stats_kernel
  int rpb;         // mode 0: rows per block (4: a wave each; 1: a block)
  int cb, rbk, rb; // mode 1: column blocks, row chunks, rows per chunk
  int fblocks;     // mode 1: blocks of stats_finalize_kernel
  uint32_t *clear; // nullable: two words stats_kernel sets to 0 (a consumer's counters)
};
__device__ __forceinline__ const float *X_row(const StatOp &o, int r) {
  return o.X + (int64_t)r * o.ld;
}

// running max |x| (m) and min (|x| - 1) (n) over a float4
__device__ __forceinline__ void mm4(uint32_t &m, uint32_t &n, float4 q) {
  const uint32_t a = __float_as_uint(q.x) & 0x7fffffffu, b = __float_as_uint(q.y) & 0x7fffffffu,
                 c = __float_as_uint(q.z) & 0x7fffffffu, d = __float_as_uint(q.w) & 0x7fffffffu;
  m = max(max(m, a), max(max(b, c), d));
  n = min(min(n, a - 1u), min(min(b - 1u, c - 1u), d - 1u));
}
__device__ __forceinline__ void mm1(uint32_t &m, uint32_t &n, float x) {
  const uint32_t a = __float_as_uint(x) & 0x7fffffffu;
  m = max(m, a);
  n = min(n, a - 1u);
}

// the nonzero |x| of row r below bound (a spread row's count; sweep of
// stats_rows' shape)
__device__ __forceinline__ uint32_t count_small_row(const StatOp &o, const float *x, float bound,
                                                    int c, int step) {
  uint32_t n = 0;
  for (; c < o.cols; c += step)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (c + i < o.cols) {
        const float a = fabsf(x[c + i]);
        n += (a < bound && a != 0.0f) ? 1u : 0u;
      }
  return n;
}

// A row held in registers by the sweep (RV float4 per thread: up to 18432
// floats per block row, 4608 per wave row), so that a spread row counts its
// small elements without a second read (c5's C3 input and output derivative
// rows are 18432 floats, and the derivative's frames are all spread: a
// second read doubled that pass, 83 us per call)
constexpr int RV = 18;
__device__ __forceinline__ void stats_rows(const StatOp &o, int blk, uint32_t *red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool wide = o.rpb == 1;
  const int r = wide ? blk : blk * 4 + wave;
  if (r >= o.rows) return;  // (wide: uniform over the block)
  const float *x = X_row(o, r);
  const int step = wide ? 1024 : 256;  // floats per sweep of the row
  const int c0 = (wide ? threadIdx.x : lane) * 4;
  const bool held = o.vec && o.cols <= RV * step;  // uniform
  float4 q[RV];
  uint32_t m = 0, n = 0xffffffffu;
  if (held) {  // every load in flight at once; past the row: zeros (never max, min or small)
#pragma unroll
    for (int j = 0; j < RV; ++j) {
      const int c = c0 + j * step;
      if (c + 4 <= o.cols) {
        q[j] = *reinterpret_cast<const float4 *>(x + c);
      } else {
        q[j].x = c < o.cols ? x[c] : 0.0f;
        q[j].y = c + 1 < o.cols ? x[c + 1] : 0.0f;
        q[j].z = c + 2 < o.cols ? x[c + 2] : 0.0f;
        q[j].w = 0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < RV; ++j) mm4(m, n, q[j]);
  } else {
    int c = c0;
    if (o.vec) {
      for (; c + 3 * step + 4 <= o.cols; c += 4 * step) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const float4 *>(x + c + j * step);
#pragma unroll
        for (int j = 0; j < 4; ++j) mm4(m, n, v[j]);
      }
      for (; c + 4 <= o.cols; c += step) mm4(m, n, *reinterpret_cast<const float4 *>(x + c));
    }
    for (; c < o.cols; c += step)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (c + i < o.cols) mm1(m, n, x[c + i]);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    m = max(m, (uint32_t)__shfl_xor((int)m, d));
    n = min(n, (uint32_t)__shfl_xor((int)n, d));
  }
  if (wide) {  // the block's maxima / minima through LDS, to every thread
    if (lane == 0) {
      red[wave] = m;
      red[4 + wave] = n;
    }
    __syncthreads();
    m = max(max(red[0], red[1]), max(red[2], red[3]));
    n = min(min(red[4], red[5]), min(red[6], red[7]));
  }
  // a spread row (f16-split.h) counts its small elements (from the registers,
  // or a second sweep of the row from L2); every other row's count is 0
  uint32_t cnt = 0;
  if (kcnn::f16x3::spread(m, n + 1u)) {  // uniform over the wave (the block)
    const float bound = kcnn::f16x3::small_bound(m);
    if (held) {
      auto small = [&](float v) { return (fabsf(v) < bound && v != 0.0f) ? 1u : 0u; };
#pragma unroll
      for (int j = 0; j < RV; ++j)
        cnt += small(q[j].x) + small(q[j].y) + small(q[j].z) + small(q[j].w);
    } else {
      cnt = count_small_row(o, x, bound, c0, step);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, d);
    if (wide) {
      __syncthreads();  // (red's maxima read above)
      if (lane == 0) red[8 + wave] = cnt;
      __syncthreads();
      cnt = red[8] + red[9] + red[10] + red[11];
    }
  }
  if (wide ? threadIdx.x == 0 : lane == 0) {
    o.out[r] = m;
    o.out[o.rows + r] = n + 1u;
    o.out[2 * (size_t)o.rows + r] = cnt;
  }
}

__device__ __forceinline__ void stats_cols(const StatOp &o, int blk) {
  const int cbi = blk % o.cb, rci = blk / o.cb;
  const int c0 = cbi * 1024 + threadIdx.x * 4;
  const int r0 = rci * o.rb, rend = min(o.rows, r0 + o.rb);
  if (c0 >= o.cols) return;
  const bool v4 = o.vec && c0 + 4 <= o.cols;
  uint32_t cm[4] = {0u, 0u, 0u, 0u};
  uint32_t cn[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  auto load = [&](int r) {
    const float *x = X_row(o, r) + c0;
    if (v4) return *reinterpret_cast<const float4 *>(x);
    float4 q;
    q.x = x[0];
    q.y = c0 + 1 < o.cols ? x[1] : 0.0f;
    q.z = c0 + 2 < o.cols ? x[2] : 0.0f;
    q.w = c0 + 3 < o.cols ? x[3] : 0.0f;
    return q;
  };
  auto take = [&](float4 q) {
    mm1(cm[0], cn[0], q.x);
    mm1(cm[1], cn[1], q.y);
    mm1(cm[2], cn[2], q.z);
    mm1(cm[3], cn[3], q.w);
  };
  int r = r0;
  for (; r + 8 <= rend; r += 8) {
    float4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = load(r + j);
#pragma unroll
    for (int j = 0; j < 8; ++j) take(q[j]);
  }
  for (; r < rend; ++r) take(load(r));
  uint32_t *dst = o.part + (size_t)rci * o.cols + c0;
  uint32_t *dsn = dst + (size_t)o.rbk * o.cols;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (c0 + i < o.cols) {
      dst[i] = cm[i];
      dsn[i] = cn[i];
    }
}

// Up to three statistics passes in one launch (their blocks in order): a
// GEMM's two operands, or the FC backward's output derivative (rows and
// columns) and weight columns (kl_gemm_stats3)
struct StatOps {
  StatOp o[3];
  // a fused pool's pending column statistics (pool-stats-dev.h): pcx x pcy
  // colmax blocks after the ops' blocks in stats_kernel, pcn count blocks
  // after the finalize blocks in stats_finalize_kernel (0: none)
  PoolColDeferred pc;
  int pcx, pcy, pcn;
};
// the op of block `blk` among the ops' `count(o)` blocks, and its block index there
template <typename Count>
__device__ __forceinline__ int pick_op(const StatOps &s, int blk, Count count, int &local) {
  const int n0 = count(s.o[0]), n1 = count(s.o[1]);
  if (blk < n0) { local = blk; return 0; }
  if (blk < n0 + n1) { local = blk - n0; return 1; }
  local = blk - n0 - n1;
  return 2;
}
__host__ __device__ inline int ncount_blocks(const StatOp &o);
__host__ __device__ inline int nfinal_blocks(const StatOp &o) {
  return o.mode == 1 && o.blocks ? o.fblocks : 0;
}

__global__ __launch_bounds__(256) void stats_kernel(StatOps s) {
  __shared__ uint32_t red[12];
  if (s.o[0].clear && blockIdx.x == 0 && threadIdx.x < 2) s.o[0].clear[threadIdx.x] = 0u;
  const int nb3 = s.o[0].blocks + s.o[1].blocks + s.o[2].blocks;
  if ((int)blockIdx.x >= nb3) {  // (uniform) a pool's column maxima
    const int k = blockIdx.x - nb3;
    pool_colmax_block(s.pc.pcol, s.pc.nblk, s.pc.npool, s.pc.colblk, k % s.pcx, k / s.pcx);
    return;
  }
  int blk;
  const int w = pick_op(s, blockIdx.x, [](const StatOp &o) { return o.blocks; }, blk);
  const StatOp &o = s.o[w];  // (uniform)
  if (o.mode == 0) stats_rows(o, blk, red);
  else stats_cols(o, blk);
}

// The column maxima / minima over the partials (64 columns per block, 4
// groups of partials through LDS); the counts zeroed for stats_count_kernel.
__global__ __launch_bounds__(256) void stats_finalize_kernel(StatOps s) {
  __shared__ uint32_t red[2][4][64];
  __shared__ PoolCountSmem psm;
  const int nf3 = nfinal_blocks(s.o[0]) + nfinal_blocks(s.o[1]) + nfinal_blocks(s.o[2]);
  if ((int)blockIdx.x >= nf3) {  // (uniform) a pool's small elements, after its maxima
    pool_count_block(s.pc.P, s.pc.ps, s.pc.R, s.pc.npool, s.pc.vec, s.pc.rowblk, s.pc.colblk,
                     blockIdx.x - nf3, s.pcn, psm);
    return;
  }
  int blk;
  const StatOp &o = s.o[pick_op(s, blockIdx.x, [](const StatOp &q) { return nfinal_blocks(q); }, blk)];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blk * 64 + lane;
  uint32_t m = 0, n = 0xffffffffu;
  if (c < o.cols) {
    const uint32_t *pm = o.part + c, *pn = o.part + (size_t)o.rbk * o.cols + c;
    int q = grp;
    for (; q + 28 < o.rbk; q += 32) {  // eight maxima and eight minima in flight
      uint32_t a[8], b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = pm[(size_t)(q + 4 * j) * o.cols];
        b[j] = pn[(size_t)(q + 4 * j) * o.cols];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        m = max(m, a[j]);
        n = min(n, b[j]);
      }
    }
    for (; q < o.rbk; q += 4) {
      m = max(m, pm[(size_t)q * o.cols]);
      n = min(n, pn[(size_t)q * o.cols]);
    }
  }
  red[0][grp][lane] = m;
  red[1][grp][lane] = n;
  __syncthreads();
  m = max(max(red[0][0][lane], red[0][1][lane]), max(red[0][2][lane], red[0][3][lane]));
  n = min(min(red[1][0][lane], red[1][1][lane]), min(red[1][2][lane], red[1][3][lane]));
  if (grp == 0 && c < o.cols) {
    o.out[c] = m;
    o.out[o.cols + c] = n + 1u;
    o.out[2 * (size_t)o.cols + c] = 0;
  }
}

// The spread columns' counts (f16-split.h) after the finalize: block (cb,
// rc) takes 64 columns x a chunk of 64 rows, leaves at once unless one of
// its columns is spread (rare), and otherwise reads its rows' 64-column
// segments (one coalesced 256-B row piece per wave and row) and adds each
// spread column's count of small elements by an integer atomic (exact and
// order-independent).
constexpr int CNT_ROWS = 64;
__host__ __device__ inline int ncount_blocks(const StatOp &o) {
  return o.mode == 1 && o.blocks ? ((o.cols + 63) / 64) * ((o.rows + CNT_ROWS - 1) / CNT_ROWS) : 0;
}
__global__ __launch_bounds__(256) void stats_count_kernel(StatOps s) {
  int blk;
  const StatOp &o = s.o[pick_op(s, blockIdx.x, [](const StatOp &q) { return ncount_blocks(q); }, blk)];
  const int ncb = (o.cols + 63) / 64;
  const int cb = blk % ncb, rc = blk / ncb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = cb * 64 + lane;
  bool spr = false;
  float bound = 0.0f;
  if (c < o.cols) {
    const uint32_t mx = o.out[c];
    spr = kcnn::f16x3::spread(mx, o.out[o.cols + c]);
    if (spr) bound = kcnn::f16x3::small_bound(mx);
  }
  if (__ballot(spr) == 0) return;  // block-uniform (the same columns in every wave)
  const int r0 = rc * CNT_ROWS, r1 = min(o.rows, r0 + CNT_ROWS);
  uint32_t cnt = 0;
  if (spr) {  // the wave's CNT_ROWS / 4 rows loaded together
    float v[CNT_ROWS / 4];
#pragma unroll
    for (int i = 0; i < CNT_ROWS / 4; ++i) {
      const int r = r0 + wave + 4 * i;
      v[i] = r < r1 ? fabsf(X_row(o, r)[c]) : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < CNT_ROWS / 4; ++i) cnt += (v[i] < bound && v[i] != 0.0f) ? 1u : 0u;
  }
  if (cnt) atomicAdd(o.out + 2 * (size_t)o.cols + c, cnt);
}

// a statistics pass over X (rows x cols, pitch ld): mode 0 per row, 1 per
// column (partials at part, stat_part_words of them)
StatOp stat_op(const float *X, int rows, int cols, int ld, int mode, uint32_t *out,
               uint32_t *part) {
  StatOp o{};
  o.X = X; o.out = out; o.part = part;
  o.rows = rows; o.cols = cols; o.ld = ld; o.mode = mode;
  o.vec = ld % 4 == 0 && (uintptr_t)X % 16 == 0;
  if (rows <= 0 || cols <= 0) return o;  // blocks 0
  if (mode == 0) {
    o.rpb = cols >= 2048 ? 1 : 4;
    o.blocks = (rows + o.rpb - 1) / o.rpb;
  } else {
    o.cb = (cols + 1023) / 1024;
    // about 1024 blocks of at least 16 rows, at most 256 row chunks
    o.rbk = std::max(1, std::min(256, std::min((rows + 15) / 16, (1024 + o.cb - 1) / o.cb)));
    o.rb = (rows + o.rbk - 1) / o.rbk;
    o.rbk = (rows + o.rb - 1) / o.rb;
    o.blocks = o.cb * o.rbk;
    o.fblocks = (cols + 63) / 64;
  }
  return o;
}
size_t stat_part_words(int rows, int cols, int mode) {
  if (mode == 0) return 0;
  const StatOp o = stat_op(nullptr, rows, cols, cols, 1, nullptr, nullptr);
  return 2 * (size_t)o.rbk * cols;
}
int stats_launch3(const StatOps &ops, hipStream_t st) {
  // empty operands: maxima 0 (no scale), minima 0 (no nonzero element)
  for (const StatOp &o : ops.o)
    if (o.blocks == 0 && o.out) {
      const size_t n = o.mode == 0 ? (size_t)std::max(o.rows, 0) : (size_t)std::max(o.cols, 0);
      if (n && hipMemsetAsync(o.out, 0, 3 * n * 4, st) != hipSuccess) return (int)hipGetLastError();
    }
  int nb = 0, nf = 0, nc = 0;
  for (const StatOp &o : ops.o) {
    nb += o.blocks;
    nf += nfinal_blocks(o);
    nc += ncount_blocks(o);
  }
  nb += ops.pcx * ops.pcy;
  nf += ops.pcn;
  if (nb == 0) return 0;
  hipLaunchKernelGGL(stats_kernel, dim3(nb), dim3(256), 0, st, ops);
  int rc = kcnn::launch_status();
  if (rc || nf == 0) return rc;
  hipLaunchKernelGGL(stats_finalize_kernel, dim3(nf), dim3(256), 0, st, ops);
  rc = kcnn::launch_status();
  if (rc || nc == 0) return rc;
  hipLaunchKernelGGL(stats_count_kernel, dim3(nc), dim3(256), 0, st, ops);
  return kcnn::launch_status();
}
int stats_launch(const StatOp &a, const StatOp &b, hipStream_t st) {
  StatOps ops{};
  ops.o[0] = a;
  ops.o[1] = b;
  ops.o[2] = StatOp{};
  return stats_launch3(ops, st);
}

// C = alpha * sum_s part[s] + beta * C, the splits added in increasing s
// (slab rows padded to np4 = N rounded up to 4: 16-B reads; a quad's columns
// past N are not stored); elements of an Inf / NaN row or column are the
// epilogue's (split 0).  The spread check of tile_epilogue on the summed
// value (unscaled: the threshold times 2^-(s_row + s_col)); a rejected
// element is not stored.  A wave with at most REJ_LOCAL of them recomputes
// them itself (wave_dot); one with more flags its 64 quads (rflag) for
// gemm_f16x3_fixup_kernel, which spreads such groups over the whole GPU: a
// spread row rejects hundreds of elements of one row, and one wave's
// wave_dots in series took milliseconds (nnet.config's weight gradients).
constexpr int REJ_LOCAL = 4;
__device__ __forceinline__ uint32_t reduce_quad(const GemmF16Args &p, int64_t e, int nq, int np4,
                                                int64_t plane, int &r, int &c, bool store) {
  const int N = p.N;
  r = (int)(e / nq);
  c = (int)(e - (int64_t)r * nq) * 4;
  // every load of the quad issued before the first test: the slabs, the
  // row's statistics and the four columns' (one 16-B load each when the
  // blocks allow; a column past N reads as non-finite, i.e. not stored)
  const float *q = p.part + (int64_t)r * np4 + c;
  float4 v = *reinterpret_cast<const float4 *>(q);
  float4 w = p.ksplit > 1 ? *reinterpret_cast<const float4 *>(q + plane) : v;
  const uint32_t ar = p.amax[r], cr = p.acnt[r];
  uint32_t bm[4], cc[4];
  if (p.bvec) {
    const uint4 x = *reinterpret_cast<const uint4 *>(p.bmax + c);
    const uint4 y = *reinterpret_cast<const uint4 *>(p.bcnt + c);
    bm[0] = x.x; bm[1] = x.y; bm[2] = x.z; bm[3] = x.w;
    cc[0] = y.x; cc[1] = y.y; cc[2] = y.z; cc[3] = y.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bm[i] = c + i < N ? p.bmax[c + i] : NONFINITE;
      cc[i] = c + i < N ? p.bcnt[c + i] : 0u;
    }
  }
  // the bias quad too, and the momentum update's W and prev quads (the 16-B
  // paths' operands, loaded here, not after the tests: one memory round trip
  // per quad instead of two; host: the update's rows 16-B aligned)
  float4 w4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), q4 = w4;
  float4 *wp = nullptr, *qp = nullptr;
  if (p.mom.W && store) {
    wp = reinterpret_cast<float4 *>(p.mom.W + (int64_t)r * p.mom.ldw + c);
    qp = reinterpret_cast<float4 *>(p.mom.prev + (int64_t)r * p.mom.ldp + c);
    if (c + 4 <= N) {
      w4 = *wp;
      q4 = *qp;
    }
  }
  float bv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (p.bias && store) {
    if (c + 4 <= N && ((uintptr_t)p.bias & 15) == 0) {
      const float4 b4 = *reinterpret_cast<const float4 *>(p.bias + c);
      bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = c + i < N ? p.bias[c + i] : 0.0f;
    }
  }
  if (p.ksplit > 1) {
    v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    for (int k = 2; k < p.ksplit; ++k) {
      w = *reinterpret_cast<const float4 *>(q + k * plane);
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
  }
  if (ar >= NONFINITE) return 0;
  const float sv[4] = {v.x, v.y, v.z, v.w};
#ifdef KCNN_EXPERIMENTS  // A/B: KCNN_RED_DEBUG & 1 drops the spread check
  const bool any = !(p.dbg & 1) && (cr | cc[0] | cc[1] | cc[2] | cc[3]) != 0 && ar != 0;
#else
  // the counts are 0 unless a group is spread, so one test skips the check
  // (an all-zero row: its products are exactly 0, no check)
  const bool any = (cr | cc[0] | cc[1] | cc[2] | cc[3]) != 0 && ar != 0;
#endif
  float *o = p.C + (int64_t)r * p.ldc + c;
  const bool fin = max(max(bm[0], bm[1]), max(bm[2], bm[3])) < NONFINITE;
  if (p.mom.W && !any && fin) {  // the fused momentum update, 16-B (host: aligned)
    if (store) {
      const MomentumEpi &m = p.mom;
      kcnn::momentum_step(p.alpha * sv[0], q4.x, w4.x, m.momentum, m.a_wd, m.a_g);
      kcnn::momentum_step(p.alpha * sv[1], q4.y, w4.y, m.momentum, m.a_wd, m.a_g);
      kcnn::momentum_step(p.alpha * sv[2], q4.z, w4.z, m.momentum, m.a_wd, m.a_g);
      kcnn::momentum_step(p.alpha * sv[3], q4.w, w4.w, m.momentum, m.a_wd, m.a_g);
      *qp = q4;
      *wp = w4;
    }
    return 0;
  }
  if (!p.mom.W && !any && fin && ((p.ldc & 3) | ((uintptr_t)p.C & 15)) == 0) {
    if (store) {  // one 16-B store (the same values)
      float4 ov = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (p.beta != 0.0f) ov = *reinterpret_cast<const float4 *>(o);
      const float oi[4] = {ov.x, ov.y, ov.z, ov.w};
      float wv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wv[i] = p.beta == 0.0f ? p.alpha * sv[i] : p.alpha * sv[i] + p.beta * oi[i];
        if (p.bias) wv[i] += bv[i];
      }
      *reinterpret_cast<float4 *>(o) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    }
    return 0;
  }
  // the check's thresholds (0: no check) of the four columns
  float thr[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (any) {
    const int er = scale_exp(ar);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // (an all-zero column: exact, no check)
      if (bm[i] >= NONFINITE || bm[i] == 0 || (cr | cc[i]) == 0) continue;
      thr[i] = __builtin_amdgcn_ldexpf(
          kcnn::f16x3::spread_weight(cr) + kcnn::f16x3::spread_weight(cc[i]),
          -(er + scale_exp(bm[i])));
    }
  }
  uint32_t rej = 0;  // bit i: column c + i is rejected
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (bm[i] >= NONFINITE) continue;  // (and columns past N)
    if (thr[i] != 0.0f && !(fabsf(sv[i]) >= thr[i])) {
      rej |= 1u << i;
      continue;
    }
    if (store) emit(p, r, c + i, sv[i]);
  }
  return rej;
}

__global__ __launch_bounds__(256) void gemm_f16x3_reduce_kernel(GemmF16Args p, int a_kc,
                                                                int b_kc) {
  const int np4 = (p.N + 3) & ~3, nq = np4 >> 2;
  const int64_t total = (int64_t)p.M * nq;
  const int64_t plane = (int64_t)p.M * np4;
  const int lane = threadIdx.x & 63;
  // e0 = the wave's first quad, a multiple of 64 below total: lane 0 is
  // active in every pass, and every group of 64 quads gets its flag written
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    // (a whole tile's quads were stored by its workgroup: no slabs, no rejections)
    int r = (int)(e / nq), c = (int)(e - (int64_t)r * nq) * 4;
    const uint32_t rej = in_split_tile(p, r, c) ? reduce_quad(p, e, nq, np4, plane, r, c, true) : 0u;
    // the wave's rejections (ballots: only the active lanes)
    const int n = __builtin_popcountll(__ballot(rej & 1)) + __builtin_popcountll(__ballot(rej & 2)) +
                  __builtin_popcountll(__ballot(rej & 4)) + __builtin_popcountll(__ballot(rej & 8));
    const bool defer = n > REJ_LOCAL && !p.fix_local;
    if (lane == 0) {
      p.rflag[e >> 6] = defer ? 1u : 0u;
      if (defer) p.rflag[(total + 63) >> 6] = p.gen;
      if (n > REJ_LOCAL && p.fix_report) *p.fix_report = 1u;
    }
    if (n == 0 || defer) continue;
    fix_rejected(p, a_kc != 0, b_kc != 0, rej, lane, [&](int l, int bit, int &row, int &col) {
      row = __builtin_amdgcn_readlane(r, l);
      col = __builtin_amdgcn_readlane(c, l) + bit;
    });
  }
}

// The flagged groups of 64 quads (gemm_f16x3_reduce_kernel), one per block
// at a time: slot s = t G + b for thread t of block b (G blocks), so the
// consecutive groups of one spread row go to different blocks.  A group's
// rejections are found again (reduce_quad, not stored) and recomputed in fp32:
//  - op(B) row-contiguous with 16-B rows (`rows`): every lane its quad's four sums, the
//    block's four waves each over a quarter of K (16-B loads of op(B)'s rows,
//    coalesced over the lanes; the lanes of one C row share op(A)'s element),
//    the quarters added in wave order, the rejected elements stored;
//  - otherwise: wave_dot per rejected element, the quads dealt to
//    the waves by lane & 3.
// Deterministic: the group's results do not depend on the block or order.
constexpr int FIX_DEPTH = 16;
// the fixup's grid: a flagged call's groups take the workgroups in turn
// (c2's weight-gradient shape with 32 spread rows, 1452 groups: +925 us at
// 128 workgroups, measured r05 by a one-off driver); an unflagged call exits at the
// first load, and the launch costs the same 4.4 us at 128 or 1024
constexpr int FIX_GRID = 1024;
__global__ __launch_bounds__(256) void gemm_f16x3_fixup_kernel(GemmF16Args p, int a_kc,
                                                               int b_kc, int rows) {
  __shared__ int list[256];
  __shared__ int nlist;
  __shared__ float4 quarter[4][64];
  const int np4 = (p.N + 3) & ~3, nq = np4 >> 2;
  const int64_t total = (int64_t)p.M * nq;
  const int64_t plane = (int64_t)p.M * np4;
  const int64_t nslots = (total + 63) >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // nothing flagged in this call (the word is another call's number, or
  // anything the workspace held: a stale match only costs the scan below)
  if (p.rflag[nslots] != p.gen) return;
  for (int64_t base = 0; base < nslots; base += (int64_t)gridDim.x * blockDim.x) {
    if (threadIdx.x == 0) nlist = 0;
    __syncthreads();
    const int64_t slot = base + (int64_t)threadIdx.x * gridDim.x + blockIdx.x;
    if (slot < nslots && p.rflag[slot] != 0) list[atomicAdd(&nlist, 1)] = (int)threadIdx.x;
    __syncthreads();
    const int n = nlist;
    for (int j = 0; j < n; ++j) {
      const int64_t e0 = (base + (int64_t)list[j] * gridDim.x + blockIdx.x) << 6;
      const int64_t e = e0 + lane;
      // (past C: row and column 0, whose loads below stay in bounds)
      int r = e < total ? (int)(e / nq) : 0;
      int c = e < total ? (int)(e - (int64_t)r * nq) * 4 : 0;
      const bool valid = e < total && in_split_tile(p, r, c);
      const uint32_t rej = valid ? reduce_quad(p, e, nq, np4, plane, r, c, false) : 0u;
      if (!rows) {
        const uint64_t mine = (lane & 3) == wave ? rej : 0u;
        fix_rejected(p, a_kc != 0, b_kc != 0, mine, lane, [&](int l, int bit, int &row, int &col) {
          row = __builtin_amdgcn_readlane(r, l);
          col = __builtin_amdgcn_readlane(c, l) + bit;
        });
        __syncthreads();
        continue;
      }
      // this wave's quarter of K for the lane's quad (r, c .. c + 3)
      const int kq = (p.K + 3) >> 2;
      const int k0 = wave * kq, k1 = min(p.K, k0 + kq);
      const int64_t sa = a_kc ? 1 : p.lda;
      const float *qa = a_kc ? p.A + (int64_t)r * p.lda + k0 : p.A + (int64_t)k0 * p.lda + r;
      const float *qb = p.B + (int64_t)k0 * p.ldb + c;
      float4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      int k = k0;
#pragma unroll 1
      for (; k + FIX_DEPTH <= k1; k += FIX_DEPTH) {
        float x[FIX_DEPTH];
        float4 y[FIX_DEPTH];
#pragma unroll
        for (int i = 0; i < FIX_DEPTH; ++i) {
          x[i] = qa[i * sa];
          y[i] = *reinterpret_cast<const float4 *>(qb + (int64_t)i * p.ldb);
        }
#pragma unroll
        for (int i = 0; i < FIX_DEPTH; ++i) {
          float4 &t = acc[i & 3];
          t.x = fmaf(x[i], y[i].x, t.x);
          t.y = fmaf(x[i], y[i].y, t.y);
          t.z = fmaf(x[i], y[i].z, t.z);
          t.w = fmaf(x[i], y[i].w, t.w);
        }
        qa += FIX_DEPTH * sa;
        qb += (int64_t)FIX_DEPTH * p.ldb;
      }
#pragma unroll 1
      for (; k < k1; ++k) {
        const float x = *qa;
        const float4 y = *reinterpret_cast<const float4 *>(qb);
        acc[0].x = fmaf(x, y.x, acc[0].x);
        acc[0].y = fmaf(x, y.y, acc[0].y);
        acc[0].z = fmaf(x, y.z, acc[0].z);
        acc[0].w = fmaf(x, y.w, acc[0].w);
        qa += sa;
        qb += p.ldb;
      }
      float4 q;
      q.x = (acc[0].x + acc[1].x) + (acc[2].x + acc[3].x);
      q.y = (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y);
      q.z = (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z);
      q.w = (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w);
      quarter[wave][lane] = q;
      __syncthreads();
      if (wave == 0 && rej) {
        const float4 q0 = quarter[0][lane], q1 = quarter[1][lane], q2 = quarter[2][lane],
                     q3 = quarter[3][lane];
        const float v[4] = {((q0.x + q1.x) + q2.x) + q3.x, ((q0.y + q1.y) + q2.y) + q3.y,
                            ((q0.z + q1.z) + q2.z) + q3.z, ((q0.w + q1.w) + q2.w) + q3.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rej >> i & 1) emit(p, r, c + i, v[i]);
      }
      __syncthreads();
    }
    __syncthreads();
  }
}

// The split-K count (and the whole tiles in front of the split ones,
// block_tile) of least modelled time: the whole tiles in nwhole / 256 rounds
// of one workgroup per CU, the split ones in ceil((tiles - nwhole) s / 256)
// rounds, a round of k steps 0.0458 k + 11.1 us (the tile prologue and
// epilogue; fitted to c2's three FC GEMMs on MI355X), and for s > 1 the
// reduce's (s + 1) fp32 reads and writes of the split tiles' share of M N
// at 4 TB/s.  (The reduce was unpriced before r06: nnet.config's 4096 x 3454
// x 4096 layers took 4 splits and an 86-92 us reduce, one split being 2.4 %
// faster per step; c2's 364-tile weight gradient split all its tiles in 2.84
// rounds, where 256 whole tiles and 108 split ones take 1 + 0.84.)
int choose_ksplit(int64_t tiles, int M, int N, int K, int *nwhole = nullptr) {
  auto round = [](int k) { return 0.0458 * k + 11.1; };
  int best = 1, best_w = 0;
  double best_t = (double)((tiles + 255) / 256) * round(K);
  for (int s = 2; s <= 4 && K / s >= 1024; ++s) {
    const int ks = (K + s - 1) / s;
    for (int64_t w = 0; w < tiles; w += 256) {
      const int64_t rest = tiles - w;
      const double t = (double)(w / 256) * round(K) + (double)((rest * s + 255) / 256) * round(ks) +
                       (double)(s + 1) * M * N * 4.0 / 4.0e6 * (double)rest / (double)tiles;
      if (t < best_t) { best_t = t; best = s; best_w = (int)w; }
    }
  }
  if (nwhole) *nwhole = best > 1 ? best_w : 0;
  return best;
}

// KCNN_F16X3_FAST (experiment build): 1 (default) the one-barrier fast
// kernel where no operand is LR, 0 the two-phase kernel (bitwise the same C)
template <int AM, int BMODE, bool RAG>
void launch_t(const GemmF16Args &a, unsigned blocks, hipStream_t st) {
  static const int fast = KCNN_KNOB("KCNN_F16X3_FAST", 1);
  static bool attr = [] {
    return hipFuncSetAttribute(
               reinterpret_cast<const void *>(&gemm_f16x3_kernel<AM, BMODE, RAG>),
               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  }();
  (void)attr;
  // (an LR operand's 16 loaded values per thread and K step spill there)
  if constexpr (AM != LR && BMODE != LR) {
    static bool fattr = [] {
      return hipFuncSetAttribute(
                 reinterpret_cast<const void *>(&gemm_f16x3_fast_kernel<AM, BMODE, RAG>),
                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
    }();
    (void)fattr;
    if (fast) {
      hipLaunchKernelGGL((gemm_f16x3_fast_kernel<AM, BMODE, RAG>), dim3(blocks), dim3(NT),
                         LDS_BYTES, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_f16x3_kernel<AM, BMODE, RAG>), dim3(blocks), dim3(NT), LDS_BYTES, st,
                     a);
}
template <bool RAG>
void launch_r(int am, int bm, const GemmF16Args &a, unsigned blocks, hipStream_t st) {
  // am: LK or a row-contiguous mode; bm likewise
  if (am == LK && bm == LK) launch_t<LK, LK, RAG>(a, blocks, st);
  else if (am == LK && bm == LT) launch_t<LK, LT, RAG>(a, blocks, st);
  else if (am == LK) launch_t<LK, LR, RAG>(a, blocks, st);
  else if (am == LT && bm == LK) launch_t<LT, LK, RAG>(a, blocks, st);
  else if (am == LT && bm == LT) launch_t<LT, LT, RAG>(a, blocks, st);
  else if (am == LT) launch_t<LT, LR, RAG>(a, blocks, st);
  else if (bm == LK) launch_t<LR, LK, RAG>(a, blocks, st);
  else if (bm == LT) launch_t<LR, LT, RAG>(a, blocks, st);
  else launch_t<LR, LR, RAG>(a, blocks, st);
}
void launch(int am, int bm, const GemmF16Args &a, unsigned blocks, hipStream_t st) {
  if (a.K % BK) launch_r<true>(am, bm, a, blocks, st);
  else launch_r<false>(am, bm, a, blocks, st);
}

size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }
// the split-K workspace: the slabs, then the reduce's flags (one word per
// 64 quads of C)
size_t slab_bytes(int s, int M, int N) {
  return align16(sizeof(float) * (size_t)s * M * ((N + 3) & ~3));
}
size_t flag_bytes(int M, int N) {
  return align16(sizeof(uint32_t) * (((size_t)M * ((N + 3) / 4) + 63) / 64 + 1));
}
size_t partial_bytes(int M, int N, int K) {
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int s = choose_ksplit(tiles, M, N, K);
  return s > 1 ? slab_bytes(s, M, N) + flag_bytes(M, N) : 0;
}

}  // namespace

extern "C" int kl_absmax_rows(const float *X, int rows, int cols, int ld, uint32_t *rmax,
                              kcnn_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols || !rmax) return (int)hipErrorInvalidValue;
  return stats_launch(stat_op(X, rows, cols, ld, 0, rmax, nullptr), StatOp{},
                      kcnn::as_stream(stream));
}
extern "C" size_t kl_absmax_cols_words(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return stat_part_words(rows, cols, 1);
}
extern "C" int kl_absmax_cols(const float *X, int rows, int cols, int ld, uint32_t *cmax,
                              uint32_t *part, kcnn_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols || !cmax) return (int)hipErrorInvalidValue;
  if (rows > 0 && cols > 0 && !part) return (int)hipErrorInvalidValue;
  return stats_launch(stat_op(X, rows, cols, ld, 1, cmax, part), StatOp{},
                      kcnn::as_stream(stream));
}

// kl_absmax_rows of R (rows x cols, pitch ld) and kl_absmax_cols of Q
// (qrows x qcols, pitch ldq; part: kl_absmax_cols_words) in one statistics
// launch (and Q's finalize / count passes): the f16x3 implicit GEMM's frame
// and filter statistics (cnsl-conv-igemm-x6.hip); clear (nullable): two
// words set to 0 by the same launch (that kernel's list counters)
extern "C" int kl_absmax_rows_cols(const float *R, int rows, int cols, int ld, uint32_t *rmax,
                                   const float *Q, int qrows, int qcols, int ldq, uint32_t *cmax,
                                   uint32_t *part, uint32_t *clear, kcnn_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols || !rmax || qrows < 0 || qcols < 0 || ldq < qcols ||
      !cmax)
    return (int)hipErrorInvalidValue;
  if (qrows > 0 && qcols > 0 && !part) return (int)hipErrorInvalidValue;
  StatOp q = stat_op(Q, qrows, qcols, ldq, 1, cmax, part);
  q.clear = clear;
  const StatOp r = stat_op(R, rows, cols, ld, 0, rmax, nullptr);
  if (clear && q.blocks + r.blocks == 0) {  // no statistics launch to clear it
    const hipError_t e = hipMemsetAsync(clear, 0, 8, kcnn::as_stream(stream));
    if (e != hipSuccess) return (int)e;
  }
  return stats_launch(q, r, kcnn::as_stream(stream));
}

// Up to three statistics passes in one set of launches (stats, finalize,
// count): op i over X_i (rows_i x cols_i, pitch ld_i), per row (mode_i 0)
// or per column (1, part_i: kl_absmax_cols_words of scratch) into the block
// out_i; X_i NULL skips op i.  The FC backward's output derivative (rows for
// the data gradient, columns for the weight gradient) and weight columns in
// one pass set instead of two (AffineComponent::Backprop).
extern "C" int kl_gemm_stats3(const float *X0, int rows0, int cols0, int ld0, int mode0,
                              uint32_t *out0, uint32_t *part0, const float *X1, int rows1,
                              int cols1, int ld1, int mode1, uint32_t *out1, uint32_t *part1,
                              const float *X2, int rows2, int cols2, int ld2, int mode2,
                              uint32_t *out2, uint32_t *part2, void *pool_cols,
                              kcnn_stream_t stream) {
  StatOps ops{};
  if (pool_cols) {  // the pool's column kernels' grids (cnsl-conv-frame.hip kcnn_pool_cols_complete)
    ops.pc = *static_cast<const PoolColDeferred *>(pool_cols);
    const int ncq = ops.pc.npool % 4 == 0 ? ops.pc.npool / 4 : ops.pc.npool;
    ops.pcx = (ncq + 255) / 256;
    ops.pcy = (ops.pc.nblk + COLMAX_ROWS - 1) / COLMAX_ROWS;
    ops.pcn = std::min(ops.pc.R, 256);
  }
  const float *X[3] = {X0, X1, X2};
  const int rows[3] = {rows0, rows1, rows2}, cols[3] = {cols0, cols1, cols2};
  const int ld[3] = {ld0, ld1, ld2}, mode[3] = {mode0, mode1, mode2};
  uint32_t *out[3] = {out0, out1, out2}, *part[3] = {part0, part1, part2};
  for (int i = 0; i < 3; ++i) {
    ops.o[i] = StatOp{};
    if (!X[i]) continue;
    if (rows[i] < 0 || cols[i] < 0 || ld[i] < cols[i] || !out[i] || (mode[i] != 0 && mode[i] != 1) ||
        (mode[i] == 1 && rows[i] > 0 && cols[i] > 0 && !part[i]))
      return (int)hipErrorInvalidValue;
    ops.o[i] = stat_op(X[i], rows[i], cols[i], ld[i], mode[i], out[i], mode[i] ? part[i] : nullptr);
  }
  return stats_launch3(ops, kcnn::as_stream(stream));
}

// C[M x N] = alpha * op(A) op(B) + beta * C with the operands' max |x| given:
// amax[i] for row i of op(A), bmax[j] for column j of op(B) (bit patterns of
// max |x|, kl_absmax_rows / kl_absmax_cols).  Needs 16-B aligned
// K-contiguous operands (A untransposed, B transposed) with pitches % 4 == 0
// and every workgroup's buffer offsets below 2^31; returns
// hipErrorNotSupported otherwise (the caller uses kl_gemm_x6).
extern "C" size_t kl_gemm_f16x3_workspace_bytes(int M, int N, int K) {
  return partial_bytes(M, N, K);
}
// The fix-up launch of a split-K call (an exit-at-once kernel of 4.4 us in
// all but the rare calls with a spread group, FIX_GRID) is skipped for a call
// site (shape, transposes, momentum or not) whose previous call deferred no
// group: the site's word in host memory, cleared by the host at each launch
// and set by the reduce when a group would have been deferred, is read at
// the next launch.  A skipped call's reduce recomputes every rejection itself
// (fix_local), so a stale or wrong guess costs time, never a result.  Up to
// FIX_SITES sites; the others always launch the fix-up.
constexpr int FIX_SITES = 256;
struct FixSites {
  std::mutex mu;
  uint32_t *flags = nullptr;  // pinned host words (1: the fix-up was needed or is unknown)
  uint32_t *dflags = nullptr; // the same words' device address
  int64_t key[FIX_SITES][6];
  int n = 0;
  bool failed = false;
};
// the word of this site, nullptr when there is none (table full, no host memory)
static uint32_t *fix_site(int M, int N, int K, int ta, int tb, int mom, uint32_t **dev) {
  static FixSites fs;
  std::lock_guard<std::mutex> lk(fs.mu);
  if (!fs.flags && !fs.failed) {
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, FIX_SITES * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) ==
            hipSuccess &&
        hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
      fs.flags = static_cast<uint32_t *>(h);
      fs.dflags = static_cast<uint32_t *>(d);
    } else {
      (void)hipGetLastError();
      fs.failed = true;
    }
  }
  if (!fs.flags) return nullptr;
  const int64_t k[6] = {M, N, K, ta, tb, mom};
  int i = 0;
  for (; i < fs.n; ++i)
    if (std::equal(k, k + 6, fs.key[i])) break;
  if (i == fs.n) {
    if (fs.n == FIX_SITES) return nullptr;
    std::copy(k, k + 6, fs.key[fs.n++]);
    __atomic_store_n(fs.flags + i, 1u, __ATOMIC_RELAXED);
  }
  *dev = fs.dflags + i;
  return fs.flags + i;
}

static int gemm_f16x3_st(int transA, int transB, int M, int N, int K, float alpha,
                         const float *A, int lda, const float *B, int ldb, float beta, float *C,
                         int ldc, const uint32_t *amax, const uint32_t *bmax, const float *bias,
                         void *ws, size_t ws_bytes, kcnn_stream_t stream,
                         const MomentumEpi *mom = nullptr) {
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0 || K == 0) return (int)hipErrorNotSupported;
  const bool a_kc = !transA, b_kc = transB != 0;
  if ((a_kc && (lda % 4 || (uintptr_t)A % 16)) || (b_kc && (ldb % 4 || (uintptr_t)B % 16)))
    return (int)hipErrorNotSupported;
  hipStream_t st = kcnn::as_stream(stream);
  GemmF16Args a{};
  a.A = A; a.B = B; a.C = C; a.amax = amax; a.bmax = bmax; a.bias = bias;
  if (mom) a.mom = *mom;
  // statistics blocks [max[n], min[n], cnt[n]] (stats_rows, stats_finalize_kernel)
  a.amin = amax + M;
  a.acnt = amax + 2 * (size_t)M;
  a.bmin = bmax + N;
  a.bcnt = bmax + 2 * (size_t)N;
  a.bvec = N % 4 == 0 && (uintptr_t)a.bmax % 16 == 0 && (uintptr_t)a.bcnt % 16 == 0;
  static const int red_dbg = KCNN_KNOB("KCNN_RED_DEBUG", 0);
  static const int gemm_dbg = KCNN_KNOB("KCNN_GEMM_DEBUG", 0);
  a.dbg = red_dbg | gemm_dbg << 4;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.alpha = alpha; a.beta = beta;
  a.tiles_m = (M + BM - 1) / BM;
  a.tiles_n = (N + BN - 1) / BN;
  const int64_t tiles = (int64_t)a.tiles_m * a.tiles_n;
  int nwhole = 0;
  int s = choose_ksplit(tiles, M, N, K, &nwhole);
#ifdef KCNN_EXPERIMENTS  // A/B: KCNN_F16X3_KSPLIT forces the split count (0: chosen), no whole tiles;
                         // KCNN_F16X3_NOWHOLE keeps the chosen count without whole tiles
  static const int ks_force = KCNN_KNOB("KCNN_F16X3_KSPLIT", 0);
  static const int no_whole = KCNN_KNOB("KCNN_F16X3_NOWHOLE", 0);
  if (ks_force > 0) s = std::min(ks_force, 4);
  if (ks_force > 0 || no_whole) nwhole = 0;
#endif
  const size_t need = s > 1 ? slab_bytes(s, M, N) + flag_bytes(M, N) : 0;
  if (need > ws_bytes || !ws) s = 1;
  if (s > 1) {
    a.part = static_cast<float *>(ws);
    a.rflag = reinterpret_cast<uint32_t *>(static_cast<char *>(ws) + slab_bytes(s, M, N));
    static std::atomic<uint32_t> calls{0};
    a.gen = ++calls;
    if (a.gen == 0) a.gen = ++calls;
  }
  a.ksplit = s;
  a.kps = ((K + s - 1) / s + BK - 1) / BK * BK;
  // every offset a workgroup forms (rows of its tile, k up to its K span +
  // 2 BK) < 2^31
  auto fits = [&](bool kc, int ld, int R, int span) {
    if (kc) return (int64_t)R * ld * 4 + (int64_t)(K + 2 * BK) * 4 < ((int64_t)1 << 31);
    return (int64_t)(span + 2 * BK) * ld * 4 + (int64_t)R * 4 < ((int64_t)1 << 31);
  };
  if (!fits(a_kc, lda, BM, a.kps) || !fits(b_kc, ldb, BN, a.kps)) return (int)hipErrorNotSupported;
  if (s == 1 || !fits(a_kc, lda, BM, K) || !fits(b_kc, ldb, BN, K)) nwhole = 0;
  a.nwhole = nwhole;
  const int64_t nb = nwhole + (tiles - nwhole) * s;
  if (nb >= ((int64_t)1 << 31)) return (int)hipErrorNotSupported;
  // a row-contiguous operand takes 16-B loads along its rows when they are
  // aligned (pitch % 4 == 0: a quad that starts inside the row count M or N
  // ends inside the pitch; its values past the count feed only C rows or
  // columns that are not stored, and the descriptors above end at the last
  // row's padded quad)
  auto mode = [](bool kc, const float *ptr, int ld) {
    if (kc) return (int)LK;
    static const int tr = KCNN_KNOB("KCNN_F16X3_TR", 1);
    return tr && ld % 4 == 0 && (uintptr_t)ptr % 16 == 0 ? (int)LT : (int)LR;
  };
  bool fix_launch = true;
  if (s > 1) {
    uint32_t *dev = nullptr;
    uint32_t *site = fix_site(M, N, K, transA != 0, transB != 0, a.mom.W != nullptr, &dev);
    if (site) {
      fix_launch = __atomic_load_n(site, __ATOMIC_RELAXED) != 0;
      __atomic_store_n(site, 0u, __ATOMIC_RELAXED);
      a.fix_report = dev;
      a.fix_local = fix_launch ? 0 : 1;
    }
  }
  launch(mode(a_kc, A, lda), mode(b_kc, B, ldb), a, (unsigned)nb, st);
  int rc = kcnn::launch_status();
  if (rc || s == 1) return rc;
  hipLaunchKernelGGL(gemm_f16x3_reduce_kernel, dim3(kcnn::grid_for((int64_t)M * ((N + 3) / 4))),
                     dim3(256), 0, st, a, a_kc ? 1 : 0, b_kc ? 1 : 0);
  rc = kcnn::launch_status();
  if (rc || !fix_launch) return rc;
  // op(B) row-contiguous: the fixup's 16-B loads along its rows
  const int rows = !b_kc && ldb % 4 == 0 && (uintptr_t)B % 16 == 0 && N % 4 == 0;
  const int64_t slots = ((int64_t)M * ((N + 3) / 4) + 63) / 64;
  hipLaunchKernelGGL(gemm_f16x3_fixup_kernel,
                     dim3((unsigned)std::min<int64_t>(FIX_GRID, (slots + 15) / 16)), dim3(256), 0, st,
                     a, a_kc ? 1 : 0, b_kc ? 1 : 0, rows);
  return kcnn::launch_status();
}
extern "C" int kl_gemm_f16x3_st(int transA, int transB, int M, int N, int K, float alpha,
                                const float *A, int lda, const float *B, int ldb, float beta,
                                float *C, int ldc, const uint32_t *amax, const uint32_t *bmax,
                                void *ws, size_t ws_bytes, kcnn_stream_t stream) {
  return gemm_f16x3_st(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, amax, bmax,
                       nullptr, ws, ws_bytes, stream);
}

// The same with the operand statistics computed here (op(A)'s rows: A's rows,
// or its columns when transposed; op(B)'s columns: B's columns, or its rows
// when transposed), one launch for both (two with a per-column one), into
// the workspace after the partial slabs.
namespace {
size_t stats_ws_words(int M, int N, int K, int transA, int transB) {
  const size_t pa = transA ? stat_part_words(K, M, 1) : 0;
  const size_t pb = transB ? 0 : stat_part_words(K, N, 1);
  return 3 * ((size_t)M + N) + 4 + pa + pb;
}
}  // namespace
extern "C" size_t kl_gemm_f16x3_full_workspace_bytes(int M, int N, int K) {
  size_t w = 0;
  for (int ta = 0; ta < 2; ++ta)
    for (int tb = 0; tb < 2; ++tb) w = std::max(w, stats_ws_words(M, N, K, ta, tb));
  return partial_bytes(M, N, K) + align16(sizeof(uint32_t) * w);
}
extern "C" int kl_gemm_f16x3(int transA, int transB, int M, int N, int K, float alpha,
                             const float *A, int lda, const float *B, int ldb, float beta,
                             float *C, int ldc, void *ws, size_t ws_bytes,
                             kcnn_stream_t stream) {
  return kl_gemm_f16x3_given(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc,
                             nullptr, nullptr, ws, ws_bytes, stream);
}
// ... with either operand's statistics supplied by its producer (nullable):
// only the missing ones are computed (one read of that operand)
extern "C" int kl_gemm_f16x3_given(int transA, int transB, int M, int N, int K, float alpha,
                                   const float *A, int lda, const float *B, int ldb, float beta,
                                   float *C, int ldc, const uint32_t *amax_given,
                                   const uint32_t *bmax_given, void *ws, size_t ws_bytes,
                                   kcnn_stream_t stream) {
  return kl_gemm_f16x3_bias(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc,
                            amax_given, bmax_given, nullptr, ws, ws_bytes, stream);
}
// ... and C += bias[col] on every row (bias nullable), in the same store: the
// FC forward's out = bias; out += in W^T without the bias copy or C's re-read
static int gemm_f16x3_full(int transA, int transB, int M, int N, int K, float alpha,
                           const float *A, int lda, const float *B, int ldb, float beta,
                           float *C, int ldc, const uint32_t *amax_given,
                           const uint32_t *bmax_given, const float *bias, void *ws,
                           size_t ws_bytes, kcnn_stream_t stream, const MomentumEpi *mom) {
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0 || K == 0) return (int)hipErrorNotSupported;
  const size_t pb = partial_bytes(M, N, K);
  if (!ws || ws_bytes < kl_gemm_f16x3_full_workspace_bytes(M, N, K))
    return (int)hipErrorInvalidValue;
  uint32_t *amax = reinterpret_cast<uint32_t *>(static_cast<char *>(ws) + pb);
  uint32_t *bmax = amax + 3 * (size_t)M;  // statistics blocks: [max, min, cnt] per group
  uint32_t *parta = bmax + 3 * (size_t)N + 4;
  uint32_t *partb = parta + (transA ? stat_part_words(K, M, 1) : 0);
  const StatOp sa = amax_given ? StatOp{}
                    : transA   ? stat_op(A, K, M, lda, 1, amax, parta)
                               : stat_op(A, M, K, lda, 0, amax, nullptr);
  const StatOp sb = bmax_given ? StatOp{}
                    : transB   ? stat_op(B, N, K, ldb, 0, bmax, nullptr)
                               : stat_op(B, K, N, ldb, 1, bmax, partb);
  if (!amax_given || !bmax_given) {
    const int rc = amax_given ? stats_launch(sb, StatOp{}, kcnn::as_stream(stream))
                              : stats_launch(sa, sb, kcnn::as_stream(stream));
    if (rc) return rc;
  }
  return gemm_f16x3_st(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc,
                       amax_given ? amax_given : amax, bmax_given ? bmax_given : bmax, bias,
                       pb ? ws : nullptr, pb, stream, mom);
}
extern "C" int kl_gemm_f16x3_bias(int transA, int transB, int M, int N, int K, float alpha,
                                  const float *A, int lda, const float *B, int ldb, float beta,
                                  float *C, int ldc, const uint32_t *amax_given,
                                  const uint32_t *bmax_given, const float *bias, void *ws,
                                  size_t ws_bytes, kcnn_stream_t stream) {
  return gemm_f16x3_full(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc,
                         amax_given, bmax_given, bias, ws, ws_bytes, stream, nullptr);
}
// The weight-gradient product applied as the momentum update in its own
// store (momentum-step.h): for every element g = (op(A) op(B))[i][j],
// prev = momentum prev + a_wd W + a_g g, W += prev, the bits of
// kl_gemm_f16x3_given(alpha 1, beta 0) into a gradient buffer followed by
// hipF_momentum_update, without the buffer's write and read.  W and prev are
// M x N with 16-B aligned rows (hipErrorNotSupported otherwise).
extern "C" int kl_gemm_f16x3_momentum(int transA, int transB, int M, int N, int K,
                                      const float *A, int lda, const float *B, int ldb,
                                      const uint32_t *amax_given, const uint32_t *bmax_given,
                                      float *W, int ldw, float *prev, int ldp, float momentum,
                                      float a_wd, float a_g, void *ws, size_t ws_bytes,
                                      kcnn_stream_t stream) {
  if (!W || !prev || ldw % 4 || ldp % 4 || (uintptr_t)W % 16 || (uintptr_t)prev % 16)
    return (int)hipErrorNotSupported;
  MomentumEpi m;
  m.W = W; m.prev = prev; m.ldw = ldw; m.ldp = ldp;
  m.momentum = momentum; m.a_wd = a_wd; m.a_g = a_g;
  return gemm_f16x3_full(transA, transB, M, N, K, 1.0f, A, lda, B, ldb, 0.0f, nullptr, ldw,
                         amax_given, bmax_given, nullptr, ws, ws_bytes, stream, &m);
}
