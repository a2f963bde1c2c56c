// cnslmat/pool-stats-dev.h -- device code of the pooled output's column
// statistics (pool-stats.h): the column maxima from the fused forward's
// per-workgroup exponent bytes, and the small elements' minima and counts
// from the suspect frames.  Shared by the standalone kernels the forward
// launches (cnsl-conv-frame.hip pool_colmax_kernel, pool_count_kernel) and
// the FC backward's statistics launches, which take this work over when the
// forward leaves it pending (kaldi-lite/cu-gemm-f16x3.hip kl_gemm_stats3).
#ifndef KCNN_CNSLMAT_POOL_STATS_DEV_H_
#define KCNN_CNSLMAT_POOL_STATS_DEV_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f16-split.h"

namespace kcnn {

// Column maxima of the pooled output from the forward's per-workgroup
// partials [nblk][npool], one exponent byte each (the |x| bits >> 23: the
// GEMM's scale needs only the binade).  colmax[c] = the largest partial's
// binade with every mantissa bit set, an upper bound in the max's binade (so
// the same scale; 0x7f... for Inf; an all-zero column gets the subnormal
// bound, harmless).  colmax zeroed by the forward; blockIdx.y takes 32
// workgroups' rows, atomic max across those chunks.
// A thread takes four columns (one dword of bytes per row; npool % 4 == 0,
// else one column), its 32 rows' loads in flight together.
constexpr int COLMAX_ROWS = 32;
// (block (bx, by) of the grid ((column quads + 255) / 256, nblk / COLMAX_ROWS))
__device__ __forceinline__ void pool_colmax_block(const uint8_t *__restrict__ pcol, int nblk,
                                                  int npool, uint32_t *__restrict__ colmax,
                                                  int bx, int by) {
  const bool quad = npool % 4 == 0;
  const int c = (bx * 256 + threadIdx.x) * (quad ? 4 : 1);
  if (c >= npool) return;
  const int b0 = by * COLMAX_ROWS, b1 = min(nblk, b0 + COLMAX_ROWS);
  uint32_t w[COLMAX_ROWS];
#pragma unroll
  for (int i = 0; i < COLMAX_ROWS; i++) {
    const int b = b0 + i;
    const uint8_t *q = pcol + (int64_t)b * npool + c;
    w[i] = b >= b1 ? 0u : quad ? *reinterpret_cast<const uint32_t *>(q) : (uint32_t)*q;
  }
  uint32_t m[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < COLMAX_ROWS; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) m[j] = max(m[j], (w[i] >> (8 * j)) & 0xffu);
#pragma unroll
  for (int j = 0; j < 4; j++)
    if (j == 0 || quad) atomicMax(colmax + c + j, (m[j] << 23) | 0x7fffffu);
}

// The pooled output's small elements (f16-split.h) after pool_colmax_kernel,
// from the exact row statistics and the column maxima, without a column
// pass.  Every small element of any finite column lies below 2^eg, eg = E -
// 17 for E the binade of the largest finite value (the largest row max), so
// only the frames whose row min lies below 2^eg hold any ("suspect" frames:
// 41 of c2's 4096), and reading those frame rows alone gives every
// column's small elements: their count (atomic add) and min (atomic min;
// 0xffffffff for none), which is all the spread test reads.  A column's
// count covers its small elements whether or not it is spread: the 2^-25
// bound the GEMM's check prices holds for every small element, so a count in
// a column that is not spread only adds checks (rare: 4 of c2's 11616
// columns have one).  A frame row's count is the GEMM's (0 unless spread),
// taken on the same read.  Every block derives the suspect list from the
// row statistics (the same list in every block) and takes its entries
// block, block + grid, ...; a non-suspect frame's count is zeroed by the
// block that owns the frame index in the same stride.
constexpr int CNT_LIST = 16;  // suspect frames per block and pass (4096 frames / 256 blocks)
__device__ __forceinline__ void count_elem(float x, float rbound, int eg, int c, int npool,
                                           uint32_t *colblk, uint32_t &rcnt) {
  const uint32_t v = __float_as_uint(x) & 0x7fffffffu;
  if (v == 0) return;
  rcnt += __uint_as_float(v) < rbound ? 1u : 0u;
  const int ev = f16x3::ebits(v);
  if (ev >= eg) return;  // the common case: small in no column
  const uint32_t cm = colblk[c];
  if (cm < f16x3::NONFINITE && ev < f16x3::ebits(cm) - 17) {
    atomicMin(colblk + npool + c, v);
    atomicAdd(colblk + 2 * (size_t)npool + c, 1u);
  }
}
// the block's shared state (a __shared__ object of the calling kernel)
struct PoolCountSmem {
  uint32_t red[2][4];
  int wsum[4];
  uint32_t list[CNT_LIST][3];  // (frame, row max, row min)
  int nlist;
};
// block b of nb (nb <= 256: a pass of 4096 frames gives a block at most
// CNT_LIST suspect frames)
__device__ __forceinline__ void pool_count_block(const float *__restrict__ P, int ps, int R,
                                                 int npool, int vec,
                                                 uint32_t *__restrict__ rowblk, uint32_t *colblk,
                                                 int b, int nb, PoolCountSmem &sm) {
  auto &red = sm.red;
  auto &wsum = sm.wsum;
  auto &list = sm.list;
  int &nlist = sm.nlist;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) nlist = 0;
  // thread t's frames t + 256 i, RF per pass (c2: one pass), their maxima
  // and minima loaded together: one memory latency
  constexpr int RF = 16;
  int base = 0;
  for (int f0 = 0; f0 < R; f0 += 256 * RF) {
    uint32_t m[RF], mn[RF];
#pragma unroll
    for (int i = 0; i < RF; i++) {
      const int f = f0 + tid + 256 * i;
      m[i] = f < R ? rowblk[f] : 0u;
      mn[i] = f < R ? rowblk[R + f] : 0u;
    }
    // eg from the largest finite row max over all frames (any Inf / NaN
    // row: every frame with a nonzero min is suspect, the safe side).  Only
    // the first pass can hold them all: with more than one pass (R > 4096)
    // the maxima are gathered by a first sweep below.
    uint32_t gm = 0, inf = 0;
    if (R <= 256 * RF) {
#pragma unroll
      for (int i = 0; i < RF; i++) {
        if (m[i] < f16x3::NONFINITE) gm = max(gm, m[i]);
        else inf = 1;
      }
    } else {
      for (int f = tid; f < R; f += 256) {
        const uint32_t x = rowblk[f];
        if (x < f16x3::NONFINITE) gm = max(gm, x);
        else inf = 1;
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      gm = max(gm, (uint32_t)__shfl_xor((int)gm, d));
      inf |= (uint32_t)__shfl_xor((int)inf, d);
    }
    if (lane == 0) {
      red[0][wave] = gm;
      red[1][wave] = inf;
    }
    __syncthreads();
    gm = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
    inf = red[1][0] | red[1][1] | red[1][2] | red[1][3];
    const int eg = inf ? 1 << 20 : gm ? f16x3::ebits(max(gm, 0x7fffffu)) - 17 : -(1 << 20);
    // the suspect frames, numbered in (pass, thread, i) order (the same list
    // in every block): per-thread counts, then a block prefix sum
    uint32_t sus = 0;
#pragma unroll
    for (int i = 0; i < RF; i++)
      if (mn[i] != 0 && f16x3::ebits(mn[i]) < eg) sus |= 1u << i;
    const int cnt = __builtin_popcount(sus);
    int inc = cnt;  // inclusive prefix over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(inc, d);
      if (lane >= d) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int idx = base + inc - cnt;
    for (int w = 0; w < wave; w++) idx += wsum[w];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
#pragma unroll
    for (int i = 0; i < RF; i++) {
      const int f = f0 + tid + 256 * i;
      if ((sus >> i) & 1) {
        if (idx % nb == b) {  // (< CNT_LIST entries: host grid)
          const int k = atomicAdd(&nlist, 1);
          list[k][0] = (uint32_t)f;
          list[k][1] = m[i];
          list[k][2] = mn[i];
        }
        idx++;
      } else if (f < R && f % nb == b) {
        rowblk[2 * (size_t)R + f] = 0;
      }
    }
    base += total;
    __syncthreads();  // (wsum, red reused)
    // the block's suspect frames of this pass: each row read once, every
    // thread's float4s of it loaded together
    const int n = nlist;
    constexpr int V = 12;  // float4 loads in flight per thread (c2: the whole row)
    for (int e = 0; e < n; e++) {
      const int f = (int)list[e][0];
      const uint32_t rmx = list[e][1], rmn = list[e][2];
      const float rbound = f16x3::spread(rmx, rmn) ? f16x3::small_bound(rmx) : 0.0f;
      const float *x = P + (int64_t)f * ps;
      uint32_t rcnt = 0;
      if (vec) {
        for (int c0 = tid * 4; c0 < npool; c0 += V * 1024) {
          float4 q[V];
#pragma unroll
          for (int j = 0; j < V; j++)
            if (c0 + j * 1024 < npool)
              q[j] = *reinterpret_cast<const float4 *>(x + c0 + j * 1024);
#pragma unroll
          for (int j = 0; j < V; j++) {
            const int c = c0 + j * 1024;
            if (c >= npool) break;
            count_elem(q[j].x, rbound, eg, c, npool, colblk, rcnt);
            count_elem(q[j].y, rbound, eg, c + 1, npool, colblk, rcnt);
            count_elem(q[j].z, rbound, eg, c + 2, npool, colblk, rcnt);
            count_elem(q[j].w, rbound, eg, c + 3, npool, colblk, rcnt);
          }
        }
      } else {
        for (int c = tid; c < npool; c += 256) count_elem(x[c], rbound, eg, c, npool, colblk, rcnt);
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) rcnt += (uint32_t)__shfl_xor((int)rcnt, d);
      if (lane == 0) red[0][wave] = rcnt;
      __syncthreads();
      if (tid == 0) rowblk[2 * (size_t)R + f] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      __syncthreads();  // (red reused)
    }
    if (tid == 0) nlist = 0;
    __syncthreads();
  }
}

}  // namespace kcnn

#endif  // KCNN_CNSLMAT_POOL_STATS_DEV_H_
