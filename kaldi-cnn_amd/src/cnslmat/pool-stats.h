// cnslmat/pool-stats.h -- the pooled output's operand statistics from the
// fused conv + pool forward.
//
// The register-pooled frame forward (cnsl-conv-frame.hip) writes, besides the
// pooled output and its routing mask, the pooled output's statistics blocks
// (the GEMM's, cu-gemm-f16x3.hip: [max[n], min[n], cnt[n]]) per frame
// (rowmax[3R]: max |value| bits, exact; min nonzero |value| bits, 0 for
// none) and per pooled column (colmax[3 npool]: the max's binade with every
// mantissa bit set, which is all the GEMM's power-of-two scale reads; the
// min over the column's elements under its small bound, 0xffffffff for
// none, which is all the spread test reads), and the count of the small
// elements (f16-split.h; a frame's only when it is spread, a column's in any
// case), through partial_words of scratch
// (kcnn_pool_stats_partial_words).  The FC GEMMs that read the pooled output
// take them as its f16x3 operand scales (kaldi-lite/cu-gemm-f16x3.hip via
// CuGemmStatsHint) instead of reading it once more.  produced = 1 when the
// launch wrote them.
#ifndef KCNN_CNSLMAT_POOL_STATS_H_
#define KCNN_CNSLMAT_POOL_STATS_H_

#include <stddef.h>
#include <stdint.h>

#include "cnsl-hip-kernels.h"  // MatrixDim, kcnn_stream_t

struct PoolStatsOut {
  uint32_t *rowmax = nullptr, *colmax = nullptr, *partials = nullptr;
  size_t partial_words = 0;
  int produced = 0;
};

// hipF_conv2d_maxpool (include/cnsl-hip-kernels.h) plus the statistics when
// its kernel gives them (stats nullable), and the scratch words they need
// (0: the layer has no frame kernel)
extern "C" {
int kcnn_conv2d_maxpool_stats(const float *in, MatrixDim in_dim, int in_height,
                              int in_width, int in_channel, int pad_h, int pad_w,
                              const float *kernel, MatrixDim kernel_dim,
                              int kernel_height, int kernel_width, int group,
                              const float *bias, float *out, MatrixDim out_dim,
                              float *pool, MatrixDim pool_dim, unsigned char *mask,
                              int mask_stride, int pool_channel_dim,
                              kcnn_stream_t stream, PoolStatsOut *stats);
size_t kcnn_conv2d_maxpool_stats_words(int rows, int in_height, int in_width,
                                       int in_channel, int kernel_height, int kernel_width,
                                       int group, int pool_channel_dim);
}

// The pooled output's column statistics (the maxima from the forward's
// exponent bytes, then the small elements' minima and counts: two small
// kernels) left to their consumer instead of launched by the forward.  The
// only reader of the column block is the FC weight-gradient GEMM, which runs
// in the backward; the FC backward's statistics launches take this work
// over (kl_gemm_stats3), and any other f16x3 GEMM that reads the column
// block first completes it (kcnn_pool_cols_complete).  The exponent bytes
// must live until then (the runtime keeps them per layer).
struct PoolColDeferred {
  const uint8_t *pcol = nullptr;  // exponent bytes [nblk][npool]
  int nblk = 0, npool = 0;
  const float *P = nullptr;       // the pooled output (suspect frames' rows)
  int ps = 0, R = 0, vec = 0;
  uint32_t *rowblk = nullptr, *colblk = nullptr;  // the statistics blocks
  int pending = 0;
};
// While a request is set on this thread, the fused forward that writes the
// statistics (kcnn_conv2d_maxpool_stats) fills it and sets pending instead
// of launching the column kernels.  Returns the previous request.
PoolColDeferred *kcnn_pool_defer_request(PoolColDeferred *d);
PoolColDeferred *kcnn_pool_defer_current();
// The column kernels of a pending request (pending -> 0); 0 or a HIP error.
int kcnn_pool_cols_complete(PoolColDeferred *d, kcnn_stream_t stream);
struct PoolColDeferScope {
  explicit PoolColDeferScope(PoolColDeferred *d) : prev(kcnn_pool_defer_request(d)) {}
  ~PoolColDeferScope() { kcnn_pool_defer_request(prev); }
  PoolColDeferred *prev;
};

#endif  // KCNN_CNSLMAT_POOL_STATS_H_
