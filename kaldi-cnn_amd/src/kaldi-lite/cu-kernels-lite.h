// kaldi-lite/cu-kernels-lite.h -- internal launchers for the generic
// CuMatrix/CuVector ops (not part of the public boundary).
#ifndef KCNN_KALDI_LITE_CU_KERNELS_LITE_H_
#define KCNN_KALDI_LITE_CU_KERNELS_LITE_H_

#include <stddef.h>
#include <stdint.h>

#include "cnsl-hip-kernels.h"

#ifdef __cplusplus
extern "C" {
#endif
int kl_set(float *d, MatrixDim dim, float v, kcnn_stream_t st);
int kl_scale(float *d, MatrixDim dim, float a, kcnn_stream_t st);
int kl_add(float *d, MatrixDim dim, float a, kcnn_stream_t st);
int kl_add_mat(float alpha, const float *A, MatrixDim ad, int transA,
               float beta, float *D, MatrixDim dd, kcnn_stream_t st);
int kl_copy_rows_from_vec(const float *v, float *D, MatrixDim dd,
                          kcnn_stream_t st);
int kl_sum_partials(const float *parts, int S, int m, int n, float beta,
                    float *C, MatrixDim cd, kcnn_stream_t st);
size_t kl_col_sum_workspace_bytes(MatrixDim md);
int kl_col_sum(const float *M, MatrixDim md, float alpha, float beta, float *v,
               void *ws, kcnn_stream_t st);
/* fp32 GEMM on the bf16 MFMAs by an exact 3-way operand split (cu-gemm-x6.hip) */
size_t kl_gemm_x6_workspace_bytes(int M, int N, int K);
int kl_gemm_x6(int transA, int transB, int M, int N, int K, float alpha,
               const float *A, int lda, const float *B, int ldb, float beta,
               float *C, int ldc, void *ws, size_t ws_bytes, kcnn_stream_t st);
/* fp32 GEMM on the f16 MFMAs: two-part f16 split under per-row / per-column
   power-of-two scales (cu-gemm-f16x3.hip).  kl_absmax_rows / kl_absmax_cols
   write a statistics block per row / column set: [max[n], min[n]], the max
   |x| and the min nonzero |x| bit patterns (0: no nonzero element), 2 n
   words (the column form needs kl_absmax_cols_words of scratch);
   kl_gemm_f16x3_st takes the blocks of op(A)'s rows and op(B)'s columns,
   kl_gemm_f16x3 computes them in its workspace.
   Both return hipErrorNotSupported for shapes outside the kernel's
   addressing limits. */
int kl_absmax_rows(const float *X, int rows, int cols, int ld, uint32_t *rmax,
                   kcnn_stream_t st);
size_t kl_absmax_cols_words(int rows, int cols);
int kl_absmax_cols(const float *X, int rows, int cols, int ld, uint32_t *cmax, uint32_t *part,
                   kcnn_stream_t st);
/* kl_absmax_rows of R and kl_absmax_cols of Q (part: kl_absmax_cols_words
   of Q's shape) in one statistics launch, which also sets clear[0] and
   clear[1] to 0 (nullable) */
int kl_absmax_rows_cols(const float *R, int rows, int cols, int ld, uint32_t *rmax,
                        const float *Q, int qrows, int qcols, int ldq, uint32_t *cmax,
                        uint32_t *part, uint32_t *clear, kcnn_stream_t stream);
/* Up to three statistics passes (rows: mode 0; columns: mode 1 with
   kl_absmax_cols_words of part) in one launch set; X_i NULL skips op i;
   pool_cols (nullable): a PoolColDeferred (cnslmat/pool-stats.h) whose
   column kernels run inside the same launches. */
int kl_gemm_stats3(const float *X0, int rows0, int cols0, int ld0, int mode0, uint32_t *out0,
                   uint32_t *part0, const float *X1, int rows1, int cols1, int ld1, int mode1,
                   uint32_t *out1, uint32_t *part1, const float *X2, int rows2, int cols2,
                   int ld2, int mode2, uint32_t *out2, uint32_t *part2, void *pool_cols,
                   kcnn_stream_t stream);
size_t kl_gemm_f16x3_workspace_bytes(int M, int N, int K);
int kl_gemm_f16x3_st(int transA, int transB, int M, int N, int K, float alpha,
                     const float *A, int lda, const float *B, int ldb, float beta, float *C,
                     int ldc, const uint32_t *amax, const uint32_t *bmax, void *ws,
                     size_t ws_bytes, kcnn_stream_t st);
size_t kl_gemm_f16x3_full_workspace_bytes(int M, int N, int K);
int kl_gemm_f16x3(int transA, int transB, int M, int N, int K, float alpha,
                  const float *A, int lda, const float *B, int ldb, float beta, float *C,
                  int ldc, void *ws, size_t ws_bytes, kcnn_stream_t st);
/* kl_gemm_f16x3 with op(A)'s row and/or op(B)'s column statistics supplied
   (nullable; e.g. from the fused conv + pool forward that wrote the operand) */
int kl_gemm_f16x3_given(int transA, int transB, int M, int N, int K, float alpha,
                        const float *A, int lda, const float *B, int ldb, float beta, float *C,
                        int ldc, const uint32_t *amax, const uint32_t *bmax, void *ws,
                        size_t ws_bytes, kcnn_stream_t st);
/* kl_gemm_f16x3_given with C += bias[j] on every row (bias nullable; after
   alpha and beta), in the kernel's own store. */
int kl_gemm_f16x3_bias(int transA, int transB, int M, int N, int K, float alpha,
                       const float *A, int lda, const float *B, int ldb, float beta, float *C,
                       int ldc, const uint32_t *amax_given, const uint32_t *bmax_given,
                       const float *bias, void *ws, size_t ws_bytes, kcnn_stream_t stream);
/* kl_gemm_f16x3_given(alpha 1, beta 0) of a weight gradient applied as the
   momentum update in the GEMM's own store (cnslmat/momentum-step.h): W and
   prev (M x N, 16-B aligned rows) get prev = momentum prev + a_wd W + a_g g,
   W += prev; the bits of the gradient buffer + hipF_momentum_update */
int kl_gemm_f16x3_momentum(int transA, int transB, int M, int N, int K, const float *A,
                           int lda, const float *B, int ldb, const uint32_t *amax_given,
                           const uint32_t *bmax_given, float *W, int ldw, float *prev, int ldp,
                           float momentum, float a_wd, float a_g, void *ws, size_t ws_bytes,
                           kcnn_stream_t stream);
/* the same product from operands already split into bf16 planes h, m, l
   (plane p of X at X + p * ps elements); kl_split_planes makes them */
int kl_split_planes(const float *src, int rows, int cols, int ld, uint16_t *dst, int ldp,
                    int64_t ps, kcnn_stream_t st);
size_t kl_gemm_planes_workspace_bytes(int M, int N, int K);
int kl_gemm_planes(int transA, int transB, int M, int N, int K, float alpha,
                   const uint16_t *A, int lda, int64_t aps, const uint16_t *B, int ldb,
                   int64_t bps, float beta, float *C, int ldc, void *ws, size_t ws_bytes,
                   kcnn_stream_t st);
int kl_dot(const float *A, MatrixDim ad, const float *B, MatrixDim bd,
           int transB, double *out_dev, kcnn_stream_t st);
#ifdef __cplusplus
}
#endif
#endif
