/*
 * include/cnsl-hip-kernels.h -- the extern "C" kernel shim of the MI355X
 * (gfx950) build of kaldi-cnn's CNN hot path.
 *
 * This header replaces the reference's CUDA launcher ABI
 * src/cnslmat/cnsl-cu-kernels.h:22-70 (`cudaF_*`, called only through the
 * `cnsl::cuda_*` overloads :73-197 from src/cnslmat/conv2D.cc).  Differences,
 * all deliberate:
 *   - no dim3 grid/block arguments: launch geometry belongs to the tuned
 *     kernel, not to the caller;
 *   - every entry takes the hipStream_t to launch on and returns an int
 *     (hipError_t value; 0 = success) instead of relying on
 *     CU_SAFE_CALL(cudaGetLastError()) in the caller (conv2D.cc:108 ff.);
 *   - float only (Conv2D's temporaries are CuMatrix<BaseFloat>,
 *     so the reference's double launchers :47-68 can never be used);
 *   - element offsets are 64-bit inside the kernels;
 *   - convolution is implicit-GEMM on MFMA: the im2col / col2im / split /
 *     copy kernels (:25-28, :35) are still exported for API completeness,
 *     but Conv2D itself never materialises the im2col matrix.
 * Plain pointers + MatrixDim only -- no C++ or torch types.
 */
#ifndef KCNN_CNSL_HIP_KERNELS_H_
#define KCNN_CNSL_HIP_KERNELS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef KCNN_MATRIXDIM_DEFINED
#define KCNN_MATRIXDIM_DEFINED
/* Kaldi's ::MatrixDim (cudamatrix/cu-matrixdim.h, upstream): passed by value,
 * element (r, c) at data[r * stride + c]. */
typedef struct MatrixDim_ {
  int32_t rows;
  int32_t cols;
  int32_t stride;
} MatrixDim;
#endif

/* An opaque HIP stream (hipStream_t); NULL = the legacy default stream. */
typedef void *kcnn_stream_t;

/* ---- reshape / bandwidth kernels (one per reference launcher) ----------- */

/* replaces cudaF_span_row_to_convmat, cnsl-cu-kernels.h:25 (im2col rows
 * [row_offset, row_offset + span.rows) of conv2D.cc:120-133). */
int hipF_span_row_to_convmat(const float *in, MatrixDim in_dim, float *span,
                             MatrixDim span_dim, int in_height, int in_width,
                             int in_channel, int kernel_height,
                             int kernel_width, int64_t row_offset,
                             kcnn_stream_t stream);
/* replaces cudaF_convmat_to_out, cnsl-cu-kernels.h:28 (col2im). */
int hipF_convmat_to_out(const float *conv_mat, MatrixDim conv_dim, float *out,
                        MatrixDim out_dim, int out_height, int out_width,
                        int num_sample, kcnn_stream_t stream);
/* replaces cudaF_add_mat_rep_vec, cnsl-cu-kernels.h:29. */
int hipF_add_mat_rep_vec(const float *vec, int rep, float *out,
                         MatrixDim out_dim, kcnn_stream_t stream);
/* replaces cudaF_flip_mat, cnsl-cu-kernels.h:30. */
int hipF_flip_mat(const float *orig, MatrixDim orig_dim, int kernel_height,
                  int kernel_width, int group, float *flip, MatrixDim flip_dim,
                  kcnn_stream_t stream);
/* replaces cudaF_pad_zero, cnsl-cu-kernels.h:31. */
int hipF_pad_zero(const float *orig, MatrixDim orig_dim, int orig_height,
                  int orig_width, int kernel_height, int kernel_width,
                  float *padmat, MatrixDim padmat_dim, kcnn_stream_t stream);
/* replaces cudaF_tp_block, cnsl-cu-kernels.h:32. */
int hipF_tp_block(const float *in, MatrixDim in_dim, float *out,
                  MatrixDim out_dim, int block_size, kcnn_stream_t stream);
/* replaces cudaF_tp_inside_block, cnsl-cu-kernels.h:33. */
int hipF_tp_inside_block(const float *in, MatrixDim in_dim, float *out,
                         MatrixDim out_dim, int block_size,
                         kcnn_stream_t stream);
/* replaces cudaF_mod_permute_row, cnsl-cu-kernels.h:34. */
int hipF_mod_permute_row(const float *in, MatrixDim in_dim, float *out,
                         MatrixDim out_dim, int block_size, int in_channel,
                         kcnn_stream_t stream);
/* replaces cudaF_copy_rows_at, cnsl-cu-kernels.h:35. */
int hipF_copy_rows_at(const float *src, MatrixDim src_dim, float *dest,
                      MatrixDim dest_dim, int64_t row_offset,
                      kcnn_stream_t stream);

/* ---- max pooling ----------------------------------------------------------
 * mode: 0 = non-overlap 3-D pool (cudaF_maxpool_prop/backprop,
 * cnsl-cu-kernels.h:36-38), 1 = overlap (cudaF_maxpoolchannel_overlap_*,
 * :39-41), 2 = overlap2D (cudaF_maxpoolchannel_overlap2D_*, :42-44).
 * backprop: write_all != 0 writes every in_deriv element (0 or the routed
 * derivative: the fused form of MaxpoolComponent::Backprop's zeroing Resize,
 * nnet-component-nnet0.cc:889); write_all == 0 touches only the routed
 * elements, like the reference kernel (cnsl-cu-kernels.cu:302-303).  The
 * overlapping modes are computed in gather form (one writer per in_deriv
 * element, contributions summed in output order): deterministic, unlike the
 * reference's racy `dest += err` (cnsl-cu-kernels.cu:395-398, :496-499). */
int hipF_maxpool_prop(const float *src, MatrixDim src_dim, float *pool,
                      MatrixDim pool_dim, int in_height, int in_width,
                      int pool_height_dim, int pool_width_dim,
                      int pool_channel_dim, int mode, kcnn_stream_t stream);
int hipF_maxpool_backprop(const float *in_val, MatrixDim in_val_dim,
                          const float *out_val, MatrixDim out_val_dim,
                          const float *out_deriv, MatrixDim out_deriv_dim,
                          float *dest, MatrixDim dest_dim, int in_height,
                          int in_width, int pool_height_dim,
                          int pool_width_dim, int pool_channel_dim, int mode,
                          int write_all, kcnn_stream_t stream);

/* MaxpoolComponent::Backprop (nnet-component-nnet0.cc:882-892, Resize to
 * zero + Maxpool_backprop A.9) of a channel-only pool from the mask written
 * by hipF_conv2d_maxpool: in_deriv[n][(pc*(j/P) + c)*P + j%P] = bit c of
 * mask[n * mask_stride + j] ? out_deriv[n][j] : 0, every element written. */
int hipF_maxpool_backprop_mask(const unsigned char *mask, int mask_stride,
                               const float *out_deriv, MatrixDim out_deriv_dim,
                               float *in_deriv, MatrixDim in_deriv_dim,
                               int in_height, int in_width,
                               int pool_channel_dim, kcnn_stream_t stream);

/* MaxpoolComponent::Backprop of a 3-D window from hipF_conv2d_maxpool3d's
 * 16-bit mask: every input written, dP of its window where its bit is set,
 * else 0 (A.9). */
int hipF_maxpool_backprop_mask3d(const unsigned short *mask, int mask_stride,
                                 const float *out_deriv, MatrixDim out_deriv_dim,
                                 float *in_deriv, MatrixDim in_deriv_dim,
                                 int in_height, int in_width, int pool_height_dim,
                                 int pool_width_dim, int pool_channel_dim,
                                 kcnn_stream_t stream);

/* ModPermuteChannel (conv2D.cc:685-727, kernel cnsl-cu-kernels.cu:505-528,
 * launcher cnsl-cu-kernels.h:45 cudaF_mod_permute_channels): moves the
 * in_height x in_width maps of `comp` into channel slot
 * c*num_component + comp_idx of `container` (or back when
 * from_comp_to_container == 0). */
int hipF_mod_permute_channels(float *comp, MatrixDim comp_dim, float *container,
                              MatrixDim container_dim, int comp_idx,
                              int num_component, int in_height, int in_width,
                              int from_comp_to_container, kcnn_stream_t stream);

/* ---- convolution (MFMA implicit GEMM) ------------------------------------
 * Replaces the im2col + cuBLAS sgemm + copy + col2im sequence of
 * CuMatrixBase::Conv2D (conv2D.cc:43-201; launchers cnsl-cu-kernels.h:25,
 * :28, :35 plus AddMatMat).  in: [R x H*W*C] with H x W maps padded
 * *virtually* by (pad_h, pad_w) zeros on each side (PaddingZero,
 * conv2D.cc:289-344, fused); kernel: [kh*kw*C x G]; out: concat ?
 * [R x oh*ow*G] (col = g*oh*ow + p) : [oh*ow*R x G] (row = p*R + n), with
 * oh = H + 2 pad_h - kh + 1.  bias (nullable, concat only) fuses
 * AddMatRepVec(bias, oh*ow) (conv2D.cc:213-242).  `workspace` may be NULL
 * when hipF_conv2d_workspace_bytes() returns 0. */
size_t hipF_conv2d_workspace_bytes(MatrixDim in_dim, int in_height,
                                   int in_width, int in_channel, int pad_h,
                                   int pad_w, int kernel_height,
                                   int kernel_width, int group);
int hipF_conv2d(const float *in, MatrixDim in_dim, int in_height, int in_width,
                int in_channel, int pad_h, int pad_w, const float *kernel,
                MatrixDim kernel_dim, int kernel_height, int kernel_width,
                int group, const float *bias, float *out, MatrixDim out_dim,
                int concat, void *workspace, size_t workspace_bytes,
                kcnn_stream_t stream);

/* ConvolutionComponent::Propagate (nnet-component-nnet0.cc:423-446) followed
 * by a channel-only MaxpoolComponent::Propagate (:869-880, pool 1 x 1 x
 * pool_channel_dim, no overlap) in one pass: out as hipF_conv2d(concat=1),
 * pool = Maxpool_prop(out) (conv2D.cc:465-559, bit-identical), and
 * mask[n * mask_stride + j] bit c = (out[n][(pc*(j/P) + c)*P + j%P] ==
 * pool[n][j]) with P = oh*ow -- the routing MaxpoolComponent::Backprop
 * (:882-892) derives from in_value == out_value.  pool_channel_dim in
 * {2, 4, 8}.  Returns -1 without launching when the geometry is not covered
 * (the caller then runs the two components separately). */
int hipF_conv2d_maxpool(const float *in, MatrixDim in_dim, int in_height,
                        int in_width, int in_channel, int pad_h, int pad_w,
                        const float *kernel, MatrixDim kernel_dim,
                        int kernel_height, int kernel_width, int group,
                        const float *bias, float *out, MatrixDim out_dim,
                        float *pool, MatrixDim pool_dim, unsigned char *mask,
                        int mask_stride, int pool_channel_dim,
                        kcnn_stream_t stream);

/* ConvolutionComponent::Propagate followed by RectifiedLinearComponent::
 * Propagate (reference nnet-component.cc:799-805, ApplyFloor(0)) in one pass:
 * out = max(conv(in) + bias, 0) in the concat layout (x < 0 -> 0, NaN kept).
 * The conv output itself is not stored.  Returns -1 without launching when
 * the shape takes a forward kernel without this epilogue (the caller then
 * runs the two components). */
int hipF_conv2d_relu(const float *in, MatrixDim in_dim, int in_height, int in_width,
                     int in_channel, int pad_h, int pad_w, const float *kernel,
                     MatrixDim kernel_dim, int kernel_height, int kernel_width,
                     int group, const float *bias, float *out, MatrixDim out_dim,
                     kcnn_stream_t stream);

/* The same fusion for a 3-D pooling window (ph x pw x pc, non-overlapping,
 * pc dividing 32, ph*pw*pc <= 16; c5's 3 x 1 x 4): pool as A.8 and a 16-bit
 * mask per pooled value, bit c*pw*ph + w*ph + h = "input (c, w, h) of the
 * window equals the max" (mask_stride in elements).  -1 = not covered. */
int hipF_conv2d_maxpool3d(const float *in, MatrixDim in_dim, int in_height,
                          int in_width, int in_channel, int pad_h, int pad_w,
                          const float *kernel, MatrixDim kernel_dim,
                          int kernel_height, int kernel_width, int group,
                          const float *bias, float *out, MatrixDim out_dim,
                          float *pool, MatrixDim pool_dim, unsigned short *mask,
                          int mask_stride, int pool_height_dim, int pool_width_dim,
                          int pool_channel_dim, kcnn_stream_t stream);

/* Weight gradient of ConvolutionComponent::Update (nnet-component-nnet0.cc:
 * 738-765 + :775): grad_W[c*kh*kw + kx*kh + ky][g] = sum_{n,p} X[n][..] *
 * dY[n][g*P + p] (ModPermuteRow'ed layout), grad_b[g] = sum_{n,p} dY[n][g*P+p].
 * Fuses TpBlock + TpInsideBlock + Conv2D(concat=false) + ModPermuteRow +
 * AddRowSumMat; deterministic split-K (fixed reduction order). */
size_t hipF_conv2d_wgrad_workspace_bytes(MatrixDim in_dim, int in_height,
                                         int in_width, int in_channel,
                                         int pad_h, int pad_w,
                                         int kernel_height, int kernel_width,
                                         int group);
int hipF_conv2d_wgrad(const float *in, MatrixDim in_dim, int in_height,
                      int in_width, int in_channel, int pad_h, int pad_w,
                      const float *out_deriv, MatrixDim out_deriv_dim,
                      int kernel_height, int kernel_width, int group,
                      float *grad_W, MatrixDim grad_W_dim, float *grad_b,
                      void *workspace, size_t workspace_bytes,
                      kcnn_stream_t stream);

/* Data gradient of ConvolutionComponent::Backprop (nnet-component-nnet0.cc:
 * 461-540): in_deriv [R x H*W*C] from out_deriv [R x oh*ow*G] and the
 * (unflipped) kernel [kh*kw*C x G] of a convolution whose input was padded
 * by (pad_h, pad_w).  Replaces either reference branch -- PaddingZero(dY) +
 * FlipMat(W) + Conv2D, or TpInsideBlock + FlipMat + AddMat(kTrans) + TpBlock
 * + PaddingZero + Conv2D + TpBlock -- with no materialised intermediate
 * (both compute the same sum).  Needs pad <= kernel - 1 (reference :533). */
size_t hipF_conv2d_dgrad_workspace_bytes(MatrixDim out_deriv_dim,
                                         int in_height, int in_width,
                                         int in_channel, int pad_h, int pad_w,
                                         int kernel_height, int kernel_width,
                                         int group);
int hipF_conv2d_dgrad(const float *out_deriv, MatrixDim out_deriv_dim,
                      int in_height, int in_width, int in_channel, int pad_h,
                      int pad_w, const float *kernel, MatrixDim kernel_dim,
                      int kernel_height, int kernel_width, int group,
                      float *in_deriv, MatrixDim in_deriv_dim, void *workspace,
                      size_t workspace_bytes, kcnn_stream_t stream);

/* Whole backward of ConvolutionComponent (Backprop with an update,
 * nnet-component-nnet0.cc:461-540 + Update :738-775): in_deriv (nullable)
 * AND grad_W / grad_b from one pass over out_deriv.  Equal to
 * hipF_conv2d_dgrad + hipF_conv2d_wgrad (same sums; to which it falls back
 * for shapes outside the fused kernel's range: kh*kw*C <= 31, group a
 * multiple of 32 up to 128, oh*ow <= 384). */
size_t hipF_conv2d_backward_workspace_bytes(MatrixDim in_dim, int in_height,
                                            int in_width, int in_channel,
                                            int pad_h, int pad_w,
                                            int kernel_height, int kernel_width,
                                            int group);
int hipF_conv2d_backward(const float *in, MatrixDim in_dim, int in_height,
                         int in_width, int in_channel, int pad_h, int pad_w,
                         const float *out_deriv, MatrixDim out_deriv_dim,
                         const float *kernel, MatrixDim kernel_dim,
                         int kernel_height, int kernel_width, int group,
                         float *in_deriv, MatrixDim in_deriv_dim, float *grad_W,
                         MatrixDim grad_W_dim, float *grad_b, void *workspace,
                         size_t workspace_bytes, kcnn_stream_t stream);

/* MaxpoolComponent::Backprop of a channel-only pool (1 x 1 x pc, pc in
 * {4, 8}) from the routing mask of hipF_conv2d_maxpool, followed by
 * hipF_conv2d_backward of the ConvolutionComponent below it, in one pass:
 * out_deriv (= hipF_maxpool_backprop_mask(mask, pool_deriv)) is built per
 * 32-map slab in LDS and never stored.  Same results as the two calls.
 * grad_W / grad_b nullable when in_deriv is not (and vice versa).  Returns
 * -1 without launching when the shape is not covered (the fused backward's
 * range, G <= 128 per launch); the caller then makes the two calls. */
int hipF_conv2d_backward_pooled(const float *in, MatrixDim in_dim, int in_height,
                                int in_width, int in_channel, int pad_h, int pad_w,
                                const unsigned char *mask, int mask_stride,
                                const float *pool_deriv, MatrixDim pool_deriv_dim,
                                int pool_channel_dim, const float *kernel,
                                MatrixDim kernel_dim, int kernel_height,
                                int kernel_width, int group, float *in_deriv,
                                MatrixDim in_deriv_dim, float *grad_W,
                                MatrixDim grad_W_dim, float *grad_b, void *workspace,
                                size_t workspace_bytes, kcnn_stream_t stream);

/* The same for a 3-D window pool_height_dim x 1 x pool_channel_dim
 * (pool_height_dim in {2, 3} dividing the conv's out-height, pool_channel_dim
 * in {4, 8}, at most 16 window elements: c5's P1 3 x 1 x 4) from the 16-bit
 * routing mask of hipF_conv2d_maxpool3d (mask_stride in elements):
 * MaxpoolComponent::Backprop (hipF_maxpool_backprop_mask3d) folded into
 * ConvolutionComponent::Backprop.  -1 without launching when not covered. */
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
                                  size_t workspace_bytes, kcnn_stream_t stream);

/* Momentum / weight-decay step of ConvolutionComponent::Update
 * (nnet-component-nnet0.cc:769-775) and FullyConnectedComponent::UpdateSimple
 * (:1137-1142), one pass:  prev = momentum*prev + a_wd*W + a_g*grad;
 * W += prev;  b += a_g*grad_b (b/grad_b nullable). */
int hipF_momentum_update(float *W, MatrixDim W_dim, float *prev,
                         MatrixDim prev_dim, const float *grad,
                         MatrixDim grad_dim, float momentum, float a_wd,
                         float a_g, float *b, const float *grad_b, int b_dim,
                         kcnn_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* KCNN_CNSL_HIP_KERNELS_H_ */
