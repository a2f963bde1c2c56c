/*
 * include/kcnn.h -- extern "C" entry points of libkcnn.so above the kernel
 * shim (include/cnsl-hip-kernels.h): the CuMatrixBase extension methods and
 * the nnet2 components, callable with plain device pointers + MatrixDim.
 *
 * Each entry replaces one reference interface:
 *   kcnn_mat_*        CuMatrixBase<float>::{Conv2D, AddMatRepVec, FlipMat,
 *                     PaddingZero, TpBlock, TpInsideBlock, ModPermuteRow,
 *                     Maxpool_prop, Maxpool_backprop}
 *                     (reference src/cudamatrix/cu-matrix.h:451-480;
 *                     bodies src/cnslmat/conv2D.cc:43-684)
 *   kcnn_component_*  nnet2::Component / UpdatableComponent virtuals as the
 *                     nnet0 components override them
 *                     (reference src/nnet0/nnet-component-nnet0.h:23-232,
 *                     src/nnet2/nnet-component.h:157-348) and the factory
 *                     Component::NewFromString / ReadNew
 *                     (src/nnet2/nnet-component.cc:38-136)
 *                     Also the upstream nnet2 components either side of
 *                     the CNN path: SpliceComponent and
 *                     RectifiedLinearComponent (src/nnet2/nnet-component.cc
 *                     :799-827, :2524-2866), by the same entry points.
 *   kcnn_nnet_*       the propagate/backprop loop of upstream nnet2's
 *                     NnetUpdater (not vendored by the reference)
 *                     over a stack of these components.
 *
 * Conventions: every pointer argument to matrix data is DEVICE memory on the
 * active HIP device; functions return 0 on success and a nonzero code on
 * failure (KALDI_ASSERT / KALDI_ERR / HIP errors), with the message in
 * kcnn_last_error().  Output matrices are caller-allocated with the sizes the
 * reference methods would Resize() them to.  All work is enqueued on the
 * stream set by kcnn_set_stream (default: the legacy NULL stream).
 */
#ifndef KCNN_KCNN_H_
#define KCNN_KCNN_H_

#include <stddef.h>
#include <stdint.h>

#include "cnsl-hip-kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- runtime ------------------------------------------------------------ */
const char *kcnn_last_error(void);
const char *kcnn_version(void);
/* Device allocations (CuDevice::Malloc calls) so far: a HIP graph captured
 * over the caching allocator's blocks stays valid while this does not move
 * (bench.py --graph). */
unsigned long long kcnn_device_malloc_calls(void);
/* The f16x3 implicit GEMM's cumulative counts since the last reset (a test
 * and bench diagnostic, no reference counterpart): out[0] its calls, out[1]
 * the tiles and out[2] the single elements its fp32 fix-up kernels
 * recomputed; reset != 0 zeroes them.  Synchronises the device. */
int kcnn_conv_fix_counts(unsigned long long *out, int reset);
/* CuDevice::SelectGpuId(use_gpu, device) (upstream cu-device.h). */
int kcnn_init(int device);
int kcnn_set_stream(kcnn_stream_t stream);
int kcnn_synchronize(void);
int kcnn_set_literal_path(int literal);  /* replay reference call sequences */
int kcnn_set_profiling(int on);
/* kcnn_nnet_* runtime: run a ConvolutionComponent followed by a
 * non-overlapping MaxpoolComponent (1 x 1 x pc, or a 3-D window) as one fused
 * forward that also saves the pool's routing mask, and backprop that pool
 * from the mask.  Outputs and derivatives are identical either way.
 *   0: off.
 *   1 (default): on; the conv output, which nothing in the training step
 *      reads any more, is not stored.  kcnn_nnet_output recomputes it on
 *      request until that conv's backprop has run, and fails after.
 *   2: on, and the conv output is stored as well.
 * Env KCNN_FUSE sets the initial mode. */
int kcnn_set_fusion(int mode);
/* How CuMatrixBase::AddMatMat (every FullyConnectedComponent GEMM) computes
 * its fp32 product (upstream: cuBLAS sgemm, cu-matrix.cc AddMatMat):
 *   0: rocBLAS sgemm on the fp32-input MFMA;
 *   1: the in-house kernel on the bf16 MFMA with each fp32 operand split
 *      exactly into three bf16 parts and the six leading cross products kept
 *      (cu-gemm-x6.hip); the dot-product error bound of sgemm (1e-5 * S per
 *      element) for operands above 2^-110;
 *   2 (default): the in-house kernel on the f16 MFMA with each operand scaled
 *      by a power of two per row of op(A) / column of op(B) and split into
 *      two f16 parts, three cross products kept (cu-gemm-f16x3.hip); the
 *      split's own bound is per scale group (f16-split.h), and the products
 *      touching a group with elements far under its max are checked and
 *      recomputed in fp32 where needed, so every element meets the 1e-5 * S
 *      bound at any fp32 range; IEEE Inf / NaN rows and columns; shapes past
 *      its 32-bit addressing run mode 1.
 * Env KCNN_GEMM (0/1/2) sets the initial mode. */
int kcnn_set_gemm_mode(int mode);
/* Kernel-family selectors (kaldi-lite/kcnn-knobs.h): each picks
 * one of the implementations of the same fp32 math: the split-operand
 * kernels on the f16 / bf16 matrix cores (f16x3: two f16 parts under a
 * power-of-two scale, three products; bf16x6: three bf16 parts, six
 * products) or the fp32-input MFMA kernels (0).
 *   "fwd_x6"   frame-resident conv forward      2 (default, f16x3) / 1 / 0
 *   "bwd_x6"   fused conv backward              1 (default) / 0
 *   "igemm_x6" implicit-GEMM forward and dgrad  2 (default: f16x3 for
 *              convolutions of >= 2^34 flop, bf16x6 below) / 3 (f16x3 for
 *              all) / 1 (bf16x6) / 0
 *   "wgrad_x6" long-kernel weight gradient      2 (default, wide bf16x6) / 3
 *              (wide f16x3) / 1 (128-wide bf16x6) / 0
 *   "gemm"     AddMatMat (= kcnn_set_gemm_mode) 2 (default, f16x3) / 1 / 0
 * The environment variables KCNN_FWD_X6, KCNN_BWD_X6, KCNN_IGEMM_X6,
 * KCNN_WGRAD_X6 and KCNN_GEMM set the initial values.  Returns nonzero for
 * an unknown name or value. */
int kcnn_set_kernel_family(const char *name, int value);
/* The current value of a selector, or -1 for an unknown name. */
int kcnn_get_kernel_family(const char *name);
/* C[m x n] = alpha * op(A) op(B) + beta * C on row-major fp32 matrices,
 * exactly CuMatrixBase::AddMatMat(alpha, A, transA, B, transB, beta) with
 * op(X) = X^T when trans_x (cu-matrix.h, upstream Kaldi). */
int kcnn_gemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
              const float *a, int lda, const float *b, int ldb, float beta,
              float *c, int ldc);
/* The bf16 plane form of an fp32 matrix (kaldi-lite/cu-gemm-x6.hip): x =
 * h + m + l exactly, the three bf16 planes [rows x cols] at dst, dst + ps,
 * dst + 2 ps (pitch ldp elements). */
int kcnn_split_planes(const float *src, int rows, int cols, int ld, uint16_t *dst, int ldp,
                      int64_t ps);
/* kcnn_gemm from plane-split operands (a, b as made by kcnn_split_planes,
 * plane strides aps, bps): the six-product bf16 MFMA kernel with no split
 * work in it.  Needs k % 32 == 0, lda / ldb / plane strides % 8 == 0 and,
 * on a row-contiguous operand (A^T or B), its row count % 8 == 0. */
int kcnn_gemm_planes(int trans_a, int trans_b, int m, int n, int k, float alpha,
                     const uint16_t *a, int lda, int64_t aps, const uint16_t *b, int ldb,
                     int64_t bps, float beta, float *c, int ldc);
/* Writes the per-function hipEvent profile (CuDevice::PrintProfile). */
int kcnn_profile_string(char *buf, size_t len);
/* Drops every accumulated and pending profile entry (CuDevice::ResetProfile). */
int kcnn_reset_profile(void);
void kcnn_set_randn_seed(uint64_t seed);
/* Host-side self test of the FastDiv helper; no GPU needed. */
int kcnn_selftest_fastdiv(void);

/* ---- CuMatrixBase methods (cu-matrix.h:451-480) ---------------------------- */
int kcnn_mat_conv2d(const float *in, MatrixDim in_dim, const float *kernel,
                    MatrixDim kernel_dim, int in_height, int in_width,
                    int in_channel, int kernel_height, int kernel_width,
                    int group, float *out, MatrixDim out_dim, int concat);
int kcnn_mat_add_mat_rep_vec(float *m, MatrixDim dim, const float *vec,
                             int vec_dim, int rep);
int kcnn_mat_flip_mat(const float *m, MatrixDim dim, int kernel_height,
                      int kernel_width, int in_channel, int group, float *flip,
                      MatrixDim flip_dim);
int kcnn_mat_padding_zero(const float *m, MatrixDim dim, int orig_height,
                          int orig_width, int orig_channel, int kernel_height,
                          int kernel_width, float *padmat, MatrixDim pad_dim);
int kcnn_mat_tp_block(const float *m, MatrixDim dim, int in_channel,
                      int block_size, float *out, MatrixDim out_dim);
int kcnn_mat_tp_inside_block(const float *m, MatrixDim dim, int group,
                             int block_size, float *out, MatrixDim out_dim);
int kcnn_mat_mod_permute_row(const float *m, MatrixDim dim, int in_channel,
                             int block_size, float *out, MatrixDim out_dim);
/* CuMatrixBase::ModPermuteChannel (conv2D.cc:685-727); comp is written when
 * from_comp_to_container == 0. */
int kcnn_mat_mod_permute_channel(float *comp, MatrixDim dim, int comp_idx,
                                 int num_component, int in_height, int in_width,
                                 float *container, MatrixDim container_dim,
                                 int from_comp_to_container);
int kcnn_mat_maxpool_prop(const float *in, MatrixDim in_dim, int in_height,
                          int in_width, int pool_height_dim,
                          int pool_width_dim, int pool_channel_dim,
                          int overlap, int overlap2D, float *out,
                          MatrixDim out_dim);
int kcnn_mat_maxpool_backprop(const float *in_value, MatrixDim in_dim,
                              const float *out_value, MatrixDim ov_dim,
                              const float *out_deriv, MatrixDim od_dim,
                              float *in_deriv, MatrixDim id_dim, int in_height,
                              int in_width, int pool_height_dim,
                              int pool_width_dim, int pool_channel_dim,
                              int overlap, int overlap2D);

/* ---- components ------------------------------------------------------------ */
typedef struct kcnn_component kcnn_component;

/* Component::NewFromString, e.g. "ConvolutionComponent in-height=40 ...". */
kcnn_component *kcnn_component_new_from_string(const char *initializer_line);
/* Component::ReadNew from a Kaldi stream file written by kcnn_component_write
 * (binary files start with the "\0B" header). */
kcnn_component *kcnn_component_read(const char *path);
int kcnn_component_write(const kcnn_component *c, const char *path, int binary);
kcnn_component *kcnn_component_copy(const kcnn_component *c);
void kcnn_component_free(kcnn_component *c);
int kcnn_component_type(const kcnn_component *c, char *buf, size_t len);
int kcnn_component_info(const kcnn_component *c, char *buf, size_t len);
int kcnn_component_input_dim(const kcnn_component *c);
int kcnn_component_output_dim(const kcnn_component *c);
/* Component::Context() (reference nnet-component.h:186-188): the frame
 * offsets the component reads per output frame -- {0} except SpliceComponent
 * (its left..right context).  Writes up to max_len offsets, returns the count
 * (-1 on error).  For propagate/backprop the input chunk is the output chunk
 * widened by this context: in_rows/num_chunks = out_rows/num_chunks +
 * back - front. */
int kcnn_component_context(const kcnn_component *c, int *offsets, int max_len);
/* NonlinearComponent::ValueSum()/DerivSum()/Count() (reference
 * nnet-component.h:377-379; accumulated by UpdateStats in Backprop when
 * to_update is set): copies up to max_len fp64 values to HOST arrays, *len =
 * their length (0 before the first update). */
int kcnn_component_nonlinear_stats(const kcnn_component *c, double *value_sum,
                                   double *deriv_sum, int max_len, int *len,
                                   double *count);
int kcnn_component_backprop_needs_input(const kcnn_component *c);
int kcnn_component_backprop_needs_output(const kcnn_component *c);
/* Component::Propagate(ChunkInfo(in_dim.cols, num_chunks, 0, rows/num_chunks-1),
 * ..., in, out). */
int kcnn_component_propagate(const kcnn_component *c, const float *in,
                             MatrixDim in_dim, float *out, MatrixDim out_dim,
                             int num_chunks);
/* Component::Backprop(..., to_update = update ? this : NULL, in_deriv);
 * in_deriv may be NULL to skip the data gradient. */
int kcnn_component_backprop(kcnn_component *c, const float *in_value,
                            MatrixDim in_dim, const float *out_value,
                            MatrixDim ov_dim, const float *out_deriv,
                            MatrixDim od_dim, float *in_deriv,
                            MatrixDim id_dim, int num_chunks, int update);
/* Parameter access.  which: 0 = linear params, 1 = bias (as a 1 x N matrix),
 * 2 = prev_grad_ (momentum buffer).  Sizes via kcnn_component_param_dim. */
int kcnn_component_param_dim(const kcnn_component *c, int which, int *rows,
                             int *cols);
int kcnn_component_get_param(const kcnn_component *c, int which, float *dst,
                             MatrixDim dst_dim);
int kcnn_component_set_param(kcnn_component *c, int which, const float *src,
                             MatrixDim src_dim);
float kcnn_component_learning_rate(const kcnn_component *c);
int kcnn_component_set_learning_rate(kcnn_component *c, float lr);
/* UpdatableComponent::DotProduct / SetZero / Scale / Add / PerturbParams. */
int kcnn_component_dot_product(const kcnn_component *a, const kcnn_component *b,
                               float *out);
int kcnn_component_set_zero(kcnn_component *c, int treat_as_gradient);
int kcnn_component_scale(kcnn_component *c, float scale);
int kcnn_component_add(kcnn_component *c, float alpha,
                       const kcnn_component *other);
int kcnn_component_perturb_params(kcnn_component *c, float stddev);
/* Data-parallel split of Update: flat gradient [linear | bias] (floats). */
int kcnn_component_num_gradient_params(const kcnn_component *c);
int kcnn_component_compute_gradient(const kcnn_component *c,
                                    const float *in_value, MatrixDim in_dim,
                                    const float *out_deriv, MatrixDim od_dim,
                                    float *grad);
int kcnn_component_apply_gradient(kcnn_component *c, const float *grad,
                                  int num_sample);
/* Backprop without update (in_deriv nullable: no data gradient) AND
 * ComputeGradient in one call; ConvolutionComponent runs both from a single
 * pass over out_deriv (hipF_conv2d_backward).  in_deriv must be preallocated
 * [rows x InputDim]. */
int kcnn_component_backprop_gradient(const kcnn_component *c,
                                     const float *in_value, MatrixDim in_dim,
                                     const float *out_deriv, MatrixDim od_dim,
                                     float *in_deriv, MatrixDim id_dim,
                                     float *grad);
/* ConvolutionComponent only: 1 if Backprop's reference branch is
 * "flip kernel" (nnet-component-nnet0.cc:489-497). */
int kcnn_component_conv_flip_branch(const kcnn_component *c);

/* ---- component stack (NnetUpdater-style) -------------------------------- */
typedef struct kcnn_nnet kcnn_nnet;
/* One component initializer line per '\n'-separated line of `config`. */
kcnn_nnet *kcnn_nnet_new(const char *config);
void kcnn_nnet_free(kcnn_nnet *n);
int kcnn_nnet_num_components(const kcnn_nnet *n);
kcnn_component *kcnn_nnet_component(kcnn_nnet *n, int i);  /* borrowed */
/* Forward over all components; keeps every layer's output for Backprop. */
int kcnn_nnet_propagate(kcnn_nnet *n, const float *in, MatrixDim in_dim);
/* Device pointer + dims of layer i's output (i = -1: the input copy). */
int kcnn_nnet_output(const kcnn_nnet *n, int i, const float **data,
                     MatrixDim *dim);
/* Device pointer + dims of d(input_i) left by the last backprop of
 * component i (rows = 0 before one ran, or when it was skipped). */
int kcnn_nnet_input_deriv(const kcnn_nnet *n, int i, const float **data,
                          MatrixDim *dim);
/* Backprop of component i given d(output_i) = the buffer filled by the
 * previous call (or `out_deriv` for the last component).  mode 0: reference
 * (update in place); 1: write the gradient into grad (device, length
 * kcnn_component_num_gradient_params) without updating; 2: data gradient
 * only; 3: the gradient only, for an updatable component that is not half
 * of a fused Conv -> Maxpool pair (a mode 2 call then adds its data
 * gradient; data parallelism starts the gradient's all-reduce in between).
 * The data gradient of component 0 is skipped when skip_first_dx. */
int kcnn_nnet_backprop_component(kcnn_nnet *n, int i, const float *out_deriv,
                                 MatrixDim od_dim, int mode, float *grad,
                                 int skip_first_dx);
/* Full backward pass, last component to first, mode 0 (reference). */
/* An affine layer (FullyConnected / Affine) in data-parallel training: its
 * parameter gradient into grad (mode 3), then between(ctx) -- where the caller
 * starts the gradient's all-reduce -- then its input derivative (mode 2),
 * unless i == 0 and skip_first_dx.  The same results as the mode 3 and mode 2
 * calls; both GEMMs' operand statistics come from one launch set. */
int kcnn_nnet_backprop_split(kcnn_nnet *n, int i, const float *out_deriv, MatrixDim od_dim,
                             float *grad, int skip_first_dx, void (*between)(void *),
                             void *ctx);
int kcnn_nnet_backprop(kcnn_nnet *n, const float *out_deriv, MatrixDim od_dim);

#ifdef __cplusplus
}
#endif
#endif /* KCNN_KCNN_H_ */
