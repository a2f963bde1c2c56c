/*
 * oracle/kcnn_oracle.h -- CPU restatement of the kaldi-cnn nnet2 CNN hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the *checker*: it may be loaded
 * by tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py,
 * never by the product (libkcnn.so has no CPU fallback and never links this).
 *
 * PARITY UNPINNED: the reference ships no golden vectors, known-answer tests
 * or fixtures for this path, and it cannot be built or run here (it needs
 * upstream Kaldi rev 4510 + CUDA).  This oracle is pinned
 * instead by (i) hand-derived known-answer tests, (ii) an independent
 * PyTorch-CPU float64 formulation of every op, and (iii) the reference's own
 * finite-difference gradient-check pattern (nnet-conv-test.cc:60-210);
 * see tests/test_oracle_cpu.py and DESIGN.md.
 *
 * Every function follows the CPU ("else") branch of the reference method it
 * names, loop order and index arithmetic included; file:line citations are
 * relative to the reference tree (src/...).
 *
 * Matrices are row-major with a pitch, exactly like Kaldi's CuMatrixBase:
 * element (r, c) lives at data[r * stride + c] (cudamatrix/cu-matrix.h:403-417).
 */
#ifndef KCNN_ORACLE_H_
#define KCNN_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  float *data;
  int32_t rows, cols, stride;
} orc_mat;

/* Accumulation precision of every reduction (GEMM inner products, row sums).
 *   0 : float, sequential in k (the reference's fp32 BLAS stand-in)
 *   1 : double accumulation, one rounding at the end ("fp64 truth")
 *   2 : double accumulation of |a|*|b| -- returns the error-bound scale
 *       S = sum_k |a_k b_k| for linear ops (used by the parity tests).        */
void orc_set_accum_mode(int mode);
int orc_get_accum_mode(void);
/* OpenMP threads used by the GEMM / im2col loops (1 = scalar reference). */
void orc_set_num_threads(int n);
/* Mode-0 GEMMs through a CBLAS sgemm (OpenBLAS's 64-bit-int build, dlopen'ed
 * from `path`; NULL goes back to the loops).  For the CPU-baseline timing. */
int orc_use_blas(const char *path);
int orc_blas_active(void);
int orc_num_threads(void);
const char *orc_last_error(void);

/* ---- BLAS stand-in (Kaldi CuMatrixBase::AddMatMat, upstream) ----------------
 * C = alpha * op(A) op(B) + beta * C, row-major, transA/transB in {0,1}.     */
int orc_gemm(float alpha, const orc_mat *A, int transA, const orc_mat *B,
             int transB, float beta, orc_mat *C);

/* ---- CuMatrixBase extensions (cudamatrix/cu-matrix.h:451-482) ---------------
 * Each returns 0 on success, -1 on a KALDI_ASSERT-equivalent violation.     */

/* conv2D.cc:43-201 (CPU branches :114-134, :158-167, :187-200). */
int orc_conv2d(const orc_mat *in, const orc_mat *kernel, int in_height,
               int in_width, int in_channel, int kernel_height,
               int kernel_width, int group, orc_mat *out, int concat);
/* conv2D.cc:213-242 (CPU :231-240). */
int orc_add_mat_rep_vec(orc_mat *m, const float *vec, int vec_dim, int rep);
/* conv2D.cc:244-287 (CPU :269-284). `flip` must be pre-sized. */
int orc_flip_mat(const orc_mat *m, int kernel_height, int kernel_width,
                 int in_channel, int group, orc_mat *flip);
/* conv2D.cc:289-344 (CPU :316-342). `padmat` must be pre-sized. */
int orc_padding_zero(const orc_mat *m, int orig_height, int orig_width,
                     int orig_channel, int kernel_height, int kernel_width,
                     orc_mat *padmat);
/* conv2D.cc:348-386 (CPU :375-385). */
int orc_tp_block(const orc_mat *m, int in_channel, int block_size,
                 orc_mat *out);
/* conv2D.cc:388-426 (CPU :415-425). */
int orc_tp_inside_block(const orc_mat *m, int group, int block_size,
                        orc_mat *out);
/* conv2D.cc:429-463 (CPU :452-462). */
int orc_mod_permute_row(const orc_mat *m, int in_channel, int block_size,
                        orc_mat *out);
/* conv2D.cc:706-725 */
int orc_mod_permute_channel(orc_mat *comp, int comp_idx, int num_component,
                            int in_height, int in_width, orc_mat *container,
                            int from_comp_to_container);
/* conv2D.cc:465-559; non-overlap CPU :531-557, overlap :541-542,
 * overlap2D follows the GPU kernel cnsl-cu-kernels.cu:405-452 (the CPU
 * branch :503-528 does not compile as committed). */
int orc_maxpool_prop(const orc_mat *in, int in_height, int in_width,
                     int pool_height_dim, int pool_width_dim,
                     int pool_channel_dim, int overlap, int overlap2D,
                     orc_mat *out);
/* conv2D.cc:565-684 (CPU :639-681): in_deriv is zeroed (component :889)
 * and every window input equal to the pooled max receives d_out.  For
 * finite d_out the CPU "+= d_out*mask" equals the GPU assignment
 * (cnsl-cu-kernels.cu:302-303) because non-overlapping windows are
 * disjoint; overlapping modes accumulate (+=), in window order. */
int orc_maxpool_backprop(const orc_mat *in_value, const orc_mat *out_value,
                         const orc_mat *out_deriv, orc_mat *in_deriv,
                         int in_height, int in_width, int pool_height_dim,
                         int pool_width_dim, int pool_channel_dim, int overlap,
                         int overlap2D);

/* ---- nnet0 components (nnet0/nnet-component-nnet0.cc) ------------------- */
typedef struct {
  int in_height, in_width, in_channel;
  int in_pad_height, in_pad_width;
  int kernel_height, kernel_width, stride, group;
  int out_height, out_width;
  float learning_rate, weight_decay, momentum;
  orc_mat W;        /* linear_params_ [kh*kw*C x G] */
  float *b;         /* bias_params_   [G]           */
  orc_mat prev;     /* prev_grad_     [kh*kw*C x G] */
} orc_conv;

/* ConvolutionComponent::Propagate :423-446. */
int orc_conv_propagate(const orc_conv *c, const orc_mat *in, orc_mat *out);
/* ConvolutionComponent::Backprop :461-544: in_deriv (pre-sized), then if
 * do_update, Update(in_value, out_deriv) :738-777 on *c. */
int orc_conv_backprop(orc_conv *c, const orc_mat *in_value,
                      const orc_mat *out_deriv, orc_mat *in_deriv,
                      int do_update);
/* The branch ConvolutionComponent::Backprop takes (:489-497): 1 = flip
 * kernel (pad out_deriv), 0 = pad kernel. */
int orc_conv_flip_branch(const orc_conv *c);
/* Update :738-777 split in two so data-parallel tests can sum gradients:
 * linear_params_grad (after ModPermuteRow, :765) and the bias row sum. */
int orc_conv_gradient(const orc_conv *c, const orc_mat *in_value,
                      const orc_mat *out_deriv, orc_mat *grad_W,
                      float *grad_b);
int orc_conv_apply(orc_conv *c, const orc_mat *grad_W, const float *grad_b,
                   int num_sample);

/* MaxpoolComponent::Propagate/Backprop :869-892. */
typedef struct {
  int in_height, in_width, in_channel;
  int pool_height_dim, pool_width_dim, pool_channel_dim;
  int overlap, overlap2D;
} orc_pool;
int orc_pool_output_dim(const orc_pool *p);  /* InitFromString :835-847 */

/* FullyConnectedComponent = AffineComponent::Propagate/Backprop
 * (nnet2/nnet-component.cc:1216-1258) + UpdateSimple
 * (nnet-component-nnet0.cc:1133-1150). */
typedef struct {
  int input_dim, output_dim;
  float learning_rate, weight_decay, momentum;
  orc_mat W;        /* [output_dim x input_dim] */
  float *b;         /* [output_dim] */
  orc_mat prev;     /* [output_dim x input_dim] */
} orc_fc;
int orc_fc_propagate(const orc_fc *f, const orc_mat *in, orc_mat *out);
int orc_fc_backprop(orc_fc *f, const orc_mat *in_value,
                    const orc_mat *out_deriv, orc_mat *in_deriv,
                    int do_update);
int orc_fc_gradient(const orc_fc *f, const orc_mat *in_value,
                    const orc_mat *out_deriv, orc_mat *grad_W, float *grad_b);
int orc_fc_apply(orc_fc *f, const orc_mat *grad_W, const float *grad_b,
                 int num_sample);

/* ---- upstream nnet2 components either side of the path ---- */
/* RectifiedLinearComponent::Propagate (nnet2/nnet-component.cc:799-806):
 * CopyFromMat + ApplyFloor(0) (`if (x < 0) x = 0`). */
int orc_relu_propagate(const orc_mat *in, orc_mat *out);
/* ::Backprop (:808-827): in_deriv = Heaviside(out_value) (x > 0 ? 1 : 0),
 * UpdateStats (:337-363) when value_sum != NULL -- fp32 column sums of
 * out_value and of the Heaviside matrix (row order), added to the fp64
 * stats, count += rows -- then MulElements(out_deriv). */
int orc_relu_backprop(const orc_mat *out_value, const orc_mat *out_deriv,
                      orc_mat *in_deriv, double *value_sum, double *deriv_sum,
                      double *count);
/* SpliceComponent::Propagate/Backprop (:2638-2819) for chunk offsets
 * [in_first, in_first + in_cs) -> [out_first, out_first + out_cs): the
 * reference's index vectors and CopyRows / AddMat sequence, literally. */
/* SpliceComponent with the chunk offsets as explicit ascending lists (the
 * upstream ChunkInfo offsets_ vector: gapped contexts) */
int orc_splice_propagate_offsets(const orc_mat *in, orc_mat *out, int num_chunks,
                                 const int *in_offsets, int in_cs, const int *out_offsets,
                                 int out_cs, const int *context, int num_splice,
                                 int const_dim);
int orc_splice_backprop_offsets(const orc_mat *out_deriv, orc_mat *in_deriv, int num_chunks,
                                const int *in_offsets, int in_cs, const int *out_offsets,
                                int out_cs, const int *context, int num_splice,
                                int const_dim);
int orc_splice_propagate(const orc_mat *in, orc_mat *out, int num_chunks, int in_first,
                         int in_cs, int out_first, int out_cs, const int *context,
                         int num_splice, int const_dim);
int orc_splice_backprop(const orc_mat *out_deriv, orc_mat *in_deriv, int num_chunks,
                        int in_first, int in_cs, int out_first, int out_cs,
                        const int *context, int num_splice, int const_dim);

#ifdef __cplusplus
}
#endif
#endif /* KCNN_ORACLE_H_ */
