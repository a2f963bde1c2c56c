// nnet2/nnet-kernels.h -- HIP launchers of the upstream nnet2 components on
// either side of the CNN path: RectifiedLinearComponent
// and SpliceComponent.  Internal to libkcnn.so (the components are the
// boundary); plain pointers + MatrixDim + stream like cnsl-hip-kernels.h.
#ifndef KCNN_NNET2_NNET_KERNELS_H_
#define KCNN_NNET2_NNET_KERNELS_H_

#include <stddef.h>

#include "cnsl-hip-kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RectifiedLinearComponent::Propagate (reference nnet-component.cc:799-806):
 * out = in, then ApplyFloor(0): x < 0 -> 0 (NaN and -0 stay). */
int kn_relu_prop(const float *in, MatrixDim in_dim, float *out, MatrixDim out_dim,
                 kcnn_stream_t st);

/* RectifiedLinearComponent::Backprop (:808-827): in_deriv = Heaviside(out_value)
 * * out_deriv (a product, so 0 * inf = NaN as in the reference).  With stats
 * != NULL also UpdateStats (:337-363): column sums (fp32, fixed order) of
 * out_value and of Heaviside(out_value) added to the fp64 value_sum/deriv_sum.
 * ws: kn_relu_stats_ws(out_dim) bytes. */
size_t kn_relu_stats_ws(MatrixDim dim);
int kn_relu_backprop(const float *out_value, MatrixDim ov_dim, const float *out_deriv,
                     MatrixDim od_dim, float *in_deriv, MatrixDim id_dim,
                     double *value_sum, double *deriv_sum, void *ws, kcnn_stream_t st);

/* SpliceComponent (:2638-2819) for contiguous chunk offsets: out row
 * (chunk, oi) takes, for context slot c, input row chunk*in_cs +
 * (out_first + oi + context[c] - in_first); the const_dim tail copies input
 * row chunk*in_cs + oi.  Backprop is the gather form of the reference's
 * CopyRows/AddMat sequence: in_deriv row r sums, over c in order, the out_deriv
 * block of the output row that read it (0 if none). */
#define KN_SPLICE_MAX_CONTEXT 64
/* Non-contiguous chunk offsets (a gapped context deeper in a stack): table
 * = 1 and in_index[c * out_cs + oi] is the in-chunk input row that splice
 * block c of output row oi reads (ChunkInfo::GetIndex of out offset oi +
 * context[c]); num_splice * out_cs <= KN_SPLICE_MAX_TAB.  table = 0: the
 * contiguous form, in row = out_first + oi + context[c] - in_first. */
#define KN_SPLICE_MAX_TAB 1024
typedef struct {
  int num_chunks, in_cs, out_cs, in_first, out_first;
  int dim, const_dim, num_splice;
  int context[KN_SPLICE_MAX_CONTEXT];
  int table;
  short in_index[KN_SPLICE_MAX_TAB];
} kn_splice_geom;
int kn_splice_prop(const float *in, MatrixDim in_dim, float *out, MatrixDim out_dim,
                   kn_splice_geom geom, kcnn_stream_t st);
int kn_splice_backprop(const float *out_deriv, MatrixDim od_dim, float *in_deriv,
                       MatrixDim id_dim, kn_splice_geom geom, kcnn_stream_t st);

/* fp64 stat vectors of NonlinearComponent (Scale/Add/UpdateStats):
 * y = beta * y + alpha * x  (x may be NULL: y = beta * y). */
int kn_dvec_update(double *y, const double *x, double alpha, double beta, int n,
                   kcnn_stream_t st);

#ifdef __cplusplus
}
#endif
#endif
