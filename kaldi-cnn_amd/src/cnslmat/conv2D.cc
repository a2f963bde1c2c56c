// cnslmat/conv2D.cc -- bodies of the CuMatrixBase extensions the reference
// grafted onto Kaldi (declarations: reference cudamatrix/cu-matrix.h:446-482,
// bodies: reference src/cnslmat/conv2D.cc).  Signatures, assertions, resize
// behaviour and results follow the reference; the work goes to the gfx950
// kernels behind include/cnsl-hip-kernels.h.  There is no CPU branch: the
// reference's `else` branches are restated, as a test checker only, in
// oracle/kcnn_oracle.c.
#include <algorithm>

#include "cnsl-hip-kernels.h"
#include "conv-update.h"
#include "pool-stats.h"
#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/cu-matrix.h"

// kcnn_pool_defer_request's request of this thread (pool-stats.h)
static thread_local PoolColDeferred *t_pool_defer = nullptr;
PoolColDeferred *kcnn_pool_defer_request(PoolColDeferred *d) {
  PoolColDeferred *prev = t_pool_defer;
  t_pool_defer = d;
  return prev;
}
PoolColDeferred *kcnn_pool_defer_current() { return t_pool_defer; }
static thread_local ConvUpdateEpi *t_conv_update = nullptr;
ConvUpdateEpi *kcnn_conv_update_request(ConvUpdateEpi *u) {
  ConvUpdateEpi *prev = t_conv_update;
  t_conv_update = u;
  return prev;
}
ConvUpdateEpi *kcnn_conv_update_current() { return t_conv_update; }

namespace kaldi {

namespace {
inline kcnn_stream_t S() {
  return reinterpret_cast<kcnn_stream_t>(CuDevice::Instantiate().Stream());
}
}  // namespace

// conv2D.cc:43-201.  One implicit-GEMM launch (no im2col buffer, no split
// loop, no cudaMemGetInfo host sync).
template <typename Real>
void CuMatrixBase<Real>::Conv2D(const CuMatrixBase<Real> &kernel,
                                int32 in_height, int32 in_width,
                                int32 in_channel, int32 kernel_height,
                                int32 kernel_width, int32 group,
                                CuMatrixBase<Real> *out, bool concat) const {
  KALDI_ASSERT(NumCols() == in_height * in_width * in_channel);     // :55
  KALDI_ASSERT(kernel.NumCols() == group);                          // :56
  KALDI_ASSERT(kernel.NumRows() == kernel_height * kernel_width * in_channel);
  KALDI_ASSERT(out != NULL);                                        // :62
  const int32 out_height = in_height - kernel_height + 1,
              out_width = in_width - kernel_width + 1;              // :59
  KALDI_ASSERT(out_height > 0 && out_width > 0);
  if (concat)
    KALDI_ASSERT(out->NumRows() == NumRows() &&
                 out->NumCols() == out_height * out_width * group);
  else
    KALDI_ASSERT(out->NumRows() == out_height * out_width * NumRows() &&
                 out->NumCols() == group);
  CuProfileScope prof("Conv2D");
  const size_t ws_bytes = hipF_conv2d_workspace_bytes(
      Dim(), in_height, in_width, in_channel, 0, 0, kernel_height,
      kernel_width, group);
  CuScratch ws_s(ws_bytes);
  void *ws = ws_s.p;
  CNSL_SAFE_CALL(hipF_conv2d(data_, Dim(), in_height, in_width, in_channel, 0,
                             0, kernel.Data(), kernel.Dim(), kernel_height,
                             kernel_width, group, nullptr, out->Data(),
                             out->Dim(), concat ? 1 : 0, ws, ws_bytes, S()));
}

// conv2D.cc:213-242.
template <typename Real>
void CuMatrixBase<Real>::AddMatRepVec(const CuVectorBase<Real> &vec,
                                      int32 rep) const {
  KALDI_ASSERT(vec.Dim() * rep == this->NumCols());                 // :216
  CuProfileScope prof("AddMatRepVec");
  CNSL_SAFE_CALL(hipF_add_mat_rep_vec(vec.Data(), rep, data_, Dim(), S()));
}

// conv2D.cc:244-287.
template <typename Real>
void CuMatrixBase<Real>::FlipMat(int32 kernel_height, int32 kernel_width,
                                 int32 in_channel, int32 group,
                                 CuMatrix<Real> *flip) const {
  KALDI_ASSERT(NumRows() == (kernel_height * kernel_width * in_channel));
  KALDI_ASSERT(flip != NULL);
  if ((flip->NumRows() != (kernel_height * kernel_width * group)) ||
      (flip->NumCols() != in_channel))                              // :251
    flip->Resize((kernel_height * kernel_width * group), in_channel, kSetZero);
  KALDI_ASSERT(NumCols() >= group);
  CuProfileScope prof("FlipMat");
  CNSL_SAFE_CALL(hipF_flip_mat(data_, Dim(), kernel_height, kernel_width, group,
                               flip->Data(), flip->Dim(), S()));
}

// conv2D.cc:289-344.
template <typename Real>
void CuMatrixBase<Real>::PaddingZero(int32 orig_height, int32 orig_width,
                                     int32 orig_channel, int32 kernel_height,
                                     int32 kernel_width,
                                     CuMatrix<Real> *padmat) const {
  KALDI_ASSERT(NumCols() == (orig_height * orig_width * orig_channel));
  KALDI_ASSERT(padmat != NULL);
  const int32 padmat_height = orig_height + 2 * (kernel_height - 1),
              padmat_width = orig_width + 2 * (kernel_width - 1);   // :295
  if (padmat->NumRows() != NumRows() ||
      padmat->NumCols() != padmat_height * padmat_width * orig_channel)
    padmat->Resize(NumRows(), padmat_height * padmat_width * orig_channel,
                   kSetZero);                                       // :299
  CuProfileScope prof("PaddingZero");
  CNSL_SAFE_CALL(hipF_pad_zero(data_, Dim(), orig_height, orig_width,
                               kernel_height, kernel_width, padmat->Data(),
                               padmat->Dim(), S()));
}

// conv2D.cc:348-386.
template <typename Real>
void CuMatrixBase<Real>::TpBlock(int32 in_channel, int32 block_size,
                                 CuMatrix<Real> *out) const {
  KALDI_ASSERT(this->NumCols() == block_size * in_channel);         // :353
  KALDI_ASSERT(out != NULL);
  if ((out->NumRows() != in_channel) ||
      (out->NumCols() != NumRows() * block_size))                   // :357
    out->Resize(in_channel, NumRows() * block_size, kSetZero);
  CuProfileScope prof("TpBlock");
  CNSL_SAFE_CALL(hipF_tp_block(data_, Dim(), out->Data(), out->Dim(),
                               block_size, S()));
}

// conv2D.cc:388-426.
template <typename Real>
void CuMatrixBase<Real>::TpInsideBlock(int32 group, int32 block_size,
                                       CuMatrix<Real> *out) const {
  KALDI_ASSERT(this->NumCols() == block_size * group);              // :393
  KALDI_ASSERT(out != NULL);
  if ((out->NumRows() != block_size * NumRows()) || (out->NumCols() != group))
    out->Resize(block_size * NumRows(), group, kSetZero);           // :398
  CuProfileScope prof("TpInsideBlock");
  CNSL_SAFE_CALL(hipF_tp_inside_block(data_, Dim(), out->Data(), out->Dim(),
                                      block_size, S()));
}

// conv2D.cc:429-463.
template <typename Real>
void CuMatrixBase<Real>::ModPermuteRow(int32 in_channel, int32 block_size,
                                       CuMatrix<Real> *out) const {
  KALDI_ASSERT(out != NULL);
  if ((out->NumRows() != NumRows()) || (out->NumCols() != NumCols()))
    out->Resize(NumRows(), NumCols(), kSetZero);                    // :435
  KALDI_ASSERT((int64)in_channel * block_size == NumRows());
  CuProfileScope prof("ModPermuteRow");
  CNSL_SAFE_CALL(hipF_mod_permute_row(data_, Dim(), out->Data(), out->Dim(),
                                      block_size, in_channel, S()));
}

// conv2D.cc:465-559.
template <typename Real>
void CuMatrixBase<Real>::Maxpool_prop(int32 in_height, int32 in_width,
                                      int32 pool_height_dim,
                                      int32 pool_width_dim,
                                      int32 pool_channel_dim, bool overlap,
                                      bool overlap2D,
                                      CuMatrixBase<Real> *out) const {
  KALDI_ASSERT(out != NULL);                                        // :468
  KALDI_ASSERT(out->NumRows() == NumRows());
  KALDI_ASSERT(pool_height_dim > 0 && pool_width_dim > 0 && pool_channel_dim > 0);
  CuProfileScope prof("Maxpool_prop");
  const int mode = overlap ? 1 : (overlap2D ? 2 : 0);               // :485-491
  CNSL_SAFE_CALL(hipF_maxpool_prop(data_, Dim(), out->Data(), out->Dim(),
                                   in_height, in_width, pool_height_dim,
                                   pool_width_dim, pool_channel_dim, mode,
                                   S()));
}

// conv2D.cc:565-684.  Routed elements only (reference kernel semantics);
// MaxpoolComponent::Backprop uses the fused zero+route form instead.
template <typename Real>
void CuMatrixBase<Real>::Maxpool_backprop(
    const CuMatrixBase<Real> &out_value, const CuMatrixBase<Real> &out_deriv,
    CuMatrix<Real> *in_deriv, int32 in_height, int32 in_width,
    int32 pool_height_dim, int32 pool_width_dim, int32 pool_channel_dim,
    bool overlap, bool overlap2D) const {
  KALDI_ASSERT(in_deriv != NULL);                                   // :570
  if ((in_deriv->NumRows() != NumRows()) || (in_deriv->NumCols() != NumCols()))
    in_deriv->Resize(NumRows(), NumCols(), kSetZero);               // :572
  KALDI_ASSERT(out_deriv.NumRows() == out_value.NumRows() &&
               out_deriv.NumCols() == out_value.NumCols() &&
               out_value.NumRows() == NumRows());
  if (overlap || overlap2D)
    KALDI_ASSERT(pool_height_dim == 1 && pool_width_dim == 1);      // :582, :585
  CuProfileScope prof("Maxpool_backprop");
  const int mode = overlap ? 1 : (overlap2D ? 2 : 0);
  CNSL_SAFE_CALL(hipF_maxpool_backprop(
      data_, Dim(), out_value.Data(), out_value.Dim(), out_deriv.Data(),
      out_deriv.Dim(), in_deriv->Data(), in_deriv->Dim(), in_height, in_width,
      pool_height_dim, pool_width_dim, pool_channel_dim, mode, 0, S()));
}

// conv2D.cc:685-727.  No resize: container is caller-sized (the reference
// only asserts it is non-NULL).
template <typename Real>
void CuMatrixBase<Real>::ModPermuteChannel(int32 comp_idx, int32 num_component,
                                           int32 in_height, int32 in_width,
                                           CuMatrixBase<Real> *container,
                                           bool fromCompToContainer) {
  KALDI_ASSERT(container != NULL);                                    // :688
  CuProfileScope prof("ModPermuteChannel");
  CNSL_SAFE_CALL(hipF_mod_permute_channels(
      data_, Dim(), container->Data(), container->Dim(), comp_idx,
      num_component, in_height, in_width, fromCompToContainer ? 1 : 0, S()));
}

// Member-wise explicit instantiation (the class itself is instantiated in
// kaldi-lite/cu-matrix.cc).
template void CuMatrixBase<float>::Conv2D(const CuMatrixBase<float> &, int32,
                                          int32, int32, int32, int32, int32,
                                          CuMatrixBase<float> *, bool) const;
template void CuMatrixBase<float>::AddMatRepVec(const CuVectorBase<float> &,
                                                int32) const;
template void CuMatrixBase<float>::FlipMat(int32, int32, int32, int32,
                                           CuMatrix<float> *) const;
template void CuMatrixBase<float>::PaddingZero(int32, int32, int32, int32,
                                               int32, CuMatrix<float> *) const;
template void CuMatrixBase<float>::TpBlock(int32, int32, CuMatrix<float> *) const;
template void CuMatrixBase<float>::TpInsideBlock(int32, int32,
                                                 CuMatrix<float> *) const;
template void CuMatrixBase<float>::ModPermuteRow(int32, int32,
                                                 CuMatrix<float> *) const;
template void CuMatrixBase<float>::ModPermuteChannel(int32, int32, int32, int32,
                                                     CuMatrixBase<float> *, bool);
template void CuMatrixBase<float>::Maxpool_prop(int32, int32, int32, int32,
                                                int32, bool, bool,
                                                CuMatrixBase<float> *) const;
template void CuMatrixBase<float>::Maxpool_backprop(
    const CuMatrixBase<float> &, const CuMatrixBase<float> &,
    CuMatrix<float> *, int32, int32, int32, int32, int32, bool, bool) const;

}  // namespace kaldi
