// nnet0/nnet-component-nnet0.cc -- the CNN components (reference
// src/nnet0/nnet-component-nnet0.cc).  Citations ":N" are lines of that file.
#include "nnet-component-nnet0.h"

#include <math.h>
#include <stdlib.h>

#include <sstream>

#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/kaldi-io.h"
#include "../nnet2/parse-from-string.h"
#include "cnsl-hip-kernels.h"
#include "cnslmat/conv-update.h"

namespace cnsl {
namespace nnet0 {

namespace {
bool g_literal = getenv("KCNN_LITERAL") != nullptr && atoi(getenv("KCNN_LITERAL")) != 0;
inline kcnn_stream_t S() {
  return reinterpret_cast<kcnn_stream_t>(CuDevice::Instantiate().Stream());
}
::MatrixDim Dense(int32 rows, int32 cols) {
  ::MatrixDim d;
  d.rows = rows; d.cols = cols; d.stride = cols;
  return d;
}
using Scratch = CuScratch;  // kaldi-lite/cu-device.h
}  // namespace

void SetLiteralPath(bool literal) { g_literal = literal; }
bool LiteralPath() { return g_literal; }

// ===========================================================================
// ConvolutionComponent
// ===========================================================================
ConvolutionComponent::ConvolutionComponent(const ConvolutionComponent &component)
    : UpdatableComponent(component),
      linear_params_(component.linear_params_),
      bias_params_(component.bias_params_),
      is_gradient_(component.is_gradient_),
      in_height_(component.in_height_),
      in_width_(component.in_width_),
      in_channel_(component.in_channel_),
      in_pad_height_(component.in_pad_height_),
      in_pad_width_(component.in_pad_width_),
      kernel_height_(component.kernel_height_),
      kernel_width_(component.kernel_width_),
      stride_(component.stride_),
      group_(component.group_),
      out_height_(component.out_height_),
      out_width_(component.out_width_),
      weight_decay_(component.weight_decay_),
      momentum_(component.momentum_),
      prev_grad_(component.prev_grad_) {}  // B9: like Copy(), keep prev_grad_

ConvolutionComponent::ConvolutionComponent(
    const CuMatrixBase<BaseFloat> &linear_params,
    const CuVectorBase<BaseFloat> &bias_params, BaseFloat learning_rate,
    int32 in_height, int32 in_width, int32 in_channels, int32 in_pad_height,
    int32 in_pad_width, int32 kernel_height, int32 kernel_width, int32 stride,
    int32 group, int32 out_height, int32 out_width, BaseFloat weight_decay,
    BaseFloat momentum)
    : UpdatableComponent(learning_rate),
      linear_params_(linear_params),
      in_height_(in_height), in_width_(in_width), in_channel_(in_channels),
      in_pad_height_(in_pad_height), in_pad_width_(in_pad_width),
      kernel_height_(kernel_height), kernel_width_(kernel_width),
      stride_(stride), group_(group), out_height_(out_height),
      out_width_(out_width), weight_decay_(weight_decay), momentum_(momentum) {
  bias_params_ = bias_params;
  KALDI_ASSERT(linear_params.NumCols() == bias_params.Dim() &&
               bias_params.Dim() != 0);                            // :225
  is_gradient_ = false;
  prev_grad_.Resize(linear_params.NumRows(), linear_params.NumCols());
}

// :232-275
void ConvolutionComponent::Init(BaseFloat learning_rate, int32 in_height,
                                int32 in_width, int32 in_channels,
                                int32 in_pad_height, int32 in_pad_width,
                                int32 kernel_height, int32 kernel_width,
                                int32 stride, int32 group, int32 out_height,
                                int32 out_width, BaseFloat param_stddev,
                                BaseFloat bias_stddev, BaseFloat weight_decay,
                                BaseFloat momentum) {
  in_height_ = in_height; in_width_ = in_width; in_channel_ = in_channels;
  in_pad_height_ = in_pad_height; in_pad_width_ = in_pad_width;
  kernel_height_ = kernel_height; kernel_width_ = kernel_width;
  stride_ = stride; group_ = group;
  out_height_ = out_height; out_width_ = out_width;
  weight_decay_ = weight_decay; momentum_ = momentum;
  KALDI_ASSERT(in_pad_height_ >= 0);
  KALDI_ASSERT(in_pad_width_ >= 0);
  KALDI_ASSERT(stride == 1);  // B6: Conv2D is always stride 1 (conv2D.cc:59)
  KALDI_ASSERT(out_height_ == 1 + (in_height + (2 * in_pad_height) - kernel_height) / stride);
  KALDI_ASSERT(out_width_ == 1 + (in_width + (2 * in_pad_width) - kernel_width) / stride);
  KALDI_ASSERT(in_height > 0 && in_width > 0 && in_channels > 0 && group > 0);
  UpdatableComponent::Init(learning_rate);
  linear_params_.Resize(KernelDim(), group);
  bias_params_.Resize(group);
  prev_grad_.Resize(KernelDim(), group);
  KALDI_ASSERT(param_stddev >= 0.0);
  linear_params_.SetRandn();
  linear_params_.Scale(param_stddev);
  prev_grad_.SetZero();
  bias_params_.SetRandn();
  bias_params_.Scale(bias_stddev);
}

// :323-385, with the reference's quirks kept or rejected as SURVEY B4-B7 say.
void ConvolutionComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  bool ok = true;
  BaseFloat learning_rate = learning_rate_;
  BaseFloat weight_decay = weight_decay_, momentum = momentum_;
  std::string matrix_filename;
  int32 in_height = 0, in_width = 0, in_channel = 0, in_pad_height = 0,
        in_pad_width = 0, kernel_height = 0, kernel_width = 0, stride = 0,
        group = 0, out_height = 0, out_width = 0;
  // B5: the `ok = ok && ...` chain makes learning-rate mandatory.
  ok = ok && ParseFromString("learning-rate", &args, &learning_rate);
  ok = ok && ParseFromString("in-height", &args, &in_height);
  ok = ok && ParseFromString("in-width", &args, &in_width);
  ok = ok && ParseFromString("in-channel", &args, &in_channel);
  ParseFromString("in-pad-height", &args, &in_pad_height);
  ParseFromString("in-pad-width", &args, &in_pad_width);
  ok = ok && ParseFromString("kernel-height", &args, &kernel_height);
  ok = ok && ParseFromString("kernel-width", &args, &kernel_width);
  ok = ok && ParseFromString("stride", &args, &stride);
  ok = ok && ParseFromString("group", &args, &group);
  ok = ok && ParseFromString("out-height", &args, &out_height);
  ok = ok && ParseFromString("out-width", &args, &out_width);
  // (the reference would go on with uninitialised values here)
  if (!ok) KALDI_ERR << "Bad initializer " << orig_args;
  if (stride != 1)
    KALDI_ERR << "stride=" << stride << " is not supported: the reference "
              << "parses it but always convolves with stride 1 (SURVEY B6)";
  KALDI_ASSERT(out_height == 1 + (in_height + (2 * in_pad_height) - kernel_height) / stride &&
               "out_height_ == 1 + (in_height + (2*in_pad_height) - kernel_height) / stride ");
  KALDI_ASSERT(out_width == 1 + (in_width + (2 * in_pad_width) - kernel_width) / stride &&
               "out_width == 1 + (in_width + (2*in_pad_width) - kernel_width) / stride");
  KALDI_ASSERT(in_pad_height >= 0 && "in-pad-height should be positive");
  KALDI_ASSERT(in_pad_width >= 0 && "in-pad-width should be positive");
  if (ParseFromString("matrix", &args, &matrix_filename))
    KALDI_ERR << "matrix= initialisation is not supported: the reference's "
              << "version sizes the bias wrongly (SURVEY B7)";
  BaseFloat param_stddev = 1.0 / std::sqrt((double)(kernel_height * kernel_width)),
            bias_stddev = 1.0;
  ParseFromString("param-stddev", &args, &param_stddev);
  ParseFromString("bias-stddev", &args, &bias_stddev);
  Init(learning_rate, in_height, in_width, in_channel, in_pad_height,
       in_pad_width, kernel_height, kernel_width, stride, group, out_height,
       out_width, param_stddev, bias_stddev, weight_decay, momentum);
  // B4: parsed after Init, so the configured values never take effect.
  BaseFloat wd_cfg = weight_decay, mom_cfg = momentum;
  ParseFromString("weight-decay", &args, &wd_cfg);
  ParseFromString("momentum", &args, &mom_cfg);
  if (wd_cfg != weight_decay_ || mom_cfg != momentum_)
    KALDI_WARN << "ConvolutionComponent ignores weight-decay=" << wd_cfg
               << " momentum=" << mom_cfg << " (reference behaviour, SURVEY B4);"
               << " using " << weight_decay_ << " / " << momentum_;
  if (!args.empty())
    KALDI_ERR << "Could not process these elements in initializer: " << args;
}

// :387-421
std::string ConvolutionComponent::Info() const {
  std::stringstream stream;
  const double size = (double)linear_params_.NumRows() * linear_params_.NumCols();
  const double linear_stddev =
      std::sqrt(TraceMatMat(linear_params_, linear_params_, kTrans) / size);
  const double bias_stddev =
      std::sqrt(VecVec(bias_params_, bias_params_) / bias_params_.Dim());
  stream << Type() << ", input-dim=" << InputDim() << " ( in-height="
         << In_height() << ", in-width=" << In_width()
         << ", in-channels=" << In_channels() << "), output-dim=" << OutputDim()
         << " ( out-height=" << Out_height() << ", out-width=" << Out_width()
         << ", group-num=" << Group() << "), kernel-dim=" << KernelDim()
         << " ( kernel-height=" << Kernel_height()
         << ", kernel-width=" << Kernel_width()
         << "), ( padding-height=" << in_pad_height_
         << ", padding-width=" << in_pad_width_
         << "), linear-params-stddev=" << linear_stddev
         << ", bias-params-stddev=" << bias_stddev
         << ", learning-rate=" << LearningRate()
         << ", weight-decay=" << weight_decay_ << ", momentum=" << momentum_;
  return stream.str();
}

// :423-446.  Fused: one implicit-GEMM launch with virtual input padding
// (replaces PaddingZero :433) and the bias add of AddMatRepVec (:443) in its
// epilogue.
void ConvolutionComponent::Propagate(const ChunkInfo &in_info,
                                     const ChunkInfo &out_info,
                                     const CuMatrixBase<BaseFloat> &in,
                                     CuMatrixBase<BaseFloat> *out) const {
  (void)out_info;
  KALDI_ASSERT(in.NumCols() == InputDim());
  KALDI_ASSERT(out->NumRows() == in.NumRows() && out->NumCols() == OutputDim());
  if (LiteralPath()) { PropagateLiteral(in_info, in, out); return; }
  CuProfileScope prof("ConvolutionComponent::Propagate");
  const size_t ws_bytes = hipF_conv2d_workspace_bytes(
      in.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
      in_pad_width_, kernel_height_, kernel_width_, group_);
  Scratch ws_s(ws_bytes);
  void *ws = ws_s.p;
  CNSL_SAFE_CALL(hipF_conv2d(in.Data(), in.Dim(), in_height_, in_width_,
                             in_channel_, in_pad_height_, in_pad_width_,
                             linear_params_.Data(), linear_params_.Dim(),
                             kernel_height_, kernel_width_, group_,
                             bias_params_.Data(), out->Data(), out->Dim(), 1,
                             ws, ws_bytes, S()));
}

bool ConvolutionComponent::PropagateMaxpool(const CuMatrixBase<BaseFloat> &in,
                                            CuMatrixBase<BaseFloat> *out,
                                            const MaxpoolComponent &pool,
                                            CuMatrixBase<BaseFloat> *pool_out,
                                            unsigned char *mask,
                                            int32 mask_stride, bool store_out,
                                            PoolStatsOut *pool_stats) const {
  const int32 pc = pool.FusableChannelPool();
  int32 ph = 1, pw = 1, pc3 = 0;
  const bool win3 = pc == 0 && pool.FusableWindow3D(&ph, &pw, &pc3);
  if (LiteralPath() || (pc == 0 && !win3) || mask == NULL) return false;
  if (pool.In_height() != out_height_ || pool.In_width() != out_width_ ||
      pool.In_channels() != group_ || pool.InputDim() != OutputDim())
    return false;
  KALDI_ASSERT(in.NumCols() == InputDim());
  KALDI_ASSERT(out->NumRows() == in.NumRows() && out->NumCols() == OutputDim());
  KALDI_ASSERT(pool_out->NumRows() == in.NumRows() &&
               pool_out->NumCols() == pool.OutputDim());
  CuProfileScope prof("ConvolutionComponent::PropagateMaxpool");
  const int rc =
      win3 ? hipF_conv2d_maxpool3d(
                 in.Data(), in.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
                 in_pad_width_, linear_params_.Data(), linear_params_.Dim(), kernel_height_,
                 kernel_width_, group_, bias_params_.Data(), store_out ? out->Data() : NULL,
                 out->Dim(), pool_out->Data(), pool_out->Dim(), reinterpret_cast<unsigned short *>(mask),
                 mask_stride, ph, pw, pc3, S())
           : kcnn_conv2d_maxpool_stats(
                 in.Data(), in.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
                 in_pad_width_, linear_params_.Data(), linear_params_.Dim(), kernel_height_,
                 kernel_width_, group_, bias_params_.Data(), store_out ? out->Data() : NULL,
                 out->Dim(), pool_out->Data(), pool_out->Dim(), mask, mask_stride, pc, S(),
                 pool_stats);
  if (rc < 0) {
    prof.Cancel();  // declined: nothing launched
    return false;
  }
  CNSL_SAFE_CALL(rc);
  return true;
}

bool ConvolutionComponent::PropagateRelu(const CuMatrixBase<BaseFloat> &in,
                                         CuMatrixBase<BaseFloat> *relu_out) const {
  if (LiteralPath()) return false;
  KALDI_ASSERT(in.NumCols() == InputDim());
  KALDI_ASSERT(relu_out->NumRows() == in.NumRows() && relu_out->NumCols() == OutputDim());
  int rc;
  {
    CuProfileScope prof("ConvolutionComponent::PropagateRelu");
    rc = hipF_conv2d_relu(in.Data(), in.Dim(), in_height_, in_width_, in_channel_,
                          in_pad_height_, in_pad_width_, linear_params_.Data(),
                          linear_params_.Dim(), kernel_height_, kernel_width_, group_,
                          bias_params_.Data(), relu_out->Data(), relu_out->Dim(), S());
    if (rc < 0) prof.Cancel();  // declined: nothing launched
  }
  if (rc < 0) return false;
  CNSL_SAFE_CALL(rc);
  return true;
}

void ConvolutionComponent::PropagateLiteral(const ChunkInfo &in_info,
                                            const CuMatrixBase<BaseFloat> &in,
                                            CuMatrixBase<BaseFloat> *out) const {
  (void)in_info;
  if (in_pad_height_ > 0 || in_pad_width_ > 0) {                   // :430
    CuMatrix<BaseFloat> padded_input(
        in.NumRows(), (in_height_ + 2 * in_pad_height_) *
                          (in_width_ + 2 * in_pad_width_) * in_channel_);
    in.PaddingZero(in_height_, in_width_, in_channel_, in_pad_height_ + 1,
                   in_pad_width_ + 1, &padded_input);               // :433
    padded_input.Conv2D(linear_params_, in_height_ + 2 * in_pad_height_,
                        in_width_ + 2 * in_pad_width_, in_channel_,
                        kernel_height_, kernel_width_, group_, out, true);
  } else {
    in.Conv2D(linear_params_, in_height_, in_width_, in_channel_,
              kernel_height_, kernel_width_, group_, out, true);    // :438
  }
  out->AddMatRepVec(bias_params_, out_height_ * out_width_);        // :443
}

void ConvolutionComponent::Scale(BaseFloat scale) {                 // :448
  linear_params_.Scale(scale);
  bias_params_.Scale(scale);
}

void ConvolutionComponent::Add(BaseFloat alpha, const UpdatableComponent &other_in) {
  const ConvolutionComponent *other =
      dynamic_cast<const ConvolutionComponent *>(&other_in);
  KALDI_ASSERT(other != NULL);
  linear_params_.AddMat(alpha, other->linear_params_);
  bias_params_.AddVec(alpha, other->bias_params_);
}

// :489-497
bool ConvolutionComponent::FlipKernelBranch() const {
  const int32 pad_kernel_size =
      (kernel_height_ + 2 * (out_height_ - in_pad_height_ - 1)) *
      (kernel_width_ + 2 * (out_width_ - in_pad_width_ - 1));
  const int32 pad_out_size =
      (out_height_ + 2 * (kernel_height_ - in_pad_height_ - 1)) *
      (out_width_ + 2 * (kernel_width_ - in_pad_width_ - 1));
  return !(pad_kernel_size < pad_out_size);
}

// :461-544.  The data gradient is computed in gather form for either branch
// (one "full" correlation of out_deriv with the 180-degree rotated kernel,
// padding virtual, no materialised intermediates); both of the reference's
// branches compute this same sum.  Then Update (:541-543), after dX.
void ConvolutionComponent::Backprop(const ChunkInfo &, const ChunkInfo &,
                                    const CuMatrixBase<BaseFloat> &in_value,
                                    const CuMatrixBase<BaseFloat> &,
                                    const CuMatrixBase<BaseFloat> &out_deriv,
                                    Component *to_update_in,
                                    CuMatrix<BaseFloat> *in_deriv) const {
  const int32 num_chunks = out_deriv.NumRows();                     // :469
  ConvolutionComponent *to_update =
      dynamic_cast<ConvolutionComponent *>(to_update_in);
  KALDI_ASSERT(out_deriv.NumCols() == OutputDim());
  if (!LiteralPath() && to_update != NULL && in_deriv != NULL) {
    // dX (with the pre-update kernel, as the reference orders it) and the
    // gradient from one pass over out_deriv, then the update step (:541).
    Scratch grad(sizeof(BaseFloat) * (size_t)NumGradientParams());
    // the step in the gradient's reduction where the frame kernels run it
    // (conv-update.h), else ApplyGradient on the gradient
    ConvUpdateEpi ue{};
    to_update->UpdateRequest(in_value.NumRows(), &ue);
    {
      ConvUpdateScope scope(&ue);
      BackpropGradient(ChunkInfo(), ChunkInfo(), in_value, in_value, out_deriv,
                       in_deriv, grad.f());
    }
    if (!ue.applied) to_update->ApplyGradient(grad.f(), in_value.NumRows());
    return;
  }
  if (in_deriv != NULL) {
    if (in_deriv->NumRows() != num_chunks || in_deriv->NumCols() != InputDim())
      in_deriv->Resize(num_chunks, InputDim(), kUndefined);
    if (LiteralPath()) {
      BackpropDataLiteral(out_deriv, in_deriv);
    } else {
      KALDI_ASSERT(kernel_height_ - 1 - in_pad_height_ >= 0 &&
                   kernel_width_ - 1 - in_pad_width_ >= 0 &&
                   "kernel must exceed the padding");               // :533
      const size_t ws_bytes = hipF_conv2d_dgrad_workspace_bytes(
          out_deriv.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
          in_pad_width_, kernel_height_, kernel_width_, group_);
      Scratch ws_s(ws_bytes);
  void *ws = ws_s.p;
      CuProfileScope prof("ConvolutionComponent::BackpropData");
      CNSL_SAFE_CALL(hipF_conv2d_dgrad(
          out_deriv.Data(), out_deriv.Dim(), in_height_, in_width_, in_channel_,
          in_pad_height_, in_pad_width_, linear_params_.Data(),
          linear_params_.Dim(), kernel_height_, kernel_width_, group_,
          in_deriv->Data(), in_deriv->Dim(), ws, ws_bytes, S()));
    }
  }
  if (to_update != NULL) to_update->Update(in_value, out_deriv);    // :541
}

// The reference's two branches, literally (:478-540).
void ConvolutionComponent::BackpropDataLiteral(
    const CuMatrixBase<BaseFloat> &out_deriv, CuMatrix<BaseFloat> *in_deriv) const {
  const int32 num_chunks = out_deriv.NumRows();
  const int32 pad_kernel_height = kernel_height_ + 2 * (out_height_ - in_pad_height_ - 1),
              pad_kernel_width = kernel_width_ + 2 * (out_width_ - in_pad_width_ - 1),
              pad_out_deriv_height = out_height_ + 2 * (kernel_height_ - in_pad_height_ - 1),
              pad_out_deriv_width = out_width_ + 2 * (kernel_width_ - in_pad_width_ - 1);
  if (!FlipKernelBranch()) {                                        // :499
    CuMatrix<BaseFloat> flip_out_deriv(out_height_ * out_width_ * group_, num_chunks);
    {
      CuMatrix<BaseFloat> out_deriv_tp(out_height_ * out_width_ * out_deriv.NumRows(), group_);
      out_deriv.TpInsideBlock(group_, out_height_ * out_width_, &out_deriv_tp);
      out_deriv_tp.FlipMat(out_height_, out_width_, num_chunks, group_, &flip_out_deriv);
    }
    CuMatrix<BaseFloat> pad_kernel(in_channel_, pad_kernel_height * pad_kernel_width * group_);
    {
      CuMatrix<BaseFloat> linear_params_tp(group_, kernel_height_ * kernel_width_ * in_channel_);
      CuMatrix<BaseFloat> linear_params_tp2(in_channel_, kernel_height_ * kernel_width_ * group_);
      linear_params_tp.AddMat(1.0, linear_params_, kTrans);         // :516
      linear_params_tp.TpBlock(in_channel_, kernel_height_ * kernel_width_, &linear_params_tp2);
      linear_params_tp2.PaddingZero(kernel_height_, kernel_width_, group_,
                                    out_height_ - in_pad_height_,
                                    out_width_ - in_pad_width_, &pad_kernel);
    }
    CuMatrix<BaseFloat> in_deriv_tmp(in_channel_, in_height_ * in_width_ * num_chunks);
    pad_kernel.Conv2D(flip_out_deriv, pad_kernel_height, pad_kernel_width, group_,
                      out_height_, out_width_, num_chunks, &in_deriv_tmp, true);
    in_deriv_tmp.TpBlock(num_chunks, in_height_ * in_width_, in_deriv); // :525
  } else {
    CuMatrix<BaseFloat> pad_out_deriv(out_deriv.NumRows(),
                                      pad_out_deriv_height * pad_out_deriv_width * group_);
    CuMatrix<BaseFloat> flip_kernel(kernel_height_ * kernel_width_ * group_, in_channel_);
    out_deriv.PaddingZero(out_height_, out_width_, group_,
                          kernel_height_ - in_pad_height_,
                          kernel_width_ - in_pad_width_, &pad_out_deriv); // :534
    linear_params_.FlipMat(kernel_height_, kernel_width_, in_channel_, group_, &flip_kernel);
    pad_out_deriv.Conv2D(flip_kernel, pad_out_deriv_height, pad_out_deriv_width,
                         group_, kernel_height_, kernel_width_, in_channel_,
                         in_deriv, true);                           // :538
  }
}

void ConvolutionComponent::SetZero(bool treat_as_gradient) {        // :546
  if (treat_as_gradient) SetLearningRate(1.0);
  linear_params_.SetZero();
  bias_params_.SetZero();
  if (treat_as_gradient) is_gradient_ = true;
}

// :556-619
void ConvolutionComponent::Read(std::istream &is, bool binary) {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  ExpectOneOrTwoTokens(is, binary, ostr_beg.str(), "<in_height>");
  ReadBasicType(is, binary, &in_height_);
  ExpectToken(is, binary, "<in_width>");
  ReadBasicType(is, binary, &in_width_);
  ExpectToken(is, binary, "<in_channel>");
  ReadBasicType(is, binary, &in_channel_);
  ExpectToken(is, binary, "<kernel_height>");
  ReadBasicType(is, binary, &kernel_height_);
  ExpectToken(is, binary, "<kernel_width>");
  ReadBasicType(is, binary, &kernel_width_);
  ExpectToken(is, binary, "<stride>");
  ReadBasicType(is, binary, &stride_);
  ExpectToken(is, binary, "<padding_height>");
  ReadBasicType(is, binary, &in_pad_height_);
  ExpectToken(is, binary, "<padding_width>");
  ReadBasicType(is, binary, &in_pad_width_);
  ExpectToken(is, binary, "<group>");
  ReadBasicType(is, binary, &group_);
  ExpectToken(is, binary, "<out_height>");
  ReadBasicType(is, binary, &out_height_);
  ExpectToken(is, binary, "<out_width>");
  ReadBasicType(is, binary, &out_width_);
  ExpectToken(is, binary, "<LearningRate>");
  ReadBasicType(is, binary, &learning_rate_);
  ExpectToken(is, binary, "<WeightDecay>");
  ReadBasicType(is, binary, &weight_decay_);
  ExpectToken(is, binary, "<Momentum>");
  ReadBasicType(is, binary, &momentum_);
  ExpectToken(is, binary, "<LinearParams>");
  linear_params_.Read(is, binary);
  ExpectToken(is, binary, "<BiasParams>");
  bias_params_.Read(is, binary);
  ExpectToken(is, binary, "<PrevGrad>");
  prev_grad_.Read(is, binary);
  std::string tok;
  ReadToken(is, binary, &tok);
  if (tok == "<AvgInput>") {  // back-compatibility (:603)
    CuVector<BaseFloat> avg_input;
    avg_input.Read(is, binary);
    BaseFloat avg_input_count;
    ExpectToken(is, binary, "<AvgInputCount>");
    ReadBasicType(is, binary, &avg_input_count);
    ReadToken(is, binary, &tok);
  }
  if (tok == "<IsGradient>") {
    ReadBasicType(is, binary, &is_gradient_);
    ExpectToken(is, binary, ostr_end.str());
  } else {
    is_gradient_ = false;
    KALDI_ASSERT(tok == ostr_end.str());
  }
}

// :621-666
void ConvolutionComponent::Write(std::ostream &os, bool binary) const {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  WriteToken(os, binary, ostr_beg.str());
  WriteToken(os, binary, "<in_height>");
  WriteBasicType(os, binary, in_height_);
  WriteToken(os, binary, "<in_width>");
  WriteBasicType(os, binary, in_width_);
  WriteToken(os, binary, "<in_channel>");
  WriteBasicType(os, binary, in_channel_);
  WriteToken(os, binary, "<kernel_height>");
  WriteBasicType(os, binary, kernel_height_);
  WriteToken(os, binary, "<kernel_width>");
  WriteBasicType(os, binary, kernel_width_);
  WriteToken(os, binary, "<stride>");
  WriteBasicType(os, binary, stride_);
  WriteToken(os, binary, "<padding_height>");
  WriteBasicType(os, binary, in_pad_height_);
  WriteToken(os, binary, "<padding_width>");
  WriteBasicType(os, binary, in_pad_width_);
  WriteToken(os, binary, "<group>");
  WriteBasicType(os, binary, group_);
  WriteToken(os, binary, "<out_height>");
  WriteBasicType(os, binary, out_height_);
  WriteToken(os, binary, "<out_width>");
  WriteBasicType(os, binary, out_width_);
  WriteToken(os, binary, "<LearningRate>");
  WriteBasicType(os, binary, learning_rate_);
  WriteToken(os, binary, "<WeightDecay>");
  WriteBasicType(os, binary, weight_decay_);
  WriteToken(os, binary, "<Momentum>");
  WriteBasicType(os, binary, momentum_);
  WriteToken(os, binary, "<LinearParams>");
  linear_params_.Write(os, binary);
  WriteToken(os, binary, "<BiasParams>");
  bias_params_.Write(os, binary);
  WriteToken(os, binary, "<PrevGrad>");
  prev_grad_.Write(os, binary);
  WriteToken(os, binary, "<IsGradient>");
  WriteBasicType(os, binary, is_gradient_);
  WriteToken(os, binary, ostr_end.str());
}

BaseFloat ConvolutionComponent::DotProduct(const UpdatableComponent &other_in) const {
  const ConvolutionComponent *other =
      dynamic_cast<const ConvolutionComponent *>(&other_in);
  KALDI_ASSERT(other != NULL);
  return TraceMatMat(linear_params_, other->linear_params_, kTrans) +
         VecVec(bias_params_, other->bias_params_);                 // :674
}

Component *ConvolutionComponent::Copy() const {                     // :679-705
  ConvolutionComponent *ans = new ConvolutionComponent();
  ans->learning_rate_ = learning_rate_;
  ans->linear_params_ = linear_params_;
  ans->bias_params_ = bias_params_;
  ans->is_gradient_ = is_gradient_;
  ans->in_height_ = in_height_;
  ans->in_width_ = in_width_;
  ans->in_channel_ = in_channel_;
  ans->kernel_height_ = kernel_height_;
  ans->kernel_width_ = kernel_width_;
  ans->stride_ = stride_;
  ans->in_pad_height_ = in_pad_height_;
  ans->in_pad_width_ = in_pad_width_;
  ans->group_ = group_;
  ans->out_height_ = out_height_;
  ans->out_width_ = out_width_;
  ans->weight_decay_ = weight_decay_;
  ans->momentum_ = momentum_;
  ans->prev_grad_ = prev_grad_;
  return ans;
}

void ConvolutionComponent::PerturbParams(BaseFloat stddev) {       // :706
  CuMatrix<BaseFloat> temp_linear_params(linear_params_);
  temp_linear_params.SetRandn();
  linear_params_.AddMat(stddev, temp_linear_params);
  CuVector<BaseFloat> temp_bias_params(bias_params_);
  temp_bias_params.SetRandn();
  bias_params_.AddVec(stddev, temp_bias_params);
}

void ConvolutionComponent::SetParams(const VectorBase<BaseFloat> &bias,
                                     const MatrixBase<BaseFloat> &linear) {
  bias_params_ = bias;
  linear_params_ = linear;
  // B8: the reference asserts bias.Dim() == linear.NumRows(); a bias has one
  // entry per group (column).
  KALDI_ASSERT(bias_params_.Dim() == linear_params_.NumCols());
  if (prev_grad_.NumRows() != linear_params_.NumRows() ||
      prev_grad_.NumCols() != linear_params_.NumCols())
    prev_grad_.Resize(linear_params_.NumRows(), linear_params_.NumCols());
}

// B8 fixed: linear params (KernelDim x Group, row-major) then Group biases.
int32 ConvolutionComponent::GetParameterDim() const {
  return KernelDim() * Group() + Group();
}
void ConvolutionComponent::Vectorize(VectorBase<BaseFloat> *params) const {
  KALDI_ASSERT(params->Dim() == GetParameterDim());
  Matrix<BaseFloat> W;
  linear_params_.CopyToMat(&W);
  Vector<BaseFloat> b;
  bias_params_.CopyToVec(&b);
  const size_t nw = (size_t)KernelDim() * Group();
  std::copy(W.Data(), W.Data() + nw, params->Data());
  std::copy(b.Data(), b.Data() + Group(), params->Data() + nw);
}
void ConvolutionComponent::UnVectorize(const VectorBase<BaseFloat> &params) {
  KALDI_ASSERT(params.Dim() == GetParameterDim());
  Matrix<BaseFloat> W(KernelDim(), Group());
  const size_t nw = (size_t)KernelDim() * Group();
  std::copy(params.Data(), params.Data() + nw, W.Data());
  Vector<BaseFloat> b(Group());
  std::copy(params.Data() + nw, params.Data() + nw + Group(), b.Data());
  linear_params_.CopyFromMat(W);
  bias_params_.CopyFromVec(b);
}

// Gradient half of Update (:745-765 + the row sum of :775), fused: one
// kernel reads X (virtually padded) and dY once; no TpBlock/TpInsideBlock/
// ModPermuteRow intermediates.  grad = [KernelDim x Group | Group].
void ConvolutionComponent::ComputeGradient(const CuMatrixBase<BaseFloat> &in_value,
                                           const CuMatrixBase<BaseFloat> &out_deriv,
                                           BaseFloat *grad) const {
  KALDI_ASSERT(in_value.NumCols() == InputDim() &&
               out_deriv.NumCols() == OutputDim() &&
               in_value.NumRows() == out_deriv.NumRows());
  CuProfileScope prof("ConvolutionComponent::ComputeGradient");
  const size_t ws_bytes = hipF_conv2d_wgrad_workspace_bytes(
      in_value.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
      in_pad_width_, kernel_height_, kernel_width_, group_);
  Scratch ws_s(ws_bytes);
  void *ws = ws_s.p;
  CNSL_SAFE_CALL(hipF_conv2d_wgrad(
      in_value.Data(), in_value.Dim(), in_height_, in_width_, in_channel_,
      in_pad_height_, in_pad_width_, out_deriv.Data(), out_deriv.Dim(),
      kernel_height_, kernel_width_, group_, grad, Dense(KernelDim(), group_),
      grad + (size_t)KernelDim() * group_, ws, ws_bytes, S()));
}

// Data gradient (:461-540) and the gradient half of Update (:745-775) from
// one streamed pass over out_deriv.
void ConvolutionComponent::BackpropGradient(const ChunkInfo &in_info,
                                            const ChunkInfo &out_info,
                                            const CuMatrixBase<BaseFloat> &in_value,
                                            const CuMatrixBase<BaseFloat> &out_value,
                                            const CuMatrixBase<BaseFloat> &out_deriv,
                                            CuMatrix<BaseFloat> *in_deriv,
                                            BaseFloat *grad) const {
  if (LiteralPath()) {
    UpdatableComponent::BackpropGradient(in_info, out_info, in_value, out_value,
                                         out_deriv, in_deriv, grad);
    return;
  }
  const int32 num_chunks = out_deriv.NumRows();
  KALDI_ASSERT(in_value.NumCols() == InputDim() &&
               out_deriv.NumCols() == OutputDim() &&
               in_value.NumRows() == num_chunks);
  if (in_deriv != NULL) {
    KALDI_ASSERT(kernel_height_ - 1 - in_pad_height_ >= 0 &&
                 kernel_width_ - 1 - in_pad_width_ >= 0 &&
                 "kernel must exceed the padding");                 // :533
    if (in_deriv->NumRows() != num_chunks || in_deriv->NumCols() != InputDim())
      in_deriv->Resize(num_chunks, InputDim(), kUndefined);
  }
  const size_t ws_bytes = hipF_conv2d_backward_workspace_bytes(
      in_value.Dim(), in_height_, in_width_, in_channel_, in_pad_height_,
      in_pad_width_, kernel_height_, kernel_width_, group_);
  Scratch ws_s(ws_bytes);
  void *ws = ws_s.p;
  CuProfileScope prof("ConvolutionComponent::BackpropGradient");
  MatrixDim idd = in_value.Dim();
  CNSL_SAFE_CALL(hipF_conv2d_backward(
      in_value.Data(), in_value.Dim(), in_height_, in_width_, in_channel_,
      in_pad_height_, in_pad_width_, out_deriv.Data(), out_deriv.Dim(),
      linear_params_.Data(), linear_params_.Dim(), kernel_height_, kernel_width_,
      group_, in_deriv ? in_deriv->Data() : nullptr,
      in_deriv ? in_deriv->Dim() : idd, grad, Dense(KernelDim(), group_),
      grad + (size_t)KernelDim() * group_, ws, ws_bytes, S()));
}

bool ConvolutionComponent::BackpropPooled(const CuMatrixBase<BaseFloat> &in_value,
                                          const MaxpoolComponent &pool,
                                          const unsigned char *mask, int32 mask_stride,
                                          const CuMatrixBase<BaseFloat> &pool_deriv,
                                          Component *to_update_in,
                                          CuMatrix<BaseFloat> *in_deriv,
                                          BaseFloat *grad) const {
  ConvolutionComponent *to_update =
      grad ? NULL : dynamic_cast<ConvolutionComponent *>(to_update_in);
  if (LiteralPath() || mask == NULL || !pool.FoldsIntoConvBackprop()) return false;
  int32 pc = pool.FusableChannelPool(), ph = 1, pw = 1;
  if (pc == 0) {
    const bool win3 = pool.FusableWindow3D(&ph, &pw, &pc);
    KALDI_ASSERT(win3);
  }
  // Backprop without in_deriv: nothing to do, or (with an update) Update in
  // the unfused path, whose gradient kernel sums in another order: keep its bits
  if (grad == NULL && in_deriv == NULL) return false;
  if (pool.In_height() != out_height_ || pool.In_width() != out_width_ ||
      pool.In_channels() != group_ || pool.InputDim() != OutputDim())
    return false;
  const int32 num_chunks = in_value.NumRows();
  KALDI_ASSERT(in_value.NumCols() == InputDim() &&
               pool_deriv.NumCols() == pool.OutputDim() &&
               pool_deriv.NumRows() == num_chunks);
  if (in_deriv != NULL) {
    if (kernel_height_ - 1 - in_pad_height_ < 0 || kernel_width_ - 1 - in_pad_width_ < 0)
      return false;
    if (in_deriv->NumRows() != num_chunks || in_deriv->NumCols() != InputDim())
      in_deriv->Resize(num_chunks, InputDim(), kUndefined);
  }
  Scratch own(grad == NULL && to_update != NULL
                  ? sizeof(BaseFloat) * (size_t)NumGradientParams() : 0);
  BaseFloat *g = grad ? grad : own.f();
  const size_t ws_bytes = g ? hipF_conv2d_backward_workspace_bytes(
                                  in_value.Dim(), in_height_, in_width_, in_channel_,
                                  in_pad_height_, in_pad_width_, kernel_height_,
                                  kernel_width_, group_)
                            : 0;
  Scratch ws_s(ws_bytes);
  void *ws = ws_s.p;
  MatrixDim idd = in_value.Dim();
  int rc;
  ConvUpdateEpi ue{};
  if (to_update != NULL) to_update->UpdateRequest(num_chunks, &ue);
  {
    ConvUpdateScope scope(to_update != NULL ? &ue : nullptr);
    CuProfileScope prof("ConvolutionComponent::BackpropPooled");
    rc = ph == 1
        ? hipF_conv2d_backward_pooled(
              in_value.Data(), in_value.Dim(), in_height_, in_width_, in_channel_,
              in_pad_height_, in_pad_width_, mask, mask_stride, pool_deriv.Data(),
              pool_deriv.Dim(), pc, linear_params_.Data(), linear_params_.Dim(),
              kernel_height_, kernel_width_, group_, in_deriv ? in_deriv->Data() : nullptr,
              in_deriv ? in_deriv->Dim() : idd, g, Dense(KernelDim(), group_),
              g ? g + (size_t)KernelDim() * group_ : nullptr, ws, ws_bytes, S())
        : hipF_conv2d_backward_pooled3d(
              in_value.Data(), in_value.Dim(), in_height_, in_width_, in_channel_,
              in_pad_height_, in_pad_width_, reinterpret_cast<const unsigned short *>(mask),
              mask_stride, pool_deriv.Data(), pool_deriv.Dim(), ph, pw, pc,
              linear_params_.Data(), linear_params_.Dim(), kernel_height_, kernel_width_,
              group_, in_deriv ? in_deriv->Data() : nullptr,
              in_deriv ? in_deriv->Dim() : idd, g, Dense(KernelDim(), group_),
              g ? g + (size_t)KernelDim() * group_ : nullptr, ws, ws_bytes, S());
    if (rc < 0) prof.Cancel();  // declined: nothing launched
  }
  if (rc < 0) return false;
  CNSL_SAFE_CALL(rc);
  if (to_update != NULL && !ue.applied) to_update->ApplyGradient(g, num_chunks);
  return true;
}

void ConvolutionComponent::UpdateRequest(int32 num_sample, ConvUpdateEpi *u) {
  KALDI_ASSERT(num_sample > 0);
  const double learning_rate = learning_rate_ / (double)num_sample;  // :767
  u->W = linear_params_.Data();
  u->ldw = linear_params_.Stride();
  u->prev = prev_grad_.Data();
  u->ldp = prev_grad_.Stride();
  u->b = bias_params_.Data();
  u->Kdim = KernelDim();
  u->G = group_;
  u->momentum = momentum_;
  u->a_wd = (BaseFloat)(-1 * learning_rate * weight_decay_);
  u->a_g = (BaseFloat)learning_rate;
  u->applied = 0;
}

// Apply half of Update (:767-775), one pass over W / prev_grad_ / grad.
void ConvolutionComponent::ApplyGradient(const BaseFloat *grad, int32 num_sample) {
  KALDI_ASSERT(num_sample > 0);
  CuProfileScope prof("ConvolutionComponent::ApplyGradient");
  const double learning_rate = learning_rate_ / (double)num_sample;  // :767
  const BaseFloat a_wd = (BaseFloat)(-1 * learning_rate * weight_decay_);
  const BaseFloat a_g = (BaseFloat)learning_rate;
  CNSL_SAFE_CALL(hipF_momentum_update(
      linear_params_.Data(), linear_params_.Dim(), prev_grad_.Data(),
      prev_grad_.Dim(), grad, Dense(KernelDim(), group_), momentum_, a_wd, a_g,
      bias_params_.Data(), grad + (size_t)KernelDim() * group_, group_, S()));
}

// :738-777 (B10: is_gradient_ is ignored and the step is divided by N).
void ConvolutionComponent::Update(const CuMatrixBase<BaseFloat> &in_value,
                                  const CuMatrixBase<BaseFloat> &out_deriv) {
  if (LiteralPath()) { UpdateLiteral(in_value, out_deriv); return; }
  Scratch grad(sizeof(BaseFloat) * (size_t)NumGradientParams());
  ComputeGradient(in_value, out_deriv, grad.f());
  ApplyGradient(grad.f(), in_value.NumRows());
}

void ConvolutionComponent::UpdateLiteral(const CuMatrixBase<BaseFloat> &in_value,
                                         const CuMatrixBase<BaseFloat> &out_deriv) {
  const int32 num_sample = in_value.NumRows();                      // :741
  const int32 in_height = in_height_ + 2 * (in_pad_height_),
              in_width = in_width_ + 2 * (in_pad_width_);
  CuMatrix<BaseFloat> in_value_tmp(in_channel_, num_sample * in_height * in_width);
  CuMatrix<BaseFloat> out_deriv_tmp(out_height_ * out_width_ * num_sample, group_);
  CuMatrix<BaseFloat> linear_params_tmp(kernel_height_ * kernel_width_ * in_channel_, group_);
  CuMatrix<BaseFloat> linear_params_grad(kernel_height_ * kernel_width_ * in_channel_, group_);
  if (in_pad_height_ > 0 || in_pad_width_ > 0) {                   // :751
    CuMatrix<BaseFloat> padded_input(num_sample, in_height * in_width * in_channel_);
    in_value.PaddingZero(in_height_, in_width_, in_channel_, in_pad_height_ + 1,
                         in_pad_width_ + 1, &padded_input);
    padded_input.TpBlock(in_channel_, in_height * in_width, &in_value_tmp);
  } else {
    in_value.TpBlock(in_channel_, in_height * in_width, &in_value_tmp);
  }
  out_deriv.TpInsideBlock(group_, out_height_ * out_width_, &out_deriv_tmp);
  in_value_tmp.Conv2D(out_deriv_tmp, in_height, in_width, num_sample,
                      out_height_, out_width_, group_, &linear_params_tmp, false);
  linear_params_tmp.ModPermuteRow(in_channel_, kernel_height_ * kernel_width_,
                                  &linear_params_grad);             // :765
  const double learning_rate = learning_rate_ / (double)num_sample;
  prev_grad_.Scale(momentum_);
  prev_grad_.AddMat(-1 * learning_rate * weight_decay_, linear_params_, kNoTrans);
  prev_grad_.AddMat(learning_rate, linear_params_grad, kNoTrans);
  linear_params_.AddMat(1.0, prev_grad_, kNoTrans);
  bias_params_.AddRowSumMat(learning_rate, out_deriv_tmp, 1.0);     // :775
}

// ===========================================================================
// MaxpoolComponent
// ===========================================================================
// :779-812
void MaxpoolComponent::Init(int32 input_dim, int32 output_dim, int32 in_height,
                            int32 in_width, int32 in_channel,
                            int32 pool_height_dim, int32 pool_width_dim,
                            int32 pool_channel_dim, bool overlap,
                            bool overlap2D) {
  input_dim_ = input_dim;
  output_dim_ = output_dim;
  in_height_ = in_height;
  in_width_ = in_width;
  in_channel_ = in_channel;
  pool_height_dim_ = pool_height_dim;
  pool_width_dim_ = pool_width_dim;
  pool_channel_dim_ = pool_channel_dim;
  overlap_ = overlap;
  overlap2D_ = overlap2D;
  KALDI_ASSERT((in_height_ * in_width_ * in_channel_) == input_dim_);
  KALDI_ASSERT(input_dim_ > 0 && output_dim_ > 0 && pool_height_dim_ > 0 &&
               pool_width_dim_ > 0 && pool_channel_dim_ > 0);
  KALDI_ASSERT(in_height_ % pool_height_dim_ == 0);
  KALDI_ASSERT(in_width_ % pool_width_dim_ == 0);
  KALDI_ASSERT((overlap && overlap2D) != true);
  if (overlap2D) {
    KALDI_ASSERT(pool_height_dim_ == 1 && pool_width_dim_ == 1);
    const int32 output_channel = output_dim_ / (in_height_ * in_width_);
    const int32 expected = (int32)pow((sqrt((double)in_channel_) - pool_channel_dim_ + 1), 2);
    KALDI_ASSERT(output_channel == expected);
  } else if (overlap) {
    KALDI_ASSERT(pool_height_dim_ == 1 && pool_width_dim_ == 1);
    KALDI_ASSERT(input_dim_ / in_channel_ * (in_channel_ - pool_channel_dim_ + 1) == output_dim_);
  } else {
    KALDI_ASSERT(input_dim_ % output_dim_ == 0);
    KALDI_ASSERT(in_channel_ % pool_channel_dim_ == 0);
    KALDI_ASSERT(input_dim_ / (pool_height_dim_ * pool_width_dim_ * pool_channel_dim_) == output_dim_);
  }
}

// :814-867
void MaxpoolComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  int32 in_height = 1, in_width = 1, in_channel = 1;
  int32 pool_height_dim = 1, pool_width_dim = 1, pool_channel_dim = 1;
  bool overlap = false, overlap2D = false;
  bool ok = ParseFromString("in-height", &args, &in_height) &&
            ParseFromString("in-width", &args, &in_width) &&
            ParseFromString("in-channel", &args, &in_channel) &&
            ParseFromString("pool-height-dim", &args, &pool_height_dim) &&
            ParseFromString("pool-width-dim", &args, &pool_width_dim) &&
            ParseFromString("pool-channel-dim", &args, &pool_channel_dim);
  ParseFromString("overlap", &args, &overlap);
  ParseFromString("overlap2D", &args, &overlap2D);
  const int32 input_dim = in_height * in_width * in_channel;
  int32 output_dim;
  if (overlap2D) {
    const int32 output_channel = (int32)pow((sqrt((double)in_channel) - pool_channel_dim + 1), 2);
    output_dim = input_dim / in_channel * output_channel;
  } else if (overlap) {
    output_dim = input_dim / in_channel * (in_channel - pool_channel_dim + 1);
  } else {
    output_dim = (pool_height_dim * pool_width_dim * pool_channel_dim) > 0
                     ? input_dim / (pool_height_dim * pool_width_dim * pool_channel_dim)
                     : 0;
  }
  if (!ok || !args.empty() || output_dim <= 0)
    KALDI_ERR << "Invalid initializer for layer of type " << Type() << ": \""
              << orig_args << "\"";
  Init(input_dim, output_dim, in_height, in_width, in_channel, pool_height_dim,
       pool_width_dim, pool_channel_dim, overlap, overlap2D);
}

// :869-880
void MaxpoolComponent::Propagate(const ChunkInfo &in_info,
                                 const ChunkInfo &out_info,
                                 const CuMatrixBase<BaseFloat> &in,
                                 CuMatrixBase<BaseFloat> *out) const {
  in_info.CheckSize(in);
  out_info.CheckSize(*out);
  CuProfileScope prof("MaxpoolComponent::Propagate");
  in.Maxpool_prop(in_height_, in_width_, pool_height_dim_, pool_width_dim_,
                  pool_channel_dim_, overlap_, overlap2D_, out);
}

// :882-892.  The zeroing Resize (:889) is fused into the routing kernel:
// every in_deriv element is written once (0 or the routed derivative).
void MaxpoolComponent::Backprop(const ChunkInfo &, const ChunkInfo &,
                                const CuMatrixBase<BaseFloat> &in_value,
                                const CuMatrixBase<BaseFloat> &out_value,
                                const CuMatrixBase<BaseFloat> &out_deriv,
                                Component *, CuMatrix<BaseFloat> *in_deriv) const {
  KALDI_ASSERT(output_dim_ == out_value.NumCols());                 // :890
  if (LiteralPath()) {
    in_deriv->Resize(in_value.NumRows(), in_value.NumCols(), kSetZero);
    in_value.Maxpool_backprop(out_value, out_deriv, in_deriv, in_height_,
                              in_width_, pool_height_dim_, pool_width_dim_,
                              pool_channel_dim_, overlap_, overlap2D_);
    return;
  }
  in_deriv->Resize(in_value.NumRows(), in_value.NumCols(), kUndefined);
  KALDI_ASSERT(out_deriv.NumRows() == out_value.NumRows() &&
               out_deriv.NumCols() == out_value.NumCols() &&
               out_value.NumRows() == in_value.NumRows());
  CuProfileScope prof("MaxpoolComponent::Backprop");
  const int mode = overlap_ ? 1 : (overlap2D_ ? 2 : 0);
  CNSL_SAFE_CALL(hipF_maxpool_backprop(
      in_value.Data(), in_value.Dim(), out_value.Data(), out_value.Dim(),
      out_deriv.Data(), out_deriv.Dim(), in_deriv->Data(), in_deriv->Dim(),
      in_height_, in_width_, pool_height_dim_, pool_width_dim_,
      pool_channel_dim_, mode, 1, S()));
}

int32 MaxpoolComponent::FusableChannelPool() const {
  const int32 pc = pool_channel_dim_;
  if (overlap_ || overlap2D_ || pool_height_dim_ != 1 || pool_width_dim_ != 1)
    return 0;
  if (!(pc == 2 || pc == 4 || pc == 8) || in_channel_ % pc != 0) return 0;
  return output_dim_ * pc == input_dim_ ? pc : 0;
}

bool MaxpoolComponent::FusableWindow3D(int32 *ph, int32 *pw, int32 *pc) const {
  if (overlap_ || overlap2D_ || (pool_height_dim_ == 1 && pool_width_dim_ == 1))
    return false;
  const int32 c = pool_channel_dim_;
  if (c <= 0 || 32 % c != 0 || in_channel_ % c != 0 ||
      pool_height_dim_ * pool_width_dim_ * c > 16 || in_height_ % pool_height_dim_ != 0 ||
      in_width_ % pool_width_dim_ != 0 ||
      output_dim_ * pool_height_dim_ * pool_width_dim_ * c != input_dim_)
    return false;
  *ph = pool_height_dim_;
  *pw = pool_width_dim_;
  *pc = c;
  return true;
}

bool MaxpoolComponent::FoldsIntoConvBackprop() const {
  // KCNN_FOLD_3D=0: 3-D windows back to BackpropFromMask + the conv's Backprop
  static const bool fold3d = KCNN_KNOB("KCNN_FOLD_3D", 1) != 0;
  const int32 c = FusableChannelPool();
  if (c == 4 || c == 8) return true;
  int32 ph, pw, pc;
  return fold3d && c == 0 && FusableWindow3D(&ph, &pw, &pc) && pw == 1 && (ph == 2 || ph == 3) &&
         (pc == 4 || pc == 8) && ph * pc <= 16;
}

int32 MaxpoolComponent::FusedMaskBytes() const {
  int32 ph, pw, pc;
  if (FusableChannelPool() > 0) return 1;
  return FusableWindow3D(&ph, &pw, &pc) ? 2 : 0;
}

void MaxpoolComponent::BackpropFromMask(const unsigned char *mask,
                                        int32 mask_stride,
                                        const CuMatrixBase<BaseFloat> &out_deriv,
                                        CuMatrix<BaseFloat> *in_deriv) const {
  KALDI_ASSERT(mask != NULL && out_deriv.NumCols() == output_dim_);
  in_deriv->Resize(out_deriv.NumRows(), input_dim_, kUndefined);  // every element written
  CuProfileScope prof("MaxpoolComponent::BackpropFromMask");
  const int32 pc = FusableChannelPool();
  if (pc > 0) {
    CNSL_SAFE_CALL(hipF_maxpool_backprop_mask(
        mask, mask_stride, out_deriv.Data(), out_deriv.Dim(), in_deriv->Data(),
        in_deriv->Dim(), in_height_, in_width_, pc, S()));
    return;
  }
  int32 ph, pw, c3;
  KALDI_ASSERT(FusableWindow3D(&ph, &pw, &c3));
  CNSL_SAFE_CALL(hipF_maxpool_backprop_mask3d(
      reinterpret_cast<const unsigned short *>(mask), mask_stride, out_deriv.Data(),
      out_deriv.Dim(), in_deriv->Data(), in_deriv->Dim(), in_height_, in_width_, ph, pw, c3,
      S()));
}

// :894-934
void MaxpoolComponent::Read(std::istream &is, bool binary) {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  ExpectOneOrTwoTokens(is, binary, ostr_beg.str(), "<InputDim>");
  ReadBasicType(is, binary, &input_dim_);
  ExpectToken(is, binary, "<in_height>");
  ReadBasicType(is, binary, &in_height_);
  ExpectToken(is, binary, "<in_width>");
  ReadBasicType(is, binary, &in_width_);
  ExpectToken(is, binary, "<in_channel>");
  ReadBasicType(is, binary, &in_channel_);
  ExpectToken(is, binary, "<OutputDim>");
  ReadBasicType(is, binary, &output_dim_);
  ExpectToken(is, binary, "<PoolHeightDim>");
  ReadBasicType(is, binary, &pool_height_dim_);
  ExpectToken(is, binary, "<PoolWidthDim>");
  ReadBasicType(is, binary, &pool_width_dim_);
  ExpectToken(is, binary, "<PoolChannelDim>");
  ReadBasicType(is, binary, &pool_channel_dim_);
  std::string tok;
  ReadToken(is, binary, &tok);
  if (tok == "<Overlap>") {
    ReadBasicType(is, binary, &overlap_);
    ReadToken(is, binary, &tok);
    if (tok == "<Overlap2D>") {
      ReadBasicType(is, binary, &overlap2D_);
      ExpectToken(is, binary, "</MaxpoolComponent>");
    } else {
      overlap2D_ = false;
      KALDI_ASSERT(tok == ostr_end.str());
    }
  } else {
    overlap_ = false;
    overlap2D_ = false;
    KALDI_ASSERT(tok == ostr_end.str());
  }
}

// :936-959
void MaxpoolComponent::Write(std::ostream &os, bool binary) const {
  WriteToken(os, binary, "<MaxpoolComponent>");
  WriteToken(os, binary, "<InputDim>");
  WriteBasicType(os, binary, input_dim_);
  WriteToken(os, binary, "<in_height>");
  WriteBasicType(os, binary, in_height_);
  WriteToken(os, binary, "<in_width>");
  WriteBasicType(os, binary, in_width_);
  WriteToken(os, binary, "<in_channel>");
  WriteBasicType(os, binary, in_channel_);
  WriteToken(os, binary, "<OutputDim>");
  WriteBasicType(os, binary, output_dim_);
  WriteToken(os, binary, "<PoolHeightDim>");
  WriteBasicType(os, binary, pool_height_dim_);
  WriteToken(os, binary, "<PoolWidthDim>");
  WriteBasicType(os, binary, pool_width_dim_);
  WriteToken(os, binary, "<PoolChannelDim>");
  WriteBasicType(os, binary, pool_channel_dim_);
  WriteToken(os, binary, "<Overlap>");
  WriteBasicType(os, binary, overlap_);
  WriteToken(os, binary, "<Overlap2D>");
  WriteBasicType(os, binary, overlap2D_);
  WriteToken(os, binary, "</MaxpoolComponent>");
}

std::string MaxpoolComponent::Info() const {                        // :961
  std::stringstream stream;
  stream << Type() << " input-dim=" << input_dim_ << " ( in-height="
         << in_height_ << ", in-width=" << in_width_
         << ", in-channels=" << in_channel_ << "), output-dim=" << output_dim_
         << ", pool_height_dim_= " << pool_height_dim_
         << ", pool_width_dim_ = " << pool_width_dim_
         << ", pool_channel_dim_ = " << pool_channel_dim_
         << ", max-pool-overlap_ = " << overlap_
         << ", max-pool-overlap_2D = " << overlap2D_;
  return stream.str();
}

// ===========================================================================
// FullyConnectedComponent
// ===========================================================================
// :980-999
void FullyConnectedComponent::Read(std::istream &is, bool binary) {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  ExpectOneOrTwoTokens(is, binary, ostr_beg.str(), "<LearningRate>");
  ReadBasicType(is, binary, &learning_rate_);
  ExpectToken(is, binary, "<LinearParams>");
  linear_params_.Read(is, binary);
  ExpectToken(is, binary, "<BiasParams>");
  bias_params_.Read(is, binary);
  ExpectToken(is, binary, "<WeightDecay>");
  ReadBasicType(is, binary, &weight_decay_);
  ExpectToken(is, binary, "<Momentum>");
  ReadBasicType(is, binary, &momentum_);
  ExpectToken(is, binary, "<PrevGrad>");
  prev_grad_.Read(is, binary);
  ExpectToken(is, binary, ostr_end.str());
}

// :1001-1020
void FullyConnectedComponent::Write(std::ostream &os, bool binary) const {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  WriteToken(os, binary, ostr_beg.str());
  WriteToken(os, binary, "<LearningRate>");
  WriteBasicType(os, binary, learning_rate_);
  WriteToken(os, binary, "<LinearParams>");
  linear_params_.Write(os, binary);
  WriteToken(os, binary, "<BiasParams>");
  bias_params_.Write(os, binary);
  WriteToken(os, binary, "<WeightDecay>");
  WriteBasicType(os, binary, weight_decay_);
  WriteToken(os, binary, "<Momentum>");
  WriteBasicType(os, binary, momentum_);
  WriteToken(os, binary, "<PrevGrad>");
  prev_grad_.Write(os, binary);
  WriteToken(os, binary, ostr_end.str());
}

// :1022-1045
void FullyConnectedComponent::Init(BaseFloat learning_rate, int32 input_dim,
                                   int32 output_dim, BaseFloat param_stddev,
                                   BaseFloat bias_stddev,
                                   BaseFloat weight_decay, BaseFloat momentum) {
  UpdatableComponent::Init(learning_rate);
  KALDI_ASSERT(input_dim > 0 && output_dim > 0);
  linear_params_.Resize(output_dim, input_dim);
  bias_params_.Resize(output_dim);
  KALDI_ASSERT(output_dim > 0 && input_dim > 0 && param_stddev >= 0.0);
  linear_params_.SetRandn();
  linear_params_.Scale(param_stddev);
  bias_params_.SetZero();
  bias_params_.Add(bias_stddev);  // a constant bias, not random (:1036-1037)
  weight_decay_ = weight_decay;
  KALDI_ASSERT(weight_decay_ > 0.0);
  momentum_ = momentum;
  KALDI_ASSERT(momentum_ > 0.0);
  prev_grad_.Resize(output_dim, input_dim);
  prev_grad_.SetZero();
}

// :1066-1100
void FullyConnectedComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  std::string matrix_filename;
  BaseFloat learning_rate = learning_rate_;
  BaseFloat weight_decay = weight_decay_, momentum = momentum_;
  int32 input_dim = -1, output_dim = -1;
  ParseFromString("learning-rate", &args, &learning_rate);
  ParseFromString("weight-decay", &args, &weight_decay);
  ParseFromString("momentum", &args, &momentum);
  if (ParseFromString("matrix", &args, &matrix_filename))
    KALDI_ERR << "matrix= initialisation is not supported (SURVEY B12)";
  bool ok = true;
  ok = ok && ParseFromString("input-dim", &args, &input_dim);
  ok = ok && ParseFromString("output-dim", &args, &output_dim);
  BaseFloat param_stddev = 1.0 / std::sqrt((double)(input_dim > 0 ? input_dim : 1)),
            bias_stddev = 1.0;
  ParseFromString("param-stddev", &args, &param_stddev);
  ParseFromString("bias-stddev", &args, &bias_stddev);
  if (!ok) KALDI_ERR << "Bad initializer " << orig_args;
  Init(learning_rate, input_dim, output_dim, param_stddev, bias_stddev,
       weight_decay, momentum);
  if (!args.empty())
    KALDI_ERR << "Could not process these elements in initializer: " << args;
}

std::string FullyConnectedComponent::Info() const {                // :1102
  std::stringstream stream;
  const double size = (double)linear_params_.NumRows() * linear_params_.NumCols();
  const double ls = std::sqrt(TraceMatMat(linear_params_, linear_params_, kTrans) / size);
  const double bs = std::sqrt(VecVec(bias_params_, bias_params_) / bias_params_.Dim());
  stream << Type() << ", input-dim=" << InputDim()
         << ", output-dim=" << OutputDim() << ", linear-params-stddev=" << ls
         << ", bias-params-stddev=" << bs
         << ", learning-rate=" << LearningRate()
         << ", weight-decay=" << weight_decay_ << ", momentum=" << momentum_;
  return stream.str();
}

Component *FullyConnectedComponent::Copy() const {                  // :1121
  FullyConnectedComponent *ans = new FullyConnectedComponent();
  ans->learning_rate_ = learning_rate_;
  ans->linear_params_ = linear_params_;
  ans->bias_params_ = bias_params_;
  ans->weight_decay_ = weight_decay_;
  ans->momentum_ = momentum_;
  ans->prev_grad_ = prev_grad_;
  ans->is_gradient_ = is_gradient_;
  return ans;
}

// grad = [OutputDim x InputDim | OutputDim]: dY^T X (:1141) and the row sum
// of dY (:1137), both unscaled.
void FullyConnectedComponent::ComputeGradient(const CuMatrixBase<BaseFloat> &in_value,
                                              const CuMatrixBase<BaseFloat> &out_deriv,
                                              BaseFloat *grad) const {
  KALDI_ASSERT(in_value.NumCols() == InputDim() &&
               out_deriv.NumCols() == OutputDim() &&
               in_value.NumRows() == out_deriv.NumRows());
  CuProfileScope prof("FullyConnectedComponent::ComputeGradient");
  CuSubMatrix<BaseFloat> gW(grad, OutputDim(), InputDim(), InputDim());
  gW.AddMatMat(1.0, out_deriv, kTrans, in_value, kNoTrans, 0.0);
  CuSubVector<BaseFloat> gb(grad + (size_t)OutputDim() * InputDim(), OutputDim());
  gb.AddRowSumMat(1.0, out_deriv, 0.0);
}

void FullyConnectedComponent::ApplyGradient(const BaseFloat *grad, int32 num_sample) {
  KALDI_ASSERT(num_sample > 0);
  CuProfileScope prof("FullyConnectedComponent::ApplyGradient");
  const double learning_rate = learning_rate_ / (double)num_sample; // :1136
  const BaseFloat a_wd = (BaseFloat)(-1 * learning_rate * weight_decay_);
  const BaseFloat a_g = (BaseFloat)learning_rate;
  CNSL_SAFE_CALL(hipF_momentum_update(
      linear_params_.Data(), linear_params_.Dim(), prev_grad_.Data(),
      prev_grad_.Dim(), grad, Dense(OutputDim(), InputDim()), momentum_, a_wd,
      a_g, bias_params_.Data(), grad + (size_t)OutputDim() * InputDim(),
      OutputDim(), S()));
}

// :1133-1150
void FullyConnectedComponent::UpdateSimple(const CuMatrixBase<BaseFloat> &in_value,
                                           const CuMatrixBase<BaseFloat> &out_deriv) {
  const int32 num_sample = in_value.NumRows();
  if (LiteralPath()) {
    const double learning_rate = learning_rate_ / (double)num_sample;
    bias_params_.AddRowSumMat(learning_rate, out_deriv, 1.0);
    prev_grad_.Scale(momentum_);
    prev_grad_.AddMat(-1 * learning_rate * weight_decay_, linear_params_, kNoTrans);
    prev_grad_.AddMatMat(learning_rate, out_deriv, kTrans, in_value, kNoTrans, 1.0);
    linear_params_.AddMat(1.0, prev_grad_, kNoTrans);
    return;
  }
  // f16x3 engine: the weight gradient applied as the momentum update in the
  // GEMM's own store (no gradient buffer: 2 x 47.6 MB of c2's traffic), the
  // bias row as in ApplyGradient; the same bits as ComputeGradient +
  // ApplyGradient (momentum-step.h), the path the data-parallel step keeps
  {
    const double learning_rate = learning_rate_ / (double)num_sample;  // :1136
    const BaseFloat a_wd = (BaseFloat)(-1 * learning_rate * weight_decay_);
    const BaseFloat a_g = (BaseFloat)learning_rate;
    CuProfileScope prof("FullyConnectedComponent::ComputeGradient");
    if (linear_params_.AddMatMatMomentum(out_deriv, kTrans, in_value, kNoTrans, &prev_grad_,
                                         momentum_, a_wd, a_g)) {
      // the bias row b = a_g colsum(dY) + b in the column sum's final pass
      // (one rounding: ApplyGradient's BiasUpdate bits, no gradient vector)
      bias_params_.AddRowSumMat(a_g, out_deriv, 1.0);
      return;
    }
  }
  Scratch grad(sizeof(BaseFloat) * (size_t)NumGradientParams());
  ComputeGradient(in_value, out_deriv, grad.f());
  ApplyGradient(grad.f(), num_sample);
}

}  // namespace nnet0
}  // namespace cnsl
