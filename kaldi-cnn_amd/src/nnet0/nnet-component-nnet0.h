// nnet0/nnet-component-nnet0.h -- ConvolutionComponent, MaxpoolComponent and
// FullyConnectedComponent with the reference's class layout and virtual
// interface (reference src/nnet0/nnet-component-nnet0.h:23-232), so they plug
// into nnet2 through the same factory names (nnet-component.cc:112-117).
//
// Execution is MI355X-native: Propagate/Backprop run fused HIP kernels
// (implicit-GEMM MFMA convolution with virtual padding and bias epilogue,
// gather-form data gradient, fused weight gradient + one-pass momentum
// update, zero-fused max-pool routing).  SetLiteralPath(true) (or
// KCNN_LITERAL=1) instead replays the reference's exact sequence of
// CuMatrixBase calls (PaddingZero, FlipMat, TpBlock, Conv2D, ...) on the
// GPU -- slower, used to cross-check the helpers as the reference uses them.
//
// ConvolutionComponentContainer (reference h:234-328) is never registered
// with the factory and is out of scope.
#ifndef KCNN_NNET0_NNET_COMPONENT_NNET0_H_
#define KCNN_NNET0_NNET_COMPONENT_NNET0_H_

#include <iostream>
#include <string>

#include "../cnslmat/pool-stats.h"
#include "../kaldi-lite/cu-matrix.h"
#include "../nnet2/nnet-component.h"

using namespace kaldi;
using namespace kaldi::nnet2;

struct ConvUpdateEpi;  // cnslmat/conv-update.h

namespace cnsl {
namespace nnet0 {

void SetLiteralPath(bool literal);
bool LiteralPath();

class MaxpoolComponent;

class ConvolutionComponent : public nnet2::UpdatableComponent {
 public:
  explicit ConvolutionComponent(const ConvolutionComponent &other);
  ConvolutionComponent()
      : is_gradient_(false), weight_decay_(0.0002), momentum_(0.9) {}
  ConvolutionComponent(const CuMatrixBase<BaseFloat> &linear_params,
                       const CuVectorBase<BaseFloat> &bias_params,
                       BaseFloat learning_rate, int32 in_height,
                       int32 in_width, int32 in_channels, int32 in_pad_height,
                       int32 in_pad_width, int32 kernel_height,
                       int32 kernel_width, int32 stride, int32 group,
                       int32 out_height, int32 out_width,
                       BaseFloat weight_decay, BaseFloat momentum);
  virtual ~ConvolutionComponent() {}

  // in  = [num_chunks x (in_height_ * in_width_ * in_channel_)]
  // out = [num_chunks x (out_height_ * out_width_ * group_)]
  // linear_params_ = [(kernel_height_ * kernel_width_ * in_channel_) x group_]
  // bias_params_ = [group_]
  virtual int32 InputDim() const { return in_height_ * in_width_ * in_channel_; }
  virtual int32 OutputDim() const { return out_height_ * out_width_ * group_; }
  inline int32 In_height() const { return in_height_; }
  inline int32 In_width() const { return in_width_; }
  inline int32 In_channels() const { return in_channel_; }
  inline int32 Out_height() const { return out_height_; }
  inline int32 Out_width() const { return out_width_; }
  inline int32 Group() const { return group_; }
  inline int32 In_pad_height() const { return in_pad_height_; }
  inline int32 In_pad_width() const { return in_pad_width_; }
  inline int32 KernelDim() const { return kernel_height_ * kernel_width_ * in_channel_; }
  inline int32 Kernel_height() const { return kernel_height_; }
  inline int32 Kernel_width() const { return kernel_width_; }

  void Init(BaseFloat learning_rate, int32 in_height, int32 in_width,
            int32 in_channels, int32 in_pad_height, int32 in_pad_width,
            int32 kernel_height, int32 kernel_width, int32 stride, int32 group,
            int32 out_height, int32 out_width, BaseFloat param_stddev,
            BaseFloat bias_stddev, BaseFloat weight_decay, BaseFloat momentum);
  virtual void InitFromString(std::string args);

  virtual std::string Info() const;
  virtual std::string Type() const { return "ConvolutionComponent"; }
  virtual bool BackpropNeedsInput() const { return true; }
  virtual bool BackpropNeedsOutput() const { return false; }
  using Component::Propagate;
  virtual void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                         const CuMatrixBase<BaseFloat> &in,
                         CuMatrixBase<BaseFloat> *out) const;
  virtual void Scale(BaseFloat scale);
  virtual void Add(BaseFloat alpha, const UpdatableComponent &other);
  virtual void Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                        const CuMatrixBase<BaseFloat> &in_value,
                        const CuMatrixBase<BaseFloat> &out_value,  // dummy
                        const CuMatrixBase<BaseFloat> &out_deriv,
                        Component *to_update,
                        CuMatrix<BaseFloat> *in_deriv) const;
  virtual void SetZero(bool treat_as_gradient);
  virtual void Read(std::istream &is, bool binary);
  virtual void Write(std::ostream &os, bool binary) const;
  virtual BaseFloat DotProduct(const UpdatableComponent &other) const;
  virtual Component *Copy() const;
  virtual void PerturbParams(BaseFloat stddev);
  virtual void SetParams(const VectorBase<BaseFloat> &bias,
                         const MatrixBase<BaseFloat> &linear);
  const CuVector<BaseFloat> &BiasParams() { return bias_params_; }
  const CuMatrix<BaseFloat> &LinearParams() { return linear_params_; }
  virtual int32 GetParameterDim() const;
  virtual void Vectorize(VectorBase<BaseFloat> *params) const;
  virtual void UnVectorize(const VectorBase<BaseFloat> &params);
  void SetWeightDecay(BaseFloat weight_decay) { weight_decay_ = weight_decay; }
  void SetMomentum(BaseFloat momentum) { momentum_ = momentum; }

  // Which data-gradient algorithm the reference's Backprop selects
  // (nnet-component-nnet0.cc:489-497): true = pad out_deriv / flip kernel.
  bool FlipKernelBranch() const;

  // Data-parallel split of Update (see UpdatableComponent).
  virtual int32 NumGradientParams() const { return KernelDim() * group_ + group_; }
  virtual void ComputeGradient(const CuMatrixBase<BaseFloat> &in_value,
                               const CuMatrixBase<BaseFloat> &out_deriv,
                               BaseFloat *grad) const;
  virtual void ApplyGradient(const BaseFloat *grad, int32 num_sample);
  // ApplyGradient's step as a request for the fused backward's reduction
  // (cnslmat/conv-update.h)
  void UpdateRequest(int32 num_sample, ::ConvUpdateEpi *u);
  // dX and the gradient from one pass over out_deriv (hipF_conv2d_backward).
  virtual void BackpropGradient(const ChunkInfo &in_info, const ChunkInfo &out_info,
                                const CuMatrixBase<BaseFloat> &in_value,
                                const CuMatrixBase<BaseFloat> &out_value,
                                const CuMatrixBase<BaseFloat> &out_deriv,
                                CuMatrix<BaseFloat> *in_deriv, BaseFloat *grad) const;

  // Propagate and the Propagate of the channel-only MaxpoolComponent `pool`
  // that consumes `out`, in one pass (hipF_conv2d_maxpool), also writing the
  // pool's routing mask [rows x mask_stride bytes] for
  // MaxpoolComponent::BackpropFromMask.  Returns false, having done nothing,
  // when the pair is not covered (literal path, other pool shapes, ...).
  // store_out = false leaves `out` unwritten (sized, contents stale): the
  // pool's backprop from the mask and this component's Backprop never read
  // it, so a training step does not need it in HBM.
  // pool_stats (nullable, channel-only pools): room for the pooled output's
  // max |value| per frame and per column (cnslmat/pool-stats.h), filled
  // (pool_stats->produced) when the kernel gives them.
  bool PropagateMaxpool(const CuMatrixBase<BaseFloat> &in,
                        CuMatrixBase<BaseFloat> *out,
                        const MaxpoolComponent &pool,
                        CuMatrixBase<BaseFloat> *pool_out, unsigned char *mask,
                        int32 mask_stride, bool store_out = true,
                        PoolStatsOut *pool_stats = NULL) const;

  // Propagate and the Propagate of a RectifiedLinearComponent that consumes
  // `out`, in one pass (hipF_conv2d_relu): relu_out = max(out, 0), `out`
  // itself not written.  Returns false, having done nothing, when the shape
  // takes a forward kernel without the ReLU epilogue.
  bool PropagateRelu(const CuMatrixBase<BaseFloat> &in,
                     CuMatrixBase<BaseFloat> *relu_out) const;

  // The Backprop of `pool` (a MaxpoolComponent fed by this component whose
  // FoldsIntoConvBackprop() holds, forward fused by PropagateMaxpool with
  // routing mask `mask`) followed by this component's Backprop, in one pass
  // (hipF_conv2d_backward_pooled[3d]): pool_deriv is the pool's out_deriv, and
  // the pool's in_deriv (this component's out_deriv) is never stored.
  // grad != NULL: BackpropGradient (gradient out, no update); else Backprop
  // with the update going to to_update.  Returns false, having done nothing,
  // when not covered (the caller then runs the two Backprops).
  bool BackpropPooled(const CuMatrixBase<BaseFloat> &in_value,
                      const MaxpoolComponent &pool, const unsigned char *mask,
                      int32 mask_stride, const CuMatrixBase<BaseFloat> &pool_deriv,
                      Component *to_update, CuMatrix<BaseFloat> *in_deriv,
                      BaseFloat *grad) const;

  // Mutable parameter access for hosts (C-ABI).
  CuMatrix<BaseFloat> &LinearParamsMutable() { return linear_params_; }
  CuVector<BaseFloat> &BiasParamsMutable() { return bias_params_; }
  CuMatrix<BaseFloat> &PrevGradMutable() { return prev_grad_; }
  BaseFloat WeightDecay() const { return weight_decay_; }
  BaseFloat Momentum() const { return momentum_; }

 protected:
  virtual void Update(const CuMatrixBase<BaseFloat> &in_value,
                      const CuMatrixBase<BaseFloat> &out_deriv);
  void PropagateLiteral(const ChunkInfo &in_info,
                        const CuMatrixBase<BaseFloat> &in,
                        CuMatrixBase<BaseFloat> *out) const;
  void BackpropDataLiteral(const CuMatrixBase<BaseFloat> &out_deriv,
                           CuMatrix<BaseFloat> *in_deriv) const;
  void UpdateLiteral(const CuMatrixBase<BaseFloat> &in_value,
                     const CuMatrixBase<BaseFloat> &out_deriv);
  const ConvolutionComponent &operator=(const ConvolutionComponent &other);

  CuMatrix<BaseFloat> linear_params_;
  CuVector<BaseFloat> bias_params_;  // Each group shares a bias value
  bool is_gradient_;
  int32 in_height_;
  int32 in_width_;
  int32 in_channel_;
  int32 in_pad_height_;
  int32 in_pad_width_;
  int32 kernel_height_;
  int32 kernel_width_;
  int32 stride_;
  int32 group_;
  int32 out_height_;
  int32 out_width_;
  BaseFloat weight_decay_;
  BaseFloat momentum_;
  CuMatrix<BaseFloat> prev_grad_;  // for momentum
};

class MaxpoolComponent : public nnet2::Component {
 public:
  void Init(int32 input_dim, int32 output_dim, int32 in_height, int32 in_width,
            int32 in_channel, int32 pool_height_dim, int32 pool_width_dim,
            int32 pool_channel_dim, bool overlap, bool overlap2D);
  explicit MaxpoolComponent(int32 input_dim, int32 output_dim, int32 in_height,
                            int32 in_width, int32 in_channel,
                            int32 pool_height_dim, int32 pool_width_dim,
                            int32 pool_channel_dim, bool overlap,
                            bool overlap2D) {
    Init(input_dim, output_dim, in_height, in_width, in_channel,
         pool_height_dim, pool_width_dim, pool_channel_dim, overlap, overlap2D);
  }
  MaxpoolComponent()
      : input_dim_(0), output_dim_(0), in_height_(0), in_width_(0),
        in_channel_(0), pool_height_dim_(0), pool_width_dim_(0),
        pool_channel_dim_(0), overlap_(false), overlap2D_(false) {}
  virtual std::string Type() const { return "MaxpoolComponent"; }
  virtual void InitFromString(std::string args);
  virtual int32 InputDim() const { return input_dim_; }
  virtual int32 OutputDim() const { return output_dim_; }
  using Component::Propagate;
  virtual void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                         const CuMatrixBase<BaseFloat> &in,
                         CuMatrixBase<BaseFloat> *out) const;
  virtual void Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                        const CuMatrixBase<BaseFloat> &in_value,
                        const CuMatrixBase<BaseFloat> &out_value,
                        const CuMatrixBase<BaseFloat> &out_deriv,
                        Component *to_update,
                        CuMatrix<BaseFloat> *in_deriv) const;
  virtual bool BackpropNeedsInput() const { return true; }
  virtual bool BackpropNeedsOutput() const { return true; }
  virtual Component *Copy() const {
    return new MaxpoolComponent(input_dim_, output_dim_, in_height_, in_width_,
                                in_channel_, pool_height_dim_, pool_width_dim_,
                                pool_channel_dim_, overlap_, overlap2D_);
  }
  virtual void Read(std::istream &is, bool binary);
  virtual void Write(std::ostream &os, bool binary) const;
  virtual std::string Info() const;

  inline int32 In_height() const { return in_height_; }
  inline int32 In_width() const { return in_width_; }
  inline int32 In_channels() const { return in_channel_; }
  // pool_channel_dim when the pool is channel-only (1 x 1 x pc, no overlap,
  // pc in {2, 4, 8}): the shape the convolution forward can fuse; else 0.
  int32 FusableChannelPool() const;
  // A non-overlapping 3-D window (ph*pw > 1) the fused forward can pool from
  // its slab with a 16-bit mask (pc divides 32, ph*pw*pc <= 16): true and
  // the window, else false.
  bool FusableWindow3D(int32 *ph, int32 *pw, int32 *pc) const;
  // Bytes per pooled value of the routing mask the fused forward writes for
  // this pool: 1 (channel-only), 2 (3-D window), 0 = not fusable.
  int32 FusedMaskBytes() const;
  // The windows whose Backprop can run inside the backward of the
  // convolution below (ConvolutionComponent::BackpropPooled): 1 x 1 x pc
  // with pc in {4, 8}, and ph x 1 x pc 3-D windows with ph in {2, 3} and
  // ph * pc <= 16 (c5's P1 3 x 1 x 4).
  bool FoldsIntoConvBackprop() const;
  // Backprop (:882-892) from the routing mask written by
  // ConvolutionComponent::PropagateMaxpool for the same minibatch: identical
  // in_deriv to Backprop(in_value, out_value, out_deriv, ...), without
  // reading in_value / out_value.
  void BackpropFromMask(const unsigned char *mask, int32 mask_stride,
                        const CuMatrixBase<BaseFloat> &out_deriv,
                        CuMatrix<BaseFloat> *in_deriv) const;

 protected:
  int32 input_dim_;
  int32 output_dim_;
  int32 in_height_;
  int32 in_width_;
  int32 in_channel_;
  int32 pool_height_dim_;
  int32 pool_width_dim_;
  int32 pool_channel_dim_;
  bool overlap_;
  bool overlap2D_;
};

class FullyConnectedComponent : public nnet2::AffineComponent {
 public:
  virtual std::string Type() const { return "FullyConnectedComponent"; }
  virtual void Read(std::istream &is, bool binary);
  virtual void Write(std::ostream &os, bool binary) const;
  void Init(BaseFloat learning_rate, int32 input_dim, int32 output_dim,
            BaseFloat param_stddev, BaseFloat bias_stddev,
            BaseFloat weight_decay, BaseFloat momentum);
  virtual void InitFromString(std::string args);
  virtual std::string Info() const;
  virtual Component *Copy() const;
  FullyConnectedComponent() : weight_decay_(0.0002), momentum_(0.9) {}
  void SetWeightDecay(BaseFloat weight_decay) { weight_decay_ = weight_decay; }
  void SetMomentum(BaseFloat momentum) { momentum_ = momentum; }

  virtual void Update(const CuMatrixBase<BaseFloat> &in_value,
                      const CuMatrixBase<BaseFloat> &out_deriv) {
    UpdateSimple(in_value, out_deriv);
  }
  virtual void UpdateSimple(const CuMatrixBase<BaseFloat> &in_value,
                            const CuMatrixBase<BaseFloat> &out_deriv);

  virtual int32 NumGradientParams() const {
    return InputDim() * OutputDim() + OutputDim();
  }
  virtual void ComputeGradient(const CuMatrixBase<BaseFloat> &in_value,
                               const CuMatrixBase<BaseFloat> &out_deriv,
                               BaseFloat *grad) const;
  virtual void ApplyGradient(const BaseFloat *grad, int32 num_sample);
  CuMatrix<BaseFloat> &PrevGradMutable() { return prev_grad_; }
  BaseFloat WeightDecay() const { return weight_decay_; }
  BaseFloat Momentum() const { return momentum_; }

 protected:
  KALDI_DISALLOW_COPY_AND_ASSIGN(FullyConnectedComponent);
  BaseFloat weight_decay_;
  BaseFloat momentum_;
  CuMatrix<BaseFloat> prev_grad_;  // for momentum
};

}  // namespace nnet0
}  // namespace cnsl

#endif  // KCNN_NNET0_NNET_COMPONENT_NNET0_H_
