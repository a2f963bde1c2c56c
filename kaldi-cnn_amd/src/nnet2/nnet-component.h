// nnet2/nnet-component.h -- the nnet2 plugin API the CNN components implement
// (reference src/nnet2/nnet-component.h: ChunkInfo :72-146, Component
// :157-269, UpdatableComponent :279-348, AffineComponent :843-941) and the
// factory hook the reference added (nnet-component.cc:112-117).  Only the
// classes the CNN path needs are provided; the other ~30 upstream nnet2
// component types are out of scope.
#ifndef KCNN_NNET2_NNET_COMPONENT_H_
#define KCNN_NNET2_NNET_COMPONENT_H_

#include <iostream>
#include <string>
#include <vector>

#include "../kaldi-lite/cu-matrix.h"
#include "../kaldi-lite/kaldi-common.h"

namespace kaldi {
namespace nnet2 {

class ChunkInfo {
 public:
  ChunkInfo() : feat_dim_(0), num_chunks_(0), first_offset_(0), last_offset_(0) {}
  ChunkInfo(int32 feat_dim, int32 num_chunks, int32 first_offset,
            int32 last_offset)
      : feat_dim_(feat_dim), num_chunks_(num_chunks),
        first_offset_(first_offset), last_offset_(last_offset) { Check(); }
  ChunkInfo(int32 feat_dim, int32 num_chunks, const std::vector<int32> offsets)
      : feat_dim_(feat_dim), num_chunks_(num_chunks),
        first_offset_(offsets.front()), last_offset_(offsets.back()),
        offsets_(offsets) {
    if (last_offset_ - first_offset_ + 1 == (int32)offsets_.size())
      offsets_.clear();
    Check();
  }
  int32 GetIndex(int32 offset) const;
  int32 GetOffset(int32 index) const;
  void MakeOffsetsContiguous() { offsets_.clear(); Check(); }
  inline int32 ChunkSize() const { return NumRows() / num_chunks_; }
  inline int32 NumChunks() const { return num_chunks_; }
  int32 NumRows() const {
    return num_chunks_ * (!offsets_.empty() ? (int32)offsets_.size()
                                            : last_offset_ - first_offset_ + 1);
  }
  int32 NumCols() const { return feat_dim_; }
  void CheckSize(const CuMatrixBase<BaseFloat> &mat) const;
  void Check() const;

 private:
  int32 feat_dim_, num_chunks_, first_offset_, last_offset_;
  std::vector<int32> offsets_;
};

class Component {
 public:
  Component() : index_(-1) {}
  virtual ~Component() {}
  virtual std::string Type() const = 0;
  virtual int32 Index() const { return index_; }
  virtual void SetIndex(int32 index) { index_ = index; }
  virtual void InitFromString(std::string args) = 0;
  virtual int32 InputDim() const = 0;
  virtual int32 OutputDim() const = 0;
  virtual std::vector<int32> Context() const { return std::vector<int32>(1, 0); }

  virtual void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                         const CuMatrixBase<BaseFloat> &in,
                         CuMatrixBase<BaseFloat> *out) const = 0;
  /// Non-virtual propagate that first resizes the output if necessary
  /// (reference nnet-component.h:203-215).
  void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                 const CuMatrixBase<BaseFloat> &in,
                 CuMatrix<BaseFloat> *out) const {
    if (out->NumRows() != out_info.NumRows() ||
        out->NumCols() != out_info.NumCols())
      out->Resize(out_info.NumRows(), out_info.NumCols());
    Propagate(in_info, out_info, in, static_cast<CuMatrixBase<BaseFloat> *>(out));
  }
  virtual void Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                        const CuMatrixBase<BaseFloat> &in_value,
                        const CuMatrixBase<BaseFloat> &out_value,
                        const CuMatrixBase<BaseFloat> &out_deriv,
                        Component *to_update,
                        CuMatrix<BaseFloat> *in_deriv) const = 0;
  virtual bool BackpropNeedsInput() const { return true; }
  virtual bool BackpropNeedsOutput() const { return true; }

  static Component *ReadNew(std::istream &is, bool binary);
  virtual Component *Copy() const = 0;
  static Component *NewFromString(const std::string &initializer_line);
  static Component *NewComponentOfType(const std::string &type);
  virtual void Read(std::istream &is, bool binary) = 0;
  virtual void Write(std::ostream &os, bool binary) const = 0;
  virtual std::string Info() const;

 private:
  int32 index_;
  KALDI_DISALLOW_COPY_AND_ASSIGN(Component);
};

class UpdatableComponent : public Component {
 public:
  UpdatableComponent(const UpdatableComponent &other)
      : Component(), learning_rate_(other.learning_rate_) {}
  void Init(BaseFloat learning_rate) { learning_rate_ = learning_rate; }
  UpdatableComponent(BaseFloat learning_rate) { Init(learning_rate); }
  UpdatableComponent() : learning_rate_(0.001) {}
  virtual ~UpdatableComponent() {}
  virtual void SetZero(bool treat_as_gradient) = 0;
  virtual BaseFloat DotProduct(const UpdatableComponent &other) const = 0;
  virtual void PerturbParams(BaseFloat stddev) = 0;
  virtual void Scale(BaseFloat scale) = 0;
  virtual void Add(BaseFloat alpha, const UpdatableComponent &other) = 0;
  void SetLearningRate(BaseFloat lrate) { learning_rate_ = lrate; }
  BaseFloat LearningRate() const { return learning_rate_; }
  virtual std::string Info() const;
  virtual int32 GetParameterDim() const { KALDI_ASSERT(0); return 0; }
  virtual void Vectorize(VectorBase<BaseFloat> *params) const { (void)params; KALDI_ASSERT(0); }
  virtual void UnVectorize(const VectorBase<BaseFloat> &params) { (void)params; KALDI_ASSERT(0); }

  // ---- data-parallel extension (MI355X build) ---------------------------
  // The reference applies its update inside Backprop (Update on to_update).
  // Data parallelism needs the raw gradient between the two halves of that
  // update so it can be all-reduced; these split it:
  //   NumGradientParams()  floats of the flat gradient (linear then bias),
  //   ComputeGradient()    writes the local-batch gradient (unscaled sums),
  //   ApplyGradient()      the reference's update math with num_sample =
  //                        the global batch size.
  // Update(in, out_deriv) == ComputeGradient + ApplyGradient(in.NumRows()).
  virtual int32 NumGradientParams() const { return 0; }
  virtual void ComputeGradient(const CuMatrixBase<BaseFloat> &in_value,
                               const CuMatrixBase<BaseFloat> &out_deriv,
                               BaseFloat *grad) const {
    (void)in_value; (void)out_deriv; (void)grad;
    KALDI_ERR << Type() << " does not support ComputeGradient";
  }
  virtual void ApplyGradient(const BaseFloat *grad, int32 num_sample) {
    (void)grad; (void)num_sample;
    KALDI_ERR << Type() << " does not support ApplyGradient";
  }
  // Backprop without update (in_deriv nullable) + ComputeGradient in one
  // call; components with a fused backward kernel override it.
  virtual void BackpropGradient(const ChunkInfo &in_info, const ChunkInfo &out_info,
                                const CuMatrixBase<BaseFloat> &in_value,
                                const CuMatrixBase<BaseFloat> &out_value,
                                const CuMatrixBase<BaseFloat> &out_deriv,
                                CuMatrix<BaseFloat> *in_deriv, BaseFloat *grad) const {
    if (in_deriv != NULL)
      Backprop(in_info, out_info, in_value, out_value, out_deriv, NULL, in_deriv);
    ComputeGradient(in_value, out_deriv, grad);
  }

 protected:
  BaseFloat learning_rate_;

 private:
  const UpdatableComponent &operator=(const UpdatableComponent &other);
};

// reference nnet-component.h:843-941, nnet-component.cc:1140-1330.
class AffineComponent : public UpdatableComponent {
  friend class AffineComponentPreconditioned;

 public:
  explicit AffineComponent(const AffineComponent &other);
  AffineComponent(const CuMatrixBase<BaseFloat> &linear_params,
                  const CuVectorBase<BaseFloat> &bias_params,
                  BaseFloat learning_rate);
  AffineComponent() : is_gradient_(false) {}
  virtual int32 InputDim() const { return linear_params_.NumCols(); }
  virtual int32 OutputDim() const { return linear_params_.NumRows(); }
  void Init(BaseFloat learning_rate, int32 input_dim, int32 output_dim,
            BaseFloat param_stddev, BaseFloat bias_stddev);
  virtual void InitFromString(std::string args);
  virtual std::string Info() const;
  virtual std::string Type() const { return "AffineComponent"; }
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
                        const CuMatrixBase<BaseFloat> &out_value,
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

  // Mutable access for hosts that move parameters in and out (C-ABI).
  CuMatrix<BaseFloat> &LinearParamsMutable() { return linear_params_; }
  CuVector<BaseFloat> &BiasParamsMutable() { return bias_params_; }

 protected:
  virtual void Update(const CuMatrixBase<BaseFloat> &in_value,
                      const CuMatrixBase<BaseFloat> &out_deriv) {
    UpdateSimple(in_value, out_deriv);
  }
  virtual void UpdateSimple(const CuMatrixBase<BaseFloat> &in_value,
                            const CuMatrixBase<BaseFloat> &out_deriv);
  const AffineComponent &operator=(const AffineComponent &other);

  CuMatrix<BaseFloat> linear_params_;  // [output_dim x input_dim]
  CuVector<BaseFloat> bias_params_;
  bool is_gradient_;
};

// ---- the upstream nnet2 components either side of the CNN path -----------
// (SpliceComponent feeds the first convolution,
// RectifiedLinearComponent follows each one in egs/exp/nnet/nnet.config.)

// reference nnet-component.h:351-409, nnet-component.cc:329-426.  The
// diagnostic stats live on the device as fp64 vectors, as CuVector<double>
// does upstream; they are allocated by the first UpdateStats (or Read).
class NonlinearComponent : public Component {
 public:
  void Init(int32 dim) { dim_ = dim; count_ = 0.0; }
  explicit NonlinearComponent(int32 dim) : value_sum_(nullptr), deriv_sum_(nullptr) {
    Init(dim);
  }
  NonlinearComponent() : dim_(0), stats_dim_(0), value_sum_(nullptr),
                         deriv_sum_(nullptr), count_(0.0) {}
  explicit NonlinearComponent(const NonlinearComponent &other);
  virtual ~NonlinearComponent();
  virtual int32 InputDim() const { return dim_; }
  virtual int32 OutputDim() const { return dim_; }
  virtual void InitFromString(std::string args);
  virtual void Read(std::istream &is, bool binary);
  virtual void Write(std::ostream &os, bool binary) const;
  void Scale(BaseFloat scale);
  void Add(BaseFloat alpha, const NonlinearComponent &other);
  // Host copies of the stats (ValueSum()/DerivSum() upstream return the
  // CuVector<double>); empty until the first UpdateStats.
  void GetValueSum(Vector<double> *v) const;
  void GetDerivSum(Vector<double> *v) const;
  double Count() const { return count_; }
  void SetDim(int32 dim);

 protected:
  friend class RectifiedLinearComponent;  // UpdateStats on to_update (:821)
  // Make the fp64 stat vectors dim_ long (zeroed) if they are not.
  void EnsureStats();
  int32 dim_;
  int32 stats_dim_;     // length of value_sum_/deriv_sum_ (0 = empty)
  double *value_sum_;   // device, stats of the output
  double *deriv_sum_;   // device, stats of the nonlinearity's derivative
  double count_;

 private:
  const NonlinearComponent &operator=(const NonlinearComponent &other);
};

// reference nnet-component.h:676-698, nnet-component.cc:799-827.
class RectifiedLinearComponent : public NonlinearComponent {
 public:
  explicit RectifiedLinearComponent(int32 dim) : NonlinearComponent(dim) {}
  explicit RectifiedLinearComponent(const RectifiedLinearComponent &other)
      : NonlinearComponent(other) {}
  RectifiedLinearComponent() {}
  virtual std::string Type() const { return "RectifiedLinearComponent"; }
  virtual Component *Copy() const { return new RectifiedLinearComponent(*this); }
  virtual bool BackpropNeedsInput() const { return false; }
  virtual bool BackpropNeedsOutput() const { return true; }
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

 private:
  RectifiedLinearComponent &operator=(const RectifiedLinearComponent &other);
};

// reference nnet-component.h:1092-1129, nnet-component.cc:2524-2866.
class SpliceComponent : public Component {
 public:
  SpliceComponent() : input_dim_(0), const_component_dim_(0) {}
  void Init(int32 input_dim, std::vector<int32> context, int32 const_component_dim = 0);
  virtual std::string Type() const { return "SpliceComponent"; }
  virtual std::string Info() const;
  virtual void InitFromString(std::string args);
  virtual int32 InputDim() const { return input_dim_; }
  virtual int32 OutputDim() const;
  virtual std::vector<int32> Context() const { return context_; }
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
  virtual bool BackpropNeedsInput() const { return false; }
  virtual bool BackpropNeedsOutput() const { return false; }
  virtual Component *Copy() const;
  virtual void Read(std::istream &is, bool binary);
  virtual void Write(std::ostream &os, bool binary) const;

 private:
  KALDI_DISALLOW_COPY_AND_ASSIGN(SpliceComponent);
  int32 input_dim_;
  std::vector<int32> context_;
  int32 const_component_dim_;
};

/// Shared by the components' Read functions (nnet-component-nnet0.cc:24-39).
void ExpectOneOrTwoTokens(std::istream &is, bool binary,
                          const std::string &token1, const std::string &token2);

}  // namespace nnet2
}  // namespace kaldi

#endif  // KCNN_NNET2_NNET_COMPONENT_H_
