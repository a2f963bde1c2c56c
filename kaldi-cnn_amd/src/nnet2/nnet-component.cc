// nnet2/nnet-component.cc -- ChunkInfo, the component factory and
// AffineComponent (reference src/nnet2/nnet-component.cc).
#include "nnet-component.h"

#include <math.h>

#include <sstream>

#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/kaldi-io.h"
#include "../nnet0/nnet-component-nnet0.h"
#include "nnet-kernels.h"
#include "parse-from-string.h"

namespace kaldi {
namespace nnet2 {

// ---- ChunkInfo (reference nnet-component.cc:2580-2625) ---------------------
int32 ChunkInfo::GetIndex(int32 offset) const {
  if (offsets_.empty()) return offset - first_offset_;
  for (size_t i = 0; i < offsets_.size(); i++)
    if (offsets_[i] == offset) return (int32)i;
  KALDI_ERR << "could not find offset " << offset;
  return -1;
}
int32 ChunkInfo::GetOffset(int32 index) const {
  if (offsets_.empty()) return first_offset_ + index;
  KALDI_ASSERT(index >= 0 && index < (int32)offsets_.size());
  return offsets_[index];
}
void ChunkInfo::Check() const {
  KALDI_ASSERT((feat_dim_ > 0) && (num_chunks_ > 0));
  if (!offsets_.empty()) {
    KALDI_ASSERT((first_offset_ == offsets_.front()) &&
                 (last_offset_ == offsets_.back()));
  } else {
    KALDI_ASSERT((first_offset_ >= 0) && (last_offset_ >= first_offset_));
    KALDI_ASSERT(last_offset_ - first_offset_ + 1 > (int32)offsets_.size());
  }
  KALDI_ASSERT(NumRows() % num_chunks_ == 0);
}
void ChunkInfo::CheckSize(const CuMatrixBase<BaseFloat> &mat) const {
  KALDI_ASSERT((mat.NumRows() == NumRows()) && (mat.NumCols() == NumCols()));
}

// ---- factory (reference nnet-component.cc:38-136) --------------------------
Component *Component::ReadNew(std::istream &is, bool binary) {
  std::string token;
  ReadToken(is, binary, &token);  // e.g. "<ConvolutionComponent>"
  if (token.size() < 3) KALDI_ERR << "bad component token " << token;
  token.erase(0, 1);
  token.erase(token.length() - 1);
  Component *ans = NewComponentOfType(token);
  if (!ans) KALDI_ERR << "Unknown component type " << token;
  ans->Read(is, binary);
  return ans;
}

Component *Component::NewComponentOfType(const std::string &component_type) {
  Component *ans = NULL;
  if (component_type == "AffineComponent") {
    ans = new AffineComponent();
  } else if (component_type == "ConvolutionComponent") {
    ans = new cnsl::nnet0::ConvolutionComponent();
  } else if (component_type == "MaxpoolComponent") {
    ans = new cnsl::nnet0::MaxpoolComponent();
  } else if (component_type == "FullyConnectedComponent") {
    ans = new cnsl::nnet0::FullyConnectedComponent();
  } else if (component_type == "RectifiedLinearComponent") {
    ans = new RectifiedLinearComponent();
  } else if (component_type == "SpliceComponent") {
    ans = new SpliceComponent();
  }
  return ans;
}

Component *Component::NewFromString(const std::string &initializer_line) {
  std::istringstream istr(initializer_line);
  std::string component_type;
  istr >> component_type >> std::ws;
  std::string rest_of_line;
  getline(istr, rest_of_line);
  Component *ans = NewComponentOfType(component_type);
  if (ans == NULL)
    KALDI_ERR << "Bad initializer line (no such type of Component): "
              << initializer_line;
  try {
    ans->InitFromString(rest_of_line);
  } catch (...) {
    delete ans;
    throw;
  }
  return ans;
}

std::string Component::Info() const {
  std::stringstream stream;
  stream << Type() << ", input-dim=" << InputDim()
         << ", output-dim=" << OutputDim();
  return stream.str();
}

std::string UpdatableComponent::Info() const {
  std::stringstream stream;
  stream << Type() << ", input-dim=" << InputDim()
         << ", output-dim=" << OutputDim() << ", learning-rate=" << LearningRate();
  return stream.str();
}

void ExpectOneOrTwoTokens(std::istream &is, bool binary,
                          const std::string &token1,
                          const std::string &token2) {
  KALDI_ASSERT(token1 != token2);
  std::string temp;
  ReadToken(is, binary, &temp);
  if (temp == token1) {
    ExpectToken(is, binary, token2);
  } else if (temp != token2) {
    KALDI_ERR << "Expecting token " << token1 << " or " << token2
              << " but got " << temp;
  }
}

// ---- ParseFromString (reference nnet-component-nnet0.cc:42-176) -------------
namespace {
template <typename F>
bool ParseGeneric(const std::string &name, std::string *string, F convert) {
  std::vector<std::string> split_string;
  SplitStringToVector(*string, " \t", true, &split_string);
  const std::string name_equals = name + "=";
  const size_t len = name_equals.length();
  for (size_t i = 0; i < split_string.size(); i++) {
    if (split_string[i].compare(0, len, name_equals) == 0) {
      if (!convert(split_string[i].substr(len)))
        KALDI_ERR << "Bad option " << split_string[i];
      *string = "";
      for (size_t j = 0; j < split_string.size(); j++) {
        if (j != i) {
          if (!string->empty()) *string += " ";
          *string += split_string[j];
        }
      }
      return true;
    }
  }
  return false;
}
}  // namespace

bool ParseFromString(const std::string &name, std::string *string,
                     int32 *param) {
  return ParseGeneric(name, string, [&](const std::string &v) {
    return ConvertStringToInteger(v, param);
  });
}
bool ParseFromString(const std::string &name, std::string *string,
                     bool *param) {
  return ParseGeneric(name, string, [&](const std::string &b) {
    if (b.empty()) return false;
    if (b[0] == 'f' || b[0] == 'F') *param = false;
    else if (b[0] == 't' || b[0] == 'T') *param = true;
    else return false;
    return true;
  });
}
bool ParseFromString(const std::string &name, std::string *string,
                     BaseFloat *param) {
  return ParseGeneric(name, string, [&](const std::string &v) {
    return ConvertStringToReal(v, param);
  });
}
bool ParseFromString(const std::string &name, std::string *string,
                     std::string *param) {
  return ParseGeneric(name, string, [&](const std::string &v) {
    *param = v;
    return true;
  });
}
bool ParseFromString(const std::string &name, std::string *string,
                     std::vector<int32> *param) {
  return ParseGeneric(name, string, [&](const std::string &v) {
    return SplitStringToIntegers(v, ":", false, param);
  });
}

// ---- AffineComponent (reference nnet-component.cc:1140-1330) -----------------
AffineComponent::AffineComponent(const AffineComponent &component)
    : UpdatableComponent(component),
      linear_params_(component.linear_params_),
      bias_params_(component.bias_params_),
      is_gradient_(component.is_gradient_) {}

AffineComponent::AffineComponent(const CuMatrixBase<BaseFloat> &linear_params,
                                 const CuVectorBase<BaseFloat> &bias_params,
                                 BaseFloat learning_rate)
    : UpdatableComponent(learning_rate),
      linear_params_(linear_params),
      bias_params_(),
      is_gradient_(false) {
  bias_params_ = bias_params;
  KALDI_ASSERT(linear_params.NumRows() == bias_params.Dim() &&
               bias_params.Dim() != 0);
}

void AffineComponent::Init(BaseFloat learning_rate, int32 input_dim,
                           int32 output_dim, BaseFloat param_stddev,
                           BaseFloat bias_stddev) {
  UpdatableComponent::Init(learning_rate);
  linear_params_.Resize(output_dim, input_dim);
  bias_params_.Resize(output_dim);
  KALDI_ASSERT(output_dim > 0 && input_dim > 0 && param_stddev >= 0.0);
  linear_params_.SetRandn();
  linear_params_.Scale(param_stddev);
  bias_params_.SetRandn();
  bias_params_.Scale(bias_stddev);
}

void AffineComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  bool ok = true;
  BaseFloat learning_rate = learning_rate_;
  int32 input_dim = -1, output_dim = -1;
  ParseFromString("learning-rate", &args, &learning_rate);
  ok = ok && ParseFromString("input-dim", &args, &input_dim);
  ok = ok && ParseFromString("output-dim", &args, &output_dim);
  BaseFloat param_stddev = 1.0 / std::sqrt((double)(input_dim > 0 ? input_dim : 1)),
            bias_stddev = 1.0;
  ParseFromString("param-stddev", &args, &param_stddev);
  ParseFromString("bias-stddev", &args, &bias_stddev);
  if (!args.empty())
    KALDI_ERR << "Could not process these elements in initializer: " << args;
  if (!ok) KALDI_ERR << "Bad initializer " << orig_args;
  Init(learning_rate, input_dim, output_dim, param_stddev, bias_stddev);
}

std::string AffineComponent::Info() const {
  std::stringstream stream;
  const double size = (double)linear_params_.NumRows() * linear_params_.NumCols();
  const double ls = std::sqrt(TraceMatMat(linear_params_, linear_params_, kTrans) / size);
  const double bs = std::sqrt(VecVec(bias_params_, bias_params_) / bias_params_.Dim());
  stream << Type() << ", input-dim=" << InputDim()
         << ", output-dim=" << OutputDim() << ", linear-params-stddev=" << ls
         << ", bias-params-stddev=" << bs
         << ", learning-rate=" << LearningRate();
  return stream.str();
}

// reference nnet-component.cc:1216-1228.
void AffineComponent::Propagate(const ChunkInfo &in_info,
                                const ChunkInfo &out_info,
                                const CuMatrixBase<BaseFloat> &in,
                                CuMatrixBase<BaseFloat> *out) const {
  in_info.CheckSize(in);
  out_info.CheckSize(*out);
  KALDI_ASSERT(in_info.NumChunks() == out_info.NumChunks());
  // CopyRowsFromVec(bias); AddMatMat(1.0, in, kNoTrans, W, kTrans, 1.0), the
  // bias added in the GEMM's store under the f16x3 engine
  out->AddMatMatBias(1.0, in, kNoTrans, linear_params_, kTrans, bias_params_);
}

void AffineComponent::Scale(BaseFloat scale) {
  linear_params_.Scale(scale);
  bias_params_.Scale(scale);
}

void AffineComponent::Add(BaseFloat alpha, const UpdatableComponent &other_in) {
  const AffineComponent *other = dynamic_cast<const AffineComponent *>(&other_in);
  KALDI_ASSERT(other != NULL);
  linear_params_.AddMat(alpha, other->linear_params_);
  bias_params_.AddVec(alpha, other->bias_params_);
}

// reference nnet-component.cc:1230-1234.
void AffineComponent::UpdateSimple(const CuMatrixBase<BaseFloat> &in_value,
                                   const CuMatrixBase<BaseFloat> &out_deriv) {
  bias_params_.AddRowSumMat(learning_rate_, out_deriv, 1.0);
  linear_params_.AddMatMat(learning_rate_, out_deriv, kTrans, in_value,
                           kNoTrans, 1.0);
}

// reference nnet-component.cc:1237-1258.
void AffineComponent::Backprop(const ChunkInfo &, const ChunkInfo &,
                               const CuMatrixBase<BaseFloat> &in_value,
                               const CuMatrixBase<BaseFloat> &,
                               const CuMatrixBase<BaseFloat> &out_deriv,
                               Component *to_update_in,
                               CuMatrix<BaseFloat> *in_deriv) const {
  AffineComponent *to_update = dynamic_cast<AffineComponent *>(to_update_in);
  in_deriv->Resize(out_deriv.NumRows(), InputDim(), kUndefined);
  // f16x3 engine: the two GEMMs' operand statistics (out_deriv's rows and
  // W's columns for the data gradient, out_deriv's columns for the update,
  // and in_value's columns when a fused pool left them pending) in one
  // launch set instead of one per GEMM
  CuGemmBackpropStats stats(out_deriv, linear_params_, to_update != NULL, &in_value);
  in_deriv->AddMatMat(1.0, out_deriv, kNoTrans, linear_params_, kNoTrans, 0.0);
  if (to_update != NULL) {
    if (to_update->is_gradient_)
      to_update->UpdateSimple(in_value, out_deriv);
    else
      to_update->Update(in_value, out_deriv);
  }
}

void AffineComponent::SetZero(bool treat_as_gradient) {
  if (treat_as_gradient) {
    SetLearningRate(1.0);
    is_gradient_ = true;
  }
  linear_params_.SetZero();
  bias_params_.SetZero();
}

// reference nnet-component.cc:1260-1305.
void AffineComponent::Read(std::istream &is, bool binary) {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  ExpectOneOrTwoTokens(is, binary, ostr_beg.str(), "<LearningRate>");
  ReadBasicType(is, binary, &learning_rate_);
  ExpectToken(is, binary, "<LinearParams>");
  linear_params_.Read(is, binary);
  ExpectToken(is, binary, "<BiasParams>");
  bias_params_.Read(is, binary);
  std::string tok;
  ReadToken(is, binary, &tok);
  if (tok == "<AvgInput>") {
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

void AffineComponent::Write(std::ostream &os, bool binary) const {
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
  WriteToken(os, binary, "<IsGradient>");
  WriteBasicType(os, binary, is_gradient_);
  WriteToken(os, binary, ostr_end.str());
}

BaseFloat AffineComponent::DotProduct(const UpdatableComponent &other_in) const {
  const AffineComponent *other = dynamic_cast<const AffineComponent *>(&other_in);
  KALDI_ASSERT(other != NULL);
  return TraceMatMat(linear_params_, other->linear_params_, kTrans) +
         VecVec(bias_params_, other->bias_params_);
}

Component *AffineComponent::Copy() const {
  AffineComponent *ans = new AffineComponent();
  ans->learning_rate_ = learning_rate_;
  ans->linear_params_ = linear_params_;
  ans->bias_params_ = bias_params_;
  ans->is_gradient_ = is_gradient_;
  return ans;
}

void AffineComponent::PerturbParams(BaseFloat stddev) {
  CuMatrix<BaseFloat> temp_linear_params(linear_params_);
  temp_linear_params.SetRandn();
  linear_params_.AddMat(stddev, temp_linear_params);
  CuVector<BaseFloat> temp_bias_params(bias_params_);
  temp_bias_params.SetRandn();
  bias_params_.AddVec(stddev, temp_bias_params);
}

void AffineComponent::SetParams(const VectorBase<BaseFloat> &bias,
                                const MatrixBase<BaseFloat> &linear) {
  bias_params_ = bias;
  linear_params_ = linear;
  KALDI_ASSERT(bias_params_.Dim() == linear_params_.NumRows());
}

int32 AffineComponent::GetParameterDim() const {
  return (InputDim() + 1) * OutputDim();
}
void AffineComponent::Vectorize(VectorBase<BaseFloat> *params) const {
  KALDI_ASSERT(params->Dim() == GetParameterDim());
  Matrix<BaseFloat> W;
  linear_params_.CopyToMat(&W);
  Vector<BaseFloat> b;
  bias_params_.CopyToVec(&b);
  const size_t nw = (size_t)InputDim() * OutputDim();
  std::copy(W.Data(), W.Data() + nw, params->Data());
  std::copy(b.Data(), b.Data() + OutputDim(), params->Data() + nw);
}
void AffineComponent::UnVectorize(const VectorBase<BaseFloat> &params) {
  KALDI_ASSERT(params.Dim() == GetParameterDim());
  Matrix<BaseFloat> W(OutputDim(), InputDim());
  const size_t nw = (size_t)InputDim() * OutputDim();
  std::copy(params.Data(), params.Data() + nw, W.Data());
  Vector<BaseFloat> b(OutputDim());
  std::copy(params.Data() + nw, params.Data() + nw + OutputDim(), b.Data());
  linear_params_.CopyFromMat(W);
  bias_params_.CopyFromVec(b);
}


// ---- NonlinearComponent (reference nnet-component.cc:329-426) ---------------
namespace {
kcnn_stream_t NS() {
  return reinterpret_cast<kcnn_stream_t>(CuDevice::Instantiate().Stream());
}
double *NewDeviceDoubles(int32 n) {
  void *p = CuDevice::Instantiate().Malloc(sizeof(double) * (size_t)n);
  CU_SAFE_CALL(hipMemsetAsync(p, 0, sizeof(double) * (size_t)n,
                              CuDevice::Instantiate().Stream()));
  return static_cast<double *>(p);
}
void FreeDeviceDoubles(double **p) {
  if (*p) CuDevice::Instantiate().Free(*p);
  *p = nullptr;
}
void ReadDeviceDoubles(std::istream &is, bool binary, int32 *dim, double **p) {
  Vector<double> v;
  v.Read(is, binary);
  FreeDeviceDoubles(p);
  *dim = v.Dim();
  if (v.Dim() == 0) return;
  *p = NewDeviceDoubles(v.Dim());
  CU_SAFE_CALL(hipMemcpyAsync(*p, v.Data(), sizeof(double) * v.Dim(), hipMemcpyHostToDevice,
                              CuDevice::Instantiate().Stream()));
  CU_SAFE_CALL(hipStreamSynchronize(CuDevice::Instantiate().Stream()));
}
void DownloadDoubles(const double *p, int32 dim, Vector<double> *v) {
  v->Resize(dim);
  if (dim == 0) return;
  CU_SAFE_CALL(hipMemcpyAsync(v->Data(), p, sizeof(double) * dim, hipMemcpyDeviceToHost,
                              CuDevice::Instantiate().Stream()));
  CU_SAFE_CALL(hipStreamSynchronize(CuDevice::Instantiate().Stream()));
}
}  // namespace

NonlinearComponent::NonlinearComponent(const NonlinearComponent &other)
    : Component(), dim_(other.dim_), stats_dim_(0), value_sum_(nullptr),
      deriv_sum_(nullptr), count_(other.count_) {
  if (other.stats_dim_ > 0) {
    stats_dim_ = other.stats_dim_;
    value_sum_ = NewDeviceDoubles(stats_dim_);
    deriv_sum_ = NewDeviceDoubles(stats_dim_);
    hipStream_t st = CuDevice::Instantiate().Stream();
    CU_SAFE_CALL(hipMemcpyAsync(value_sum_, other.value_sum_, sizeof(double) * stats_dim_,
                                hipMemcpyDeviceToDevice, st));
    CU_SAFE_CALL(hipMemcpyAsync(deriv_sum_, other.deriv_sum_, sizeof(double) * stats_dim_,
                                hipMemcpyDeviceToDevice, st));
  }
}

NonlinearComponent::~NonlinearComponent() {
  FreeDeviceDoubles(&value_sum_);
  FreeDeviceDoubles(&deriv_sum_);
}

void NonlinearComponent::SetDim(int32 dim) {
  KALDI_ASSERT(dim > 0);
  dim_ = dim;
  FreeDeviceDoubles(&value_sum_);
  FreeDeviceDoubles(&deriv_sum_);
  stats_dim_ = 0;
  EnsureStats();
  count_ = 0.0;
}

void NonlinearComponent::EnsureStats() {
  if (stats_dim_ == dim_ && value_sum_ && deriv_sum_) return;
  FreeDeviceDoubles(&value_sum_);
  FreeDeviceDoubles(&deriv_sum_);
  value_sum_ = NewDeviceDoubles(dim_);
  deriv_sum_ = NewDeviceDoubles(dim_);
  stats_dim_ = dim_;
  count_ = 0.0;  // :341-352: resizing the stats restarts the count
}

void NonlinearComponent::Scale(BaseFloat scale) {
  if (stats_dim_ > 0) {
    CNSL_SAFE_CALL(kn_dvec_update(value_sum_, nullptr, 0.0, scale, stats_dim_, NS()));
    CNSL_SAFE_CALL(kn_dvec_update(deriv_sum_, nullptr, 0.0, scale, stats_dim_, NS()));
  }
  count_ *= scale;
}

void NonlinearComponent::Add(BaseFloat alpha, const NonlinearComponent &other) {
  if (other.stats_dim_ > 0) {
    if (stats_dim_ == 0) {
      const double keep = count_;
      EnsureStats();
      count_ = keep;
    }
    KALDI_ASSERT(stats_dim_ == other.stats_dim_);
    CNSL_SAFE_CALL(kn_dvec_update(value_sum_, other.value_sum_, alpha, 1.0, stats_dim_, NS()));
    CNSL_SAFE_CALL(kn_dvec_update(deriv_sum_, other.deriv_sum_, alpha, 1.0, stats_dim_, NS()));
  }
  count_ += alpha * other.count_;
}

void NonlinearComponent::GetValueSum(Vector<double> *v) const {
  DownloadDoubles(value_sum_, stats_dim_, v);
}
void NonlinearComponent::GetDerivSum(Vector<double> *v) const {
  DownloadDoubles(deriv_sum_, stats_dim_, v);
}

void NonlinearComponent::Read(std::istream &is, bool binary) {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  ExpectOneOrTwoTokens(is, binary, ostr_beg.str(), "<Dim>");
  ReadBasicType(is, binary, &dim_);
  ExpectToken(is, binary, "<ValueSum>");
  int32 vd = 0, dd = 0;
  ReadDeviceDoubles(is, binary, &vd, &value_sum_);
  ExpectToken(is, binary, "<DerivSum>");
  ReadDeviceDoubles(is, binary, &dd, &deriv_sum_);
  if (vd != dd) KALDI_ERR << Type() << ": ValueSum/DerivSum sizes differ (" << vd << ", "
                          << dd << ")";
  stats_dim_ = vd;
  ExpectToken(is, binary, "<Count>");
  ReadBasicType(is, binary, &count_);
  ExpectToken(is, binary, ostr_end.str());
}

void NonlinearComponent::Write(std::ostream &os, bool binary) const {
  std::ostringstream ostr_beg, ostr_end;
  ostr_beg << "<" << Type() << ">";
  ostr_end << "</" << Type() << ">";
  WriteToken(os, binary, ostr_beg.str());
  WriteToken(os, binary, "<Dim>");
  WriteBasicType(os, binary, dim_);
  Vector<double> v;
  WriteToken(os, binary, "<ValueSum>");
  GetValueSum(&v);
  v.Write(os, binary);
  WriteToken(os, binary, "<DerivSum>");
  GetDerivSum(&v);
  v.Write(os, binary);
  WriteToken(os, binary, "<Count>");
  WriteBasicType(os, binary, count_);
  WriteToken(os, binary, ostr_end.str());
}

void NonlinearComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  int32 dim;
  bool ok = ParseFromString("dim", &args, &dim);
  if (!ok || !args.empty() || dim <= 0)
    KALDI_ERR << "Invalid initializer for layer of type " << Type() << ": \""
              << orig_args << "\"";
  Init(dim);
}

// ---- RectifiedLinearComponent (reference nnet-component.cc:799-827) ---------
void RectifiedLinearComponent::Propagate(const ChunkInfo &in_info,
                                         const ChunkInfo &out_info,
                                         const CuMatrixBase<BaseFloat> &in,
                                         CuMatrixBase<BaseFloat> *out) const {
  in_info.CheckSize(in);
  out_info.CheckSize(*out);
  // out->CopyFromMat(in); out->ApplyFloor(0.0) -- one pass
  CNSL_SAFE_CALL(kn_relu_prop(in.Data(), in.Dim(), out->Data(), out->Dim(), NS()));
}

void RectifiedLinearComponent::Backprop(const ChunkInfo &, const ChunkInfo &,
                                        const CuMatrixBase<BaseFloat> &,
                                        const CuMatrixBase<BaseFloat> &out_value,
                                        const CuMatrixBase<BaseFloat> &out_deriv,
                                        Component *to_update,
                                        CuMatrix<BaseFloat> *in_deriv) const {
  in_deriv->Resize(out_deriv.NumRows(), out_deriv.NumCols(), kUndefined);
  // CopyFromMat(out_value); ApplyHeaviside(); UpdateStats(out_value, in_deriv)
  // on to_update; MulElements(out_deriv) -- one pass plus the stat reduction.
  NonlinearComponent *u = to_update ? dynamic_cast<NonlinearComponent *>(to_update) : nullptr;
  double *vs = nullptr, *ds = nullptr;
  size_t ws_bytes = 0;
  if (u != nullptr) {
    KALDI_ASSERT(out_value.NumCols() == u->InputDim());
    u->EnsureStats();
    u->count_ += out_value.NumRows();
    vs = u->value_sum_;
    ds = u->deriv_sum_;
    ws_bytes = kn_relu_stats_ws(out_deriv.Dim());
  }
  void *ws = ws_bytes ? CuDevice::Instantiate().Malloc(ws_bytes) : nullptr;
  const int rc = kn_relu_backprop(out_value.Data(), out_value.Dim(), out_deriv.Data(),
                                  out_deriv.Dim(), in_deriv->Data(), in_deriv->Dim(), vs,
                                  ds, ws, NS());
  if (ws) CuDevice::Instantiate().Free(ws);
  CNSL_SAFE_CALL(rc);
}

// ---- SpliceComponent (reference nnet-component.cc:2524-2866) ----------------
std::string SpliceComponent::Info() const {
  std::stringstream stream;
  std::ostringstream os;
  for (int32 c : context_) os << c << " ";
  stream << Component::Info() << ", context=" << os.str();
  if (const_component_dim_ != 0)
    stream << ", const_component_dim=" << const_component_dim_;
  return stream.str();
}

void SpliceComponent::Init(int32 input_dim, std::vector<int32> context,
                           int32 const_component_dim) {
  input_dim_ = input_dim;
  const_component_dim_ = const_component_dim;
  context_ = context;
  KALDI_ASSERT(context_.size() > 0);
  KALDI_ASSERT(input_dim_ > 0 && context_.front() <= 0 && context_.back() >= 0);
  for (size_t i = 1; i < context_.size(); i++)  // IsSortedAndUniq
    KALDI_ASSERT(context_[i - 1] < context_[i]);
  KALDI_ASSERT(const_component_dim_ >= 0 && const_component_dim_ < input_dim_);
  if ((int)context_.size() > KN_SPLICE_MAX_CONTEXT)
    KALDI_ERR << "SpliceComponent: at most " << KN_SPLICE_MAX_CONTEXT
              << " context offsets supported, got " << context_.size();
}

void SpliceComponent::InitFromString(std::string args) {
  std::string orig_args(args);
  int32 input_dim, left_context, right_context;
  std::vector<int32> context;
  bool in_dim_ok = ParseFromString("input-dim", &args, &input_dim);
  bool context_ok = ParseFromString("context", &args, &context);
  bool left_right_context_ok = ParseFromString("left-context", &args, &left_context) &&
                               ParseFromString("right-context", &args, &right_context);
  int32 const_component_dim = 0;
  ParseFromString("const-component-dim", &args, &const_component_dim);
  if (!(in_dim_ok && (context_ok || left_right_context_ok)) || !args.empty() ||
      input_dim <= 0)
    KALDI_ERR << "Invalid initializer for layer of type " << Type() << ": \""
              << orig_args << "\"";
  if (left_right_context_ok) {
    KALDI_ASSERT(context.size() == 0);
    for (int32 i = -left_context; i <= right_context; i++) context.push_back(i);
  }
  Init(input_dim, context, const_component_dim);
}

int32 SpliceComponent::OutputDim() const {
  return (input_dim_ - const_component_dim_) * (int32)context_.size() +
         const_component_dim_;
}

namespace {
// The splice geometry of a pair of ChunkInfos.  Contiguous offsets (every
// chunk info of a contiguous context) use the arithmetic form; otherwise
// (a gapped context deeper in a stack) the row table of in-chunk indices,
// ChunkInfo::GetIndex(out offset + context[c]) as in the reference's index
// vectors (nnet-component.cc:2670-2681).
kn_splice_geom SpliceGeom(const ChunkInfo &in_info, const ChunkInfo &out_info,
                          const std::vector<int32> &context, int32 input_dim,
                          int32 const_dim) {
  in_info.Check();
  out_info.Check();
  KALDI_ASSERT(in_info.NumChunks() == out_info.NumChunks());
  const int32 in_cs = in_info.ChunkSize(), out_cs = out_info.ChunkSize();
  if (out_cs <= 0)
    KALDI_ERR << "Splicing features: output will have zero dimension. "
              << "Probably a code error.";
  kn_splice_geom g;
  g.num_chunks = in_info.NumChunks();
  g.in_cs = in_cs;
  g.out_cs = out_cs;
  g.in_first = in_info.GetOffset(0);
  g.out_first = out_info.GetOffset(0);
  g.const_dim = const_dim;
  g.dim = input_dim - const_dim;
  g.num_splice = (int)context.size();
  if (g.num_splice > KN_SPLICE_MAX_CONTEXT)
    KALDI_ERR << "SpliceComponent: more than " << KN_SPLICE_MAX_CONTEXT << " spliced frames";
  const bool contiguous = in_info.GetOffset(in_cs - 1) - g.in_first + 1 == in_cs &&
                          out_info.GetOffset(out_cs - 1) - g.out_first + 1 == out_cs;
  g.table = contiguous ? 0 : 1;
  if (!contiguous && (int64_t)g.num_splice * out_cs > KN_SPLICE_MAX_TAB)
    KALDI_ERR << "SpliceComponent: " << g.num_splice << " x " << out_cs
              << " spliced rows per chunk exceed the row table (" << KN_SPLICE_MAX_TAB << ")";
  for (int c = 0; c < g.num_splice; c++) {
    g.context[c] = context[c];
    if (contiguous) {
      // every spliced frame must exist in the input chunk (GetIndex asserts)
      (void)in_info.GetIndex(g.out_first + context[c]);
      (void)in_info.GetIndex(out_info.GetOffset(out_cs - 1) + context[c]);
    } else {
      for (int32 oi = 0; oi < out_cs; oi++)
        g.in_index[c * out_cs + oi] =
            (short)in_info.GetIndex(out_info.GetOffset(oi) + context[c]);
    }
  }
  return g;
}
}  // namespace

void SpliceComponent::Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                                const CuMatrixBase<BaseFloat> &in,
                                CuMatrixBase<BaseFloat> *out) const {
  in_info.CheckSize(in);
  out_info.CheckSize(*out);
  kn_splice_geom g = SpliceGeom(in_info, out_info, context_, input_dim_,
                                const_component_dim_);
  CNSL_SAFE_CALL(kn_splice_prop(in.Data(), in.Dim(), out->Data(), out->Dim(), g, NS()));
}

void SpliceComponent::Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                               const CuMatrixBase<BaseFloat> &,
                               const CuMatrixBase<BaseFloat> &,
                               const CuMatrixBase<BaseFloat> &out_deriv, Component *,
                               CuMatrix<BaseFloat> *in_deriv) const {
  out_info.CheckSize(out_deriv);
  in_deriv->Resize(in_info.NumRows(), in_info.NumCols(), kUndefined);
  KALDI_ASSERT(OutputDim() == out_deriv.NumCols());
  kn_splice_geom g = SpliceGeom(in_info, out_info, context_, input_dim_,
                                const_component_dim_);
  CNSL_SAFE_CALL(kn_splice_backprop(out_deriv.Data(), out_deriv.Dim(), in_deriv->Data(),
                                    in_deriv->Dim(), g, NS()));
}

Component *SpliceComponent::Copy() const {
  SpliceComponent *ans = new SpliceComponent();
  ans->input_dim_ = input_dim_;
  ans->context_ = context_;
  ans->const_component_dim_ = const_component_dim_;
  return ans;
}

void SpliceComponent::Read(std::istream &is, bool binary) {
  ExpectOneOrTwoTokens(is, binary, "<SpliceComponent>", "<InputDim>");
  ReadBasicType(is, binary, &input_dim_);
  std::string token;
  ReadToken(is, false, &token);
  if (token == "<LeftContext>") {
    int32 left_context = 0, right_context = 0;
    std::vector<int32> context;
    ReadBasicType(is, binary, &left_context);
    ExpectToken(is, binary, "<RightContext>");
    ReadBasicType(is, binary, &right_context);
    for (int32 i = -1 * left_context; i <= right_context; i++) context.push_back(i);
    context_ = context;
  } else if (token == "<Context>") {
    ReadIntegerVector(is, binary, &context_);
  } else {
    KALDI_ERR << "Unknown token" << token << ", the model might be corrupted";
  }
  ExpectToken(is, binary, "<ConstComponentDim>");
  ReadBasicType(is, binary, &const_component_dim_);
  ExpectToken(is, binary, "</SpliceComponent>");
}

void SpliceComponent::Write(std::ostream &os, bool binary) const {
  WriteToken(os, binary, "<SpliceComponent>");
  WriteToken(os, binary, "<InputDim>");
  WriteBasicType(os, binary, input_dim_);
  WriteToken(os, binary, "<Context>");
  WriteIntegerVector(os, binary, context_);
  WriteToken(os, binary, "<ConstComponentDim>");
  WriteBasicType(os, binary, const_component_dim_);
  WriteToken(os, binary, "</SpliceComponent>");
}

}  // namespace nnet2
}  // namespace kaldi
