// nnet2/nnet-component.cc -- ChunkInfo, the component factory and
// AffineComponent (reference src/nnet2/nnet-component.cc).
#include "nnet-component.h"

#include <math.h>

#include <sstream>

#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/kaldi-io.h"
#include "../nnet0/nnet-component-nnet0.h"
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
  out->CopyRowsFromVec(bias_params_);
  out->AddMatMat(1.0, in, kNoTrans, linear_params_, kTrans, 1.0);
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

}  // namespace nnet2
}  // namespace kaldi
