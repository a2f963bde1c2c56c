// kaldi-lite/cu-matrix.cc -- generic CuMatrix/CuVector methods on HIP.
#include "cu-matrix.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <limits>
#include <mutex>
#include <sstream>

#include "cu-device.h"
#include "cu-kernels-lite.h"
#include "../cnslmat/pool-stats.h"
#include "kaldi-io.h"

namespace kaldi {

namespace {
inline kcnn_stream_t S() {
  return reinterpret_cast<kcnn_stream_t>(CuDevice::Instantiate().Stream());
}
inline MatrixIndexT PaddedStride(MatrixIndexT cols) {
  return (cols + 15) / 16 * 16;
}
::MatrixDim VecDim(MatrixIndexT n) {
  ::MatrixDim d;
  d.rows = 1; d.cols = n; d.stride = n;
  return d;
}

// splitmix64 -> Box-Muller (double), deterministic per process.
std::mutex g_rng_mu;
uint64_t g_rng_state = 20261015ull;
uint64_t splitmix64() {
  uint64_t z = (g_rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
}  // namespace

void SetRandnSeed(uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_rng_mu);
  g_rng_state = seed;
}

void RandnFill(float *dst, size_t n) {
  std::lock_guard<std::mutex> lk(g_rng_mu);
  for (size_t i = 0; i < n; i += 2) {
    const double u1 = ((splitmix64() >> 11) + 1.0) * (1.0 / 9007199254740993.0);
    const double u2 = (splitmix64() >> 11) * (1.0 / 9007199254740992.0);
    const double r = sqrt(-2.0 * log(u1));
    dst[i] = (float)(r * cos(2.0 * M_PI * u2));
    if (i + 1 < n) dst[i + 1] = (float)(r * sin(2.0 * M_PI * u2));
  }
}

// ---------------------------------------------------------------------------
// Host containers: Kaldi text/binary formats (upstream matrix/kaldi-matrix.cc,
// kaldi-vector.cc).
template <typename Real>
void MatrixBase<Real>::Write(std::ostream &os, bool binary) const {
  if (binary) {
    WriteToken(os, binary, sizeof(Real) == 4 ? "FM" : "DM");
    WriteBasicType(os, binary, (int32)rows_);
    WriteBasicType(os, binary, (int32)cols_);
    os.write(reinterpret_cast<const char *>(data_.data()),
             sizeof(Real) * data_.size());
  } else {
    if (cols_ == 0) {
      os << " [ ]\n";
    } else {
      os << " [";
      os.precision(std::numeric_limits<Real>::max_digits10);
      for (MatrixIndexT i = 0; i < rows_; i++) {
        os << "\n  ";
        for (MatrixIndexT j = 0; j < cols_; j++) os << (*this)(i, j) << " ";
      }
      os << "]\n";
    }
  }
  if (os.fail()) KALDI_ERR << "failed to write matrix";
}

template <typename Real>
void MatrixBase<Real>::Read(std::istream &is, bool binary) {
  if (binary) {
    std::string tok;
    ReadToken(is, binary, &tok);
    if (tok != (sizeof(Real) == 4 ? "FM" : "DM"))
      KALDI_ERR << "expected matrix token FM, got " << tok;
    int32 r, c;
    ReadBasicType(is, binary, &r);
    ReadBasicType(is, binary, &c);
    Resize(r, c);
    is.read(reinterpret_cast<char *>(data_.data()), sizeof(Real) * data_.size());
    if (is.fail()) KALDI_ERR << "failed to read matrix data";
    return;
  }
  std::string tok;
  is >> tok;
  if (tok != "[") KALDI_ERR << "expected '[' reading text matrix, got " << tok;
  std::vector<std::vector<Real>> rows;
  std::string line;
  std::getline(is, line);  // rest of the "[" line
  bool done = false;
  {
    std::istringstream ls(line);
    std::string t;
    while (ls >> t) {
      if (t == "]") { done = true; break; }
      KALDI_ERR << "unexpected '" << t << "' after '['";
    }
  }
  while (!done && std::getline(is, line)) {
    std::istringstream ls(line);
    std::vector<Real> row;
    std::string t;
    while (ls >> t) {
      if (t == "]") { done = true; break; }
      float v;
      if (!ConvertStringToReal(t, &v)) KALDI_ERR << "bad matrix element " << t;
      row.push_back((Real)v);
    }
    if (!row.empty()) rows.push_back(row);
  }
  if (!done) KALDI_ERR << "unterminated text matrix";
  const MatrixIndexT r = (MatrixIndexT)rows.size();
  const MatrixIndexT c = r ? (MatrixIndexT)rows[0].size() : 0;
  Resize(r, c);
  for (MatrixIndexT i = 0; i < r; i++) {
    if ((MatrixIndexT)rows[i].size() != c) KALDI_ERR << "ragged text matrix";
    for (MatrixIndexT j = 0; j < c; j++) (*this)(i, j) = rows[i][j];
  }
}

template <typename Real>
void VectorBase<Real>::Write(std::ostream &os, bool binary) const {
  if (binary) {
    WriteToken(os, binary, sizeof(Real) == 4 ? "FV" : "DV");
    WriteBasicType(os, binary, (int32)data_.size());
    os.write(reinterpret_cast<const char *>(data_.data()),
             sizeof(Real) * data_.size());
  } else {
    os.precision(std::numeric_limits<Real>::max_digits10);
    os << " [ ";
    for (auto v : data_) os << v << " ";
    os << "]\n";
  }
  if (os.fail()) KALDI_ERR << "failed to write vector";
}

template <typename Real>
void VectorBase<Real>::Read(std::istream &is, bool binary) {
  if (binary) {
    std::string tok;
    ReadToken(is, binary, &tok);
    if (tok != (sizeof(Real) == 4 ? "FV" : "DV"))
      KALDI_ERR << "expected vector token FV, got " << tok;
    int32 d;
    ReadBasicType(is, binary, &d);
    Resize(d);
    is.read(reinterpret_cast<char *>(data_.data()), sizeof(Real) * d);
    if (is.fail()) KALDI_ERR << "failed to read vector data";
    return;
  }
  std::string tok;
  is >> tok;
  if (tok != "[") KALDI_ERR << "expected '[' reading text vector, got " << tok;
  data_.clear();
  while (is >> tok) {
    if (tok == "]") return;
    char *end = nullptr;
    const double v = strtod(tok.c_str(), &end);
    if (tok.empty() || *end != '\0') KALDI_ERR << "bad vector element " << tok;
    data_.push_back((Real)v);
  }
  KALDI_ERR << "unterminated text vector";
}

// ---------------------------------------------------------------------------
template <typename Real>
void CuMatrixBase<Real>::SetZero() {
  if (num_rows_ == 0 || num_cols_ == 0) return;
  CU_SAFE_CALL(hipMemset2DAsync(data_, sizeof(Real) * stride_, 0,
                                sizeof(Real) * num_cols_, num_rows_,
                                CuDevice::Instantiate().Stream()));
}
template <typename Real>
void CuMatrixBase<Real>::Set(Real v) { CNSL_SAFE_CALL(kl_set(data_, Dim(), v, S())); }
template <typename Real>
void CuMatrixBase<Real>::Add(Real v) { CNSL_SAFE_CALL(kl_add(data_, Dim(), v, S())); }
template <typename Real>
void CuMatrixBase<Real>::Scale(Real v) { CNSL_SAFE_CALL(kl_scale(data_, Dim(), v, S())); }

template <typename Real>
void CuMatrixBase<Real>::SetRandn() {
  Matrix<Real> h(num_rows_, num_cols_);
  RandnFill(h.Data(), (size_t)num_rows_ * num_cols_);
  CopyFromMat(h);
}

template <typename Real>
void CuMatrixBase<Real>::CopyFromMat(const CuMatrixBase<Real> &src,
                                     MatrixTransposeType trans) {
  if (trans == kNoTrans) {
    KALDI_ASSERT(src.NumRows() == num_rows_ && src.NumCols() == num_cols_);
    if (num_rows_ == 0 || num_cols_ == 0) return;
    CU_SAFE_CALL(hipMemcpy2DAsync(data_, sizeof(Real) * stride_, src.Data(),
                                  sizeof(Real) * src.Stride(),
                                  sizeof(Real) * num_cols_, num_rows_,
                                  hipMemcpyDeviceToDevice,
                                  CuDevice::Instantiate().Stream()));
  } else {
    KALDI_ASSERT(src.NumCols() == num_rows_ && src.NumRows() == num_cols_);
    CNSL_SAFE_CALL(kl_add_mat(1.0f, src.Data(), src.Dim(), 1, 0.0f, data_, Dim(), S()));
  }
}

template <typename Real>
void CuMatrixBase<Real>::CopyFromMat(const MatrixBase<Real> &src) {
  KALDI_ASSERT(src.NumRows() == num_rows_ && src.NumCols() == num_cols_);
  if (num_rows_ == 0 || num_cols_ == 0) return;
  CU_SAFE_CALL(hipMemcpy2DAsync(data_, sizeof(Real) * stride_, src.Data(),
                                sizeof(Real) * src.Stride(),
                                sizeof(Real) * num_cols_, num_rows_,
                                hipMemcpyHostToDevice,
                                CuDevice::Instantiate().Stream()));
  CuDevice::Instantiate().Synchronize();  // host buffer may die after return
}

template <typename Real>
void CuMatrixBase<Real>::CopyToMat(MatrixBase<Real> *dst) const {
  if (dst->NumRows() != num_rows_ || dst->NumCols() != num_cols_)
    dst->Resize(num_rows_, num_cols_);
  if (num_rows_ == 0 || num_cols_ == 0) return;
  CU_SAFE_CALL(hipMemcpy2DAsync(dst->Data(), sizeof(Real) * dst->Stride(),
                                data_, sizeof(Real) * stride_,
                                sizeof(Real) * num_cols_, num_rows_,
                                hipMemcpyDeviceToHost,
                                CuDevice::Instantiate().Stream()));
  CuDevice::Instantiate().Synchronize();
}

template <typename Real>
void CuMatrixBase<Real>::AddMat(Real alpha, const CuMatrixBase<Real> &A,
                                MatrixTransposeType trans) {
  if (trans == kNoTrans)
    KALDI_ASSERT(A.NumRows() == num_rows_ && A.NumCols() == num_cols_);
  else
    KALDI_ASSERT(A.NumCols() == num_rows_ && A.NumRows() == num_cols_);
  CNSL_SAFE_CALL(kl_add_mat(alpha, A.Data(), A.Dim(), trans == kTrans, 1.0f,
                            data_, Dim(), S()));
}

static thread_local const CuGemmStatsHint *g_stats_hints = nullptr;

CuGemmStatsHint::CuGemmStatsHint(const float *data, MatrixIndexT rows, MatrixIndexT cols,
                                 MatrixIndexT stride, const uint32_t *rmax,
                                 const uint32_t *cmax)
    : rowmax(rmax), colmax(cmax), data_(data), rows_(rows), cols_(cols), stride_(stride),
      prev_(g_stats_hints) {
  g_stats_hints = this;
}
CuGemmStatsHint::~CuGemmStatsHint() { g_stats_hints = prev_; }
const CuGemmStatsHint *CuGemmStatsHint::Find(const float *data, MatrixIndexT rows,
                                             MatrixIndexT cols, MatrixIndexT stride) {
  for (const CuGemmStatsHint *h = g_stats_hints; h; h = h->prev_)
    if (h->data_ == data && h->rows_ == rows && h->cols_ == cols && h->stride_ == stride)
      return h;
  return nullptr;
}

// a hint's column block for a GEMM, its pending work run first
static const uint32_t *hint_cols(const CuGemmStatsHint *h, kcnn_stream_t st) {
  if (h->pending) CNSL_SAFE_CALL(kcnn_pool_cols_complete(h->pending, st));
  return h->colmax;
}

CuGemmBackpropStats::CuGemmBackpropStats(const CuMatrixBase<float> &dy,
                                         const CuMatrixBase<float> &W, bool cols,
                                         const CuMatrixBase<float> *in) {
  CuDevice &dev = CuDevice::Instantiate();
  const int N = dy.NumRows(), O = dy.NumCols(), I = W.NumCols();
  if (dev.GemmMode() != 2 || N == 0 || O == 0 || I == 0 || W.NumRows() != O) return;
  // an enclosing launch set already covers them (kcnn_nnet_backprop_split:
  // the gradient and the data gradient of one layer around the caller's
  // all-reduce, one statistics pass for both)
  {
    const CuGemmStatsHint *hd = CuGemmStatsHint::Find(dy.Data(), N, O, dy.Stride());
    const CuGemmStatsHint *hw = CuGemmStatsHint::Find(W.Data(), O, I, W.Stride());
    if (hd && hd->rowmax && (!cols || hd->colmax) && hw && hw->colmax && !hw->pending) return;
  }
  // blocks [max, min, cnt]: dy rows (N), dy columns (O), W columns (I), then
  // the column partials
  const size_t pd = cols ? kl_absmax_cols_words(N, O) : 0, pw = kl_absmax_cols_words(O, I);
  const size_t words = 3 * ((size_t)N + O + I) + pd + pw;
  ws_ = dev.Malloc(words * 4);
  uint32_t *rows_d = static_cast<uint32_t *>(ws_), *cols_d = rows_d + 3 * (size_t)N,
           *cols_w = cols_d + 3 * (size_t)O, *part_d = cols_w + 3 * (size_t)I,
           *part_w = part_d + pd;
  // the layer input's pending column statistics (the fused pool's) join these
  // launches: the weight-gradient GEMM below reads them
  PoolColDeferred *pc = nullptr;
  if (cols && in) {
    const CuGemmStatsHint *h =
        CuGemmStatsHint::Find(in->Data(), in->NumRows(), in->NumCols(), in->Stride());
    if (h && h->pending && h->pending->pending) pc = h->pending;
  }
  CNSL_SAFE_CALL(kl_gemm_stats3(dy.Data(), N, O, dy.Stride(), 0, rows_d, nullptr,
                                cols ? dy.Data() : nullptr, N, O, dy.Stride(), 1, cols_d, part_d,
                                W.Data(), O, I, W.Stride(), 1, cols_w, part_w, pc,
                                reinterpret_cast<kcnn_stream_t>(dev.Stream())));
  if (pc) pc->pending = 0;
  hint_d_ = new CuGemmStatsHint(dy.Data(), N, O, dy.Stride(), rows_d, cols ? cols_d : nullptr);
  hint_w_ = new CuGemmStatsHint(W.Data(), O, I, W.Stride(), nullptr, cols_w);
}
CuGemmBackpropStats::~CuGemmBackpropStats() {
  delete hint_w_;
  delete hint_d_;
  if (ws_) CuDevice::Instantiate().Free(ws_);
}

// The f16x3 product (mode 2) of aligned operands Ap, Bp (A, B themselves, or
// their padded copies; A and B name the operands for the statistics hints),
// plus bias[j] on every row when bias != NULL.  False when the kernel
// declines (past its 32-bit addressing): C is untouched then, and the bf16x6
// kernel (same error bound) takes the product.
template <typename Real>
bool CuMatrixBase<Real>::GemmF16x3(Real alpha, const CuMatrixBase<Real> &A,
                                   const CuMatrixBase<Real> &Ap, MatrixTransposeType transA,
                                   const CuMatrixBase<Real> &B, const CuMatrixBase<Real> &Bp,
                                   MatrixTransposeType transB, Real beta, const Real *bias) {
  const MatrixIndexT m = num_rows_, n = num_cols_;
  const MatrixIndexT k = transA == kNoTrans ? A.NumCols() : A.NumRows();
  CuDevice &dev0 = CuDevice::Instantiate();
  // op(A)'s row / op(B)'s column statistics from their producer, if any
  // (CuGemmStatsHint: e.g. the fused conv + pool forward's pooled output)
  const CuGemmStatsHint *ha = CuGemmStatsHint::Find(A.Data(), A.NumRows(), A.NumCols(),
                                                    A.Stride());
  const CuGemmStatsHint *hb = CuGemmStatsHint::Find(B.Data(), B.NumRows(), B.NumCols(),
                                                    B.Stride());
  const uint32_t *ag = ha ? (transA == kNoTrans ? ha->rowmax : hint_cols(ha, S())) : nullptr;
  const uint32_t *bg = hb ? (transB == kNoTrans ? hint_cols(hb, S()) : hb->rowmax) : nullptr;
  const size_t wsf = kl_gemm_f16x3_full_workspace_bytes(m, n, k);
  void *wf = dev0.Malloc(wsf);
  const int rc = kl_gemm_f16x3_bias(transA == kTrans, transB == kTrans, m, n, k, alpha,
                                    Ap.Data(), Ap.Stride(), Bp.Data(), Bp.Stride(), beta, data_,
                                    stride_, ag, bg, bias, wf, wsf, S());
  dev0.Free(wf);
  if (rc == (int)hipErrorNotSupported) return false;
  CNSL_SAFE_CALL(rc);
  return true;
}

template <typename Real>
bool CuMatrixBase<Real>::AddMatMatMomentum(const CuMatrixBase<Real> &A,
                                           MatrixTransposeType transA,
                                           const CuMatrixBase<Real> &B,
                                           MatrixTransposeType transB, CuMatrixBase<Real> *prev,
                                           Real momentum, Real a_wd, Real a_g) {
  const MatrixIndexT m = num_rows_, n = num_cols_;
  const MatrixIndexT k = transA == kNoTrans ? A.NumCols() : A.NumRows();
  CuDevice &dev0 = CuDevice::Instantiate();
  auto aligned = [](const CuMatrixBase<Real> &X) {
    return X.Stride() % 4 == 0 && reinterpret_cast<uintptr_t>(X.Data()) % 16 == 0;
  };
  if (dev0.GemmMode() != 2 || m == 0 || n == 0 || k == 0 || !aligned(A) || !aligned(B) ||
      !aligned(*this) || !aligned(*prev))
    return false;
  KALDI_ASSERT((transA == kNoTrans ? A.NumRows() : A.NumCols()) == m &&
               (transB == kNoTrans ? B.NumCols() : B.NumRows()) == n &&
               (transB == kNoTrans ? B.NumRows() : B.NumCols()) == k &&
               prev->NumRows() == m && prev->NumCols() == n);
  CuProfileScope prof("AddMatMat");
  const CuGemmStatsHint *ha = CuGemmStatsHint::Find(A.Data(), A.NumRows(), A.NumCols(),
                                                    A.Stride());
  const CuGemmStatsHint *hb = CuGemmStatsHint::Find(B.Data(), B.NumRows(), B.NumCols(),
                                                    B.Stride());
  const uint32_t *ag = ha ? (transA == kNoTrans ? ha->rowmax : hint_cols(ha, S())) : nullptr;
  const uint32_t *bg = hb ? (transB == kNoTrans ? hint_cols(hb, S()) : hb->rowmax) : nullptr;
  const size_t wsf = kl_gemm_f16x3_full_workspace_bytes(m, n, k);
  void *wf = dev0.Malloc(wsf);
  const int rc = kl_gemm_f16x3_momentum(transA == kTrans, transB == kTrans, m, n, k, A.Data(),
                                        A.Stride(), B.Data(), B.Stride(), ag, bg, data_, stride_,
                                        prev->Data(), prev->Stride(), momentum, a_wd, a_g, wf,
                                        wsf, S());
  dev0.Free(wf);
  if (rc == (int)hipErrorNotSupported) return false;
  CNSL_SAFE_CALL(rc);
  return true;
}

template <typename Real>
void CuMatrixBase<Real>::AddMatMatBias(Real alpha, const CuMatrixBase<Real> &A,
                                       MatrixTransposeType transA, const CuMatrixBase<Real> &B,
                                       MatrixTransposeType transB,
                                       const CuVectorBase<Real> &bias) {
  const MatrixIndexT k = transA == kNoTrans ? A.NumCols() : A.NumRows();
  KALDI_ASSERT(bias.Dim() == num_cols_);
  CuDevice &dev0 = CuDevice::Instantiate();
  auto aligned = [](const CuMatrixBase<Real> &X) {
    return X.Stride() % 4 == 0 && reinterpret_cast<uintptr_t>(X.Data()) % 16 == 0;
  };
  if (dev0.GemmMode() == 2 && num_rows_ > 0 && num_cols_ > 0 && k > 0 && aligned(A) &&
      aligned(B)) {
    KALDI_ASSERT((transA == kNoTrans ? A.NumRows() : A.NumCols()) == num_rows_ &&
                 (transB == kNoTrans ? B.NumCols() : B.NumRows()) == num_cols_ &&
                 (transB == kNoTrans ? B.NumRows() : B.NumCols()) == k);
    CuProfileScope prof("AddMatMat");
    if (GemmF16x3(alpha, A, A, transA, B, B, transB, 0.0f, bias.Data())) return;
  }
  CopyRowsFromVec(bias);
  AddMatMat(alpha, A, transA, B, transB, 1.0f);
}

template <typename Real>
void CuMatrixBase<Real>::AddMatMat(Real alpha, const CuMatrixBase<Real> &A,
                                   MatrixTransposeType transA,
                                   const CuMatrixBase<Real> &B,
                                   MatrixTransposeType transB, Real beta) {
  const MatrixIndexT m = transA == kNoTrans ? A.NumRows() : A.NumCols();
  const MatrixIndexT k = transA == kNoTrans ? A.NumCols() : A.NumRows();
  const MatrixIndexT kb = transB == kNoTrans ? B.NumRows() : B.NumCols();
  const MatrixIndexT n = transB == kNoTrans ? B.NumCols() : B.NumRows();
  KALDI_ASSERT(k == kb && m == num_rows_ && n == num_cols_);
  if (m == 0 || n == 0) return;
  if (k == 0) { if (beta != 1.0f) Scale(beta); return; }
  CuProfileScope prof("AddMatMat");
  CuDevice &dev0 = CuDevice::Instantiate();
  const int mode = dev0.GemmMode();
  if (mode >= 1) {
    // fp32 product on the f16 (mode 2, cu-gemm-f16x3.hip) or bf16 (mode 1,
    // cu-gemm-x6.hip) MFMAs from a split of each operand.  Their 16-B loads
    // need the K-contiguous operands (A untransposed, B transposed)
    // row-aligned; one that is not (a caller's matrix with an odd pitch,
    // e.g. an output derivative of 3454 columns) is copied once into a
    // padded-pitch CuMatrix, which costs far less than the GEMM.  So is a
    // row-contiguous one under f16x3, whose 16-B transposed loads (LT) take
    // 450 -> ~260 us on nnet.config's last FC weight gradient (the one-column
    // loads' kernel otherwise).
    auto aligned = [](const CuMatrixBase<Real> &X) {
      return X.Stride() % 4 == 0 && reinterpret_cast<uintptr_t>(X.Data()) % 16 == 0;
    };
    CuMatrix<Real> Acopy, Bcopy;
    const CuMatrixBase<Real> *Ap = &A, *Bp = &B;
    if ((transA == kNoTrans || mode == 2) && !aligned(A)) { Acopy = A; Ap = &Acopy; }
    if ((transB == kTrans || mode == 2) && !aligned(B)) { Bcopy = B; Bp = &Bcopy; }
    if (mode == 2 && GemmF16x3(alpha, A, *Ap, transA, B, *Bp, transB, beta, nullptr)) return;
    const size_t wsb = kl_gemm_x6_workspace_bytes(m, n, k);
    void *ws = wsb ? dev0.Malloc(wsb) : nullptr;
    const int rc = kl_gemm_x6(transA == kTrans, transB == kTrans, m, n, k, alpha,
                              Ap->Data(), Ap->Stride(), Bp->Data(), Bp->Stride(), beta,
                              data_, stride_, ws, wsb, S());
    if (ws) dev0.Free(ws);
    // The operands are aligned here, so the kernel declines (hipErrorInvalidValue)
    // only past its grid limit (2^31 workgroups: M x N beyond 2^46 values).
    // No silent switch of engine: that is the "gemm" family's to choose.
    if (rc == (int)hipErrorInvalidValue)
      KALDI_ERR << "AddMatMat: " << m << " x " << n << " x " << k
                << " is outside the bf16x6 GEMM's limits; select rocBLAS sgemm with "
                   "kcnn_set_kernel_family(\"gemm\", 0)";
    CNSL_SAFE_CALL(rc);
    return;
  }
  // Row-major C = op(A) op(B)  <=>  column-major C^T = op(B)^T op(A)^T.
  const rocblas_operation opB =
      transB == kTrans ? rocblas_operation_transpose : rocblas_operation_none;
  const rocblas_operation opA =
      transA == kTrans ? rocblas_operation_transpose : rocblas_operation_none;
  // A thin output with a long K (the FC forward: 4096 x 1024, K = 11616)
  // gives too few output tiles to fill 256 CUs: split K over a strided
  // batch, then sum the partials in a fixed order.
  int nsplit = 1;
  {
    const int64_t tiles = (int64_t)((m + 255) / 256) * ((n + 255) / 256);
    if (tiles < 128 && k >= 4096) {
      for (int s : {4, 2})
        if (k % s == 0 && k / s >= 1024 && tiles * s <= 512) { nsplit = s; break; }
    }
    static const int e = KCNN_KNOB("KCNN_GEMM_SPLITK", 0);
    if (e >= 1 && k % e == 0) nsplit = e;
  }
  if (nsplit > 1) {
    CuDevice &dev = CuDevice::Instantiate();
    const int S_ = nsplit;
    const int kc = k / S_;
    const rocblas_stride sA = transA == kNoTrans ? kc : (rocblas_stride)kc * A.Stride();
    const rocblas_stride sB = transB == kNoTrans ? (rocblas_stride)kc * B.Stride() : kc;
    float *part = static_cast<float *>(dev.Malloc(sizeof(float) * (size_t)S_ * m * n));
    const float zero = 0.0f;
    rocblas_status st = rocblas_sgemm_strided_batched(
        dev.GetBlasHandle(), opB, opA, n, m, kc, &alpha, B.Data(), B.Stride(),
        sB, A.Data(), A.Stride(), sA, &zero, part, n, (rocblas_stride)m * n, S_);
    int rc = st == rocblas_status_success
                 ? kl_sum_partials(part, S_, m, n, beta, data_, Dim(), S())
                 : -1;
    dev.Free(part);
    if (st != rocblas_status_success)
      KALDI_ERR << "rocblas_sgemm_strided_batched failed with status " << (int)st;
    CNSL_SAFE_CALL(rc);
    return;
  }
  rocblas_status st = rocblas_sgemm(
      CuDevice::Instantiate().GetBlasHandle(), opB, opA, n, m, k, &alpha,
      B.Data(), B.Stride(), A.Data(), A.Stride(), &beta, data_, stride_);
  if (st != rocblas_status_success)
    KALDI_ERR << "rocblas_sgemm failed with status " << (int)st;
}

template <typename Real>
void CuMatrixBase<Real>::CopyRowsFromVec(const CuVectorBase<Real> &v) {
  KALDI_ASSERT(v.Dim() == num_cols_);
  CNSL_SAFE_CALL(kl_copy_rows_from_vec(v.Data(), data_, Dim(), S()));
}
template <typename Real>
void CuMatrixBase<Real>::CopyRowsFromVec(const VectorBase<Real> &v) {
  CuVector<Real> tmp;
  tmp = v;
  CopyRowsFromVec(tmp);
}

template <typename Real>
Real CuMatrixBase<Real>::Sum() const {
  Matrix<Real> h;
  CopyToMat(&h);
  double s = 0;
  for (MatrixIndexT i = 0; i < h.NumRows(); i++)
    for (MatrixIndexT j = 0; j < h.NumCols(); j++) s += h(i, j);
  return (Real)s;
}

template <typename Real>
CuSubMatrix<Real> CuMatrixBase<Real>::Range(MatrixIndexT ro, MatrixIndexT nr,
                                            MatrixIndexT co,
                                            MatrixIndexT nc) const {
  KALDI_ASSERT(ro >= 0 && co >= 0 && nr >= 0 && nc >= 0 &&
               ro + nr <= num_rows_ && co + nc <= num_cols_);
  return CuSubMatrix<Real>(data_ + (int64)ro * stride_ + co, nr, nc, stride_);
}
template <typename Real>
CuSubMatrix<Real> CuMatrixBase<Real>::RowRange(MatrixIndexT ro,
                                               MatrixIndexT nr) const {
  return Range(ro, nr, 0, num_cols_);
}
template <typename Real>
CuSubMatrix<Real> CuMatrixBase<Real>::ColRange(MatrixIndexT co,
                                               MatrixIndexT nc) const {
  return Range(0, num_rows_, co, nc);
}

template <typename Real>
void CuMatrixBase<Real>::Write(std::ostream &os, bool binary) const {
  Matrix<Real> h;
  CopyToMat(&h);
  h.Write(os, binary);
}

// ---- CuMatrix -------------------------------------------------------------
template <typename Real>
void CuMatrix<Real>::Destroy() {
  if (this->data_ && !borrowed_) CuDevice::Instantiate().Free(this->data_);
  this->data_ = nullptr;
  this->num_rows_ = this->num_cols_ = this->stride_ = 0;
  borrowed_ = false;
}

template <typename Real>
void CuMatrix<Real>::Resize(MatrixIndexT rows, MatrixIndexT cols,
                            MatrixResizeType resize_type) {
  KALDI_ASSERT(rows >= 0 && cols >= 0);
  if (rows == this->num_rows_ && cols == this->num_cols_) {
    if (resize_type == kSetZero) this->SetZero();
    return;
  }
  if (borrowed_)
    KALDI_ERR << "cannot resize a matrix bound to external memory from "
              << this->num_rows_ << "x" << this->num_cols_ << " to " << rows
              << "x" << cols;
  if (resize_type == kCopyData) {
    CuMatrix<Real> tmp(rows, cols, kSetZero);
    const MatrixIndexT r = std::min(rows, this->num_rows_);
    const MatrixIndexT c = std::min(cols, this->num_cols_);
    if (r > 0 && c > 0) tmp.Range(0, r, 0, c).CopyFromMat(this->Range(0, r, 0, c));
    Swap(&tmp);
    return;
  }
  Destroy();
  if (rows == 0 || cols == 0) return;
  const MatrixIndexT stride = PaddedStride(cols);
  this->data_ = static_cast<Real *>(
      CuDevice::Instantiate().Malloc(sizeof(Real) * (size_t)rows * stride));
  this->num_rows_ = rows;
  this->num_cols_ = cols;
  this->stride_ = stride;
  if (resize_type == kSetZero) this->SetZero();
}

template <typename Real>
void CuMatrix<Real>::Swap(CuMatrix<Real> *o) {
  std::swap(this->data_, o->data_);
  std::swap(this->num_rows_, o->num_rows_);
  std::swap(this->num_cols_, o->num_cols_);
  std::swap(this->stride_, o->stride_);
  std::swap(borrowed_, o->borrowed_);
}

template <typename Real>
void CuMatrix<Real>::Borrow(Real *data, MatrixIndexT rows, MatrixIndexT cols,
                            MatrixIndexT stride) {
  Destroy();
  this->data_ = data;
  this->num_rows_ = rows;
  this->num_cols_ = cols;
  this->stride_ = stride;
  borrowed_ = true;
}

template <typename Real>
CuMatrix<Real> &CuMatrix<Real>::operator=(const CuMatrixBase<Real> &o) {
  if (static_cast<const CuMatrixBase<Real> *>(this) == &o) return *this;
  Resize(o.NumRows(), o.NumCols(), kUndefined);
  this->CopyFromMat(o);
  return *this;
}
template <typename Real>
CuMatrix<Real> &CuMatrix<Real>::operator=(const CuMatrix<Real> &o) {
  return *this = static_cast<const CuMatrixBase<Real> &>(o);
}
template <typename Real>
CuMatrix<Real> &CuMatrix<Real>::operator=(const MatrixBase<Real> &o) {
  Resize(o.NumRows(), o.NumCols(), kUndefined);
  this->CopyFromMat(o);
  return *this;
}

template <typename Real>
void CuMatrix<Real>::Read(std::istream &is, bool binary) {
  Matrix<Real> h;
  h.Read(is, binary);
  *this = h;
}

// ---- vectors ----------------------------------------------------------------
template <typename Real>
void CuVectorBase<Real>::SetZero() {
  if (dim_ == 0) return;
  CU_SAFE_CALL(hipMemsetAsync(data_, 0, sizeof(Real) * dim_,
                              CuDevice::Instantiate().Stream()));
}
template <typename Real>
void CuVectorBase<Real>::Set(Real v) { CNSL_SAFE_CALL(kl_set(data_, VecDim(dim_), v, S())); }
template <typename Real>
void CuVectorBase<Real>::Add(Real v) { CNSL_SAFE_CALL(kl_add(data_, VecDim(dim_), v, S())); }
template <typename Real>
void CuVectorBase<Real>::Scale(Real v) { CNSL_SAFE_CALL(kl_scale(data_, VecDim(dim_), v, S())); }
template <typename Real>
void CuVectorBase<Real>::SetRandn() {
  Vector<Real> h(dim_);
  RandnFill(h.Data(), dim_);
  CopyFromVec(h);
}
template <typename Real>
void CuVectorBase<Real>::CopyFromVec(const CuVectorBase<Real> &v) {
  KALDI_ASSERT(v.Dim() == dim_);
  if (dim_ == 0) return;
  CU_SAFE_CALL(hipMemcpyAsync(data_, v.Data(), sizeof(Real) * dim_,
                              hipMemcpyDeviceToDevice,
                              CuDevice::Instantiate().Stream()));
}
template <typename Real>
void CuVectorBase<Real>::CopyFromVec(const VectorBase<Real> &v) {
  KALDI_ASSERT(v.Dim() == dim_);
  if (dim_ == 0) return;
  CU_SAFE_CALL(hipMemcpyAsync(data_, v.Data(), sizeof(Real) * dim_,
                              hipMemcpyHostToDevice,
                              CuDevice::Instantiate().Stream()));
  CuDevice::Instantiate().Synchronize();
}
template <typename Real>
void CuVectorBase<Real>::CopyToVec(VectorBase<Real> *v) const {
  if (v->Dim() != dim_) v->Resize(dim_);
  if (dim_ == 0) return;
  CU_SAFE_CALL(hipMemcpyAsync(v->Data(), data_, sizeof(Real) * dim_,
                              hipMemcpyDeviceToHost,
                              CuDevice::Instantiate().Stream()));
  CuDevice::Instantiate().Synchronize();
}
template <typename Real>
void CuVectorBase<Real>::AddVec(Real alpha, const CuVectorBase<Real> &v,
                                Real beta) {
  KALDI_ASSERT(v.Dim() == dim_);
  CNSL_SAFE_CALL(kl_add_mat(alpha, v.Data(), VecDim(dim_), 0, beta, data_,
                            VecDim(dim_), S()));
}
template <typename Real>
void CuVectorBase<Real>::AddRowSumMat(Real alpha, const CuMatrixBase<Real> &M,
                                      Real beta) {
  KALDI_ASSERT(M.NumCols() == dim_);
  CuDevice &dev = CuDevice::Instantiate();
  void *ws = dev.Malloc(kl_col_sum_workspace_bytes(M.Dim()));
  const int rc = kl_col_sum(M.Data(), M.Dim(), alpha, beta, data_, ws, S());
  dev.Free(ws);
  CNSL_SAFE_CALL(rc);
}
template <typename Real>
void CuVectorBase<Real>::CopyColFromMat(const CuMatrixBase<Real> &M,
                                        MatrixIndexT col) {
  KALDI_ASSERT(M.NumRows() == dim_ && col >= 0 && col < M.NumCols());
  if (dim_ == 0) return;
  CU_SAFE_CALL(hipMemcpy2DAsync(data_, sizeof(Real), M.Data() + col,
                                sizeof(Real) * M.Stride(), sizeof(Real), dim_,
                                hipMemcpyDeviceToDevice,
                                CuDevice::Instantiate().Stream()));
}
template <typename Real>
CuSubVector<Real> CuVectorBase<Real>::Range(MatrixIndexT o,
                                            MatrixIndexT l) const {
  KALDI_ASSERT(o >= 0 && l >= 0 && o + l <= dim_);
  return CuSubVector<Real>(data_ + o, l);
}
template <typename Real>
void CuVectorBase<Real>::Write(std::ostream &os, bool binary) const {
  Vector<Real> h;
  CopyToVec(&h);
  h.Write(os, binary);
}

template <typename Real>
void CuVector<Real>::Destroy() {
  if (this->data_ && !borrowed_) CuDevice::Instantiate().Free(this->data_);
  this->data_ = nullptr;
  this->dim_ = 0;
  borrowed_ = false;
}
template <typename Real>
void CuVector<Real>::Resize(MatrixIndexT d, MatrixResizeType t) {
  KALDI_ASSERT(d >= 0);
  if (d == this->dim_) {
    if (t == kSetZero) this->SetZero();
    return;
  }
  if (borrowed_) KALDI_ERR << "cannot resize a vector bound to external memory";
  Destroy();
  if (d == 0) return;
  this->data_ = static_cast<Real *>(CuDevice::Instantiate().Malloc(sizeof(Real) * d));
  this->dim_ = d;
  if (t == kSetZero) this->SetZero();
}
template <typename Real>
void CuVector<Real>::Borrow(Real *data, MatrixIndexT dim) {
  Destroy();
  this->data_ = data;
  this->dim_ = dim;
  borrowed_ = true;
}
template <typename Real>
CuVector<Real> &CuVector<Real>::operator=(const CuVectorBase<Real> &o) {
  if (static_cast<const CuVectorBase<Real> *>(this) == &o) return *this;
  Resize(o.Dim(), kUndefined);
  this->CopyFromVec(o);
  return *this;
}
template <typename Real>
CuVector<Real> &CuVector<Real>::operator=(const CuVector<Real> &o) {
  return *this = static_cast<const CuVectorBase<Real> &>(o);
}
template <typename Real>
CuVector<Real> &CuVector<Real>::operator=(const VectorBase<Real> &o) {
  Resize(o.Dim(), kUndefined);
  this->CopyFromVec(o);
  return *this;
}
template <typename Real>
void CuVector<Real>::Read(std::istream &is, bool binary) {
  Vector<Real> h;
  h.Read(is, binary);
  *this = h;
}

template <typename Real>
Real TraceMatMat(const CuMatrixBase<Real> &A, const CuMatrixBase<Real> &B,
                 MatrixTransposeType trans) {
  if (trans == kTrans)
    KALDI_ASSERT(A.NumRows() == B.NumRows() && A.NumCols() == B.NumCols());
  else
    KALDI_ASSERT(A.NumRows() == B.NumCols() && A.NumCols() == B.NumRows());
  CuDevice &dev = CuDevice::Instantiate();
  double *d = static_cast<double *>(dev.Malloc(sizeof(double)));
  int rc = kl_dot(A.Data(), A.Dim(), B.Data(), B.Dim(), trans == kNoTrans, d, S());
  double h = 0;
  if (rc == 0)
    rc = (int)hipMemcpyAsync(&h, d, sizeof(double), hipMemcpyDeviceToHost,
                             dev.Stream());
  dev.Synchronize();
  dev.Free(d);
  CNSL_SAFE_CALL(rc);
  return (Real)h;
}

template <typename Real>
Real VecVec(const CuVectorBase<Real> &a, const CuVectorBase<Real> &b) {
  KALDI_ASSERT(a.Dim() == b.Dim());
  CuSubMatrix<Real> A(const_cast<Real *>(a.Data()), 1, a.Dim(), a.Dim());
  CuSubMatrix<Real> B(const_cast<Real *>(b.Data()), 1, b.Dim(), b.Dim());
  return TraceMatMat(A, B, kTrans);
}

template class VectorBase<float>;
template class VectorBase<double>;
template class MatrixBase<float>;
template class CuMatrixBase<float>;
template class CuMatrix<float>;
template class CuVectorBase<float>;
template class CuVector<float>;
template float TraceMatMat(const CuMatrixBase<float> &, const CuMatrixBase<float> &,
                           MatrixTransposeType);
template float VecVec(const CuVectorBase<float> &, const CuVectorBase<float> &);

}  // namespace kaldi
