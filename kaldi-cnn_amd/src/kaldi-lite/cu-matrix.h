// kaldi-lite/cu-matrix.h -- HIP-native CuMatrixBase / CuMatrix / CuSubMatrix,
// CuVectorBase / CuVector / CuSubVector and the host Matrix / Vector they
// exchange data with: the subset of upstream cudamatrix/ + matrix/ listed in
// SURVEY Appendix C, with the same names and signatures so the nnet0
// components compile unchanged against it.
//
// Layout is Kaldi's: row-major with a pitch, element (r, c) at
// data_[r * stride_ + c] (reference cudamatrix/cu-matrix.h:403-417,
// :518-528).  Strides are padded to a multiple of 16 floats (64 B) so rows
// start on cache-line boundaries.  Only Real = float is instantiated
// (SURVEY B15).
//
// The ten cnsl extensions the reference grafted onto CuMatrixBase
// (cu-matrix.h:446-482) are declared here with their signatures verbatim;
// their bodies live in cnslmat/conv2D.cc.
#ifndef KCNN_KALDI_LITE_CU_MATRIX_H_
#define KCNN_KALDI_LITE_CU_MATRIX_H_

#include <istream>
#include <ostream>
#include <vector>

#include "cnsl-hip-kernels.h"  // ::MatrixDim
#include "kaldi-common.h"

namespace kaldi {

template <typename Real> class CuMatrix;
template <typename Real> class CuSubMatrix;
template <typename Real> class CuVectorBase;
template <typename Real> class CuSubVector;

// ---- host containers ------------------------------------------------------
template <typename Real>
class VectorBase {
 public:
  MatrixIndexT Dim() const { return (MatrixIndexT)data_.size(); }
  Real *Data() { return data_.data(); }
  const Real *Data() const { return data_.data(); }
  Real &operator()(MatrixIndexT i) { return data_[i]; }
  Real operator()(MatrixIndexT i) const { return data_[i]; }
  void Resize(MatrixIndexT d) { data_.assign(d, Real(0)); }
  void Read(std::istream &is, bool binary);
  void Write(std::ostream &os, bool binary) const;

 protected:
  std::vector<Real> data_;
};
template <typename Real>
class Vector : public VectorBase<Real> {
 public:
  Vector() {}
  explicit Vector(MatrixIndexT d) { this->Resize(d); }
};

template <typename Real>
class MatrixBase {
 public:
  MatrixIndexT NumRows() const { return rows_; }
  MatrixIndexT NumCols() const { return cols_; }
  MatrixIndexT Stride() const { return cols_; }
  Real *Data() { return data_.data(); }
  const Real *Data() const { return data_.data(); }
  Real &operator()(MatrixIndexT r, MatrixIndexT c) { return data_[(size_t)r * cols_ + c]; }
  Real operator()(MatrixIndexT r, MatrixIndexT c) const { return data_[(size_t)r * cols_ + c]; }
  void Resize(MatrixIndexT r, MatrixIndexT c) {
    rows_ = r; cols_ = c; data_.assign((size_t)r * c, Real(0));
  }
  void Read(std::istream &is, bool binary);
  void Write(std::ostream &os, bool binary) const;

 protected:
  MatrixIndexT rows_ = 0, cols_ = 0;
  std::vector<Real> data_;
};
template <typename Real>
class Matrix : public MatrixBase<Real> {
 public:
  Matrix() {}
  Matrix(MatrixIndexT r, MatrixIndexT c) { this->Resize(r, c); }
};

// ---- device matrices ------------------------------------------------------
template <typename Real>
class CuMatrixBase {
 public:
  MatrixIndexT NumRows() const { return num_rows_; }
  MatrixIndexT NumCols() const { return num_cols_; }
  MatrixIndexT Stride() const { return stride_; }
  ::MatrixDim Dim() const {
    ::MatrixDim d;
    d.rows = num_rows_; d.cols = num_cols_; d.stride = stride_;
    return d;
  }
  // (Kaldi keeps Data() protected with friends; public here for the shim.)
  Real *Data() { return data_; }
  const Real *Data() const { return data_; }
  Real *RowData(MatrixIndexT r) { return data_ + (int64)r * stride_; }
  const Real *RowData(MatrixIndexT r) const { return data_ + (int64)r * stride_; }

  void SetZero();
  void Set(Real value);
  void Add(Real value);
  void Scale(Real value);
  void SetRandn();  // N(0,1) from the host generator (deterministic seed)
  void CopyFromMat(const CuMatrixBase<Real> &src,
                   MatrixTransposeType trans = kNoTrans);
  void CopyFromMat(const MatrixBase<Real> &src);  // host -> device
  void CopyToMat(MatrixBase<Real> *dst) const;    // device -> host
  /// *this += alpha * op(A)
  void AddMat(Real alpha, const CuMatrixBase<Real> &A,
              MatrixTransposeType trans = kNoTrans);
  /// *this = alpha * op(A) op(B) + beta * *this   (rocBLAS sgemm)
  void AddMatMat(Real alpha, const CuMatrixBase<Real> &A,
                 MatrixTransposeType transA, const CuMatrixBase<Real> &B,
                 MatrixTransposeType transB, Real beta);
  /// *this = alpha * op(A) op(B) + bias on every row (an FC forward's
  /// CopyRowsFromVec(bias); AddMatMat(alpha, A, tA, B, tB, 1.0) in one pass
  /// under the f16x3 engine; those two calls otherwise)
  void AddMatMatBias(Real alpha, const CuMatrixBase<Real> &A, MatrixTransposeType transA,
                     const CuMatrixBase<Real> &B, MatrixTransposeType transB,
                     const CuVectorBase<Real> &bias);
  /// this = W: the momentum update with the gradient op(A) op(B) applied in
  /// the f16x3 GEMM's store (kl_gemm_f16x3_momentum; prev = momentum prev +
  /// a_wd W + a_g g, W += prev), without a gradient buffer.  False when the
  /// engine is not f16x3 or an operand is not 16-B aligned: nothing is
  /// changed then and the caller takes the gradient buffer path.
  bool AddMatMatMomentum(const CuMatrixBase<Real> &A, MatrixTransposeType transA,
                         const CuMatrixBase<Real> &B, MatrixTransposeType transB,
                         CuMatrixBase<Real> *prev, Real momentum, Real a_wd, Real a_g);
  /// every row = v
  void CopyRowsFromVec(const CuVectorBase<Real> &v);
  void CopyRowsFromVec(const VectorBase<Real> &v);  // host vector
  Real Sum() const;

  CuSubMatrix<Real> Range(MatrixIndexT row_offset, MatrixIndexT num_rows,
                          MatrixIndexT col_offset, MatrixIndexT num_cols) const;
  CuSubMatrix<Real> RowRange(MatrixIndexT row_offset,
                             MatrixIndexT num_rows) const;
  CuSubMatrix<Real> ColRange(MatrixIndexT col_offset,
                             MatrixIndexT num_cols) const;

  void Write(std::ostream &os, bool binary) const;

  // ---- added by hwaran (reference cudamatrix/cu-matrix.h:446-482) --------
  // Convolution 'this' with kernel => out
  // this matrix : row = num_chunks, col=in_height * in_width * in_channel
  void Conv2D(const CuMatrixBase<Real> &kernel, int32 in_height,
              int32 in_width, int32 in_channel, int32 kernel_height,
              int32 kernel_width, int32 group, CuMatrixBase<Real> *out,
              bool concat) const;
  // if vec = [1 2 3] and rep = 2 => vec2 = [ 1 1 2 2 3 3];
  // this = this + repmat(vec2, NumRows(), 1);
  void AddMatRepVec(const CuVectorBase<Real> &vec, int32 rep) const;
  // this [(kernel_height*kernel_width*in_channel) x group]
  // flip [(kernel_height*kernel_width*group) x in_channel]
  void FlipMat(int32 kernel_height, int32 kernel_width, int32 in_channel,
               int32 group, CuMatrix<Real> *flip) const;
  // zero padding along the edge of every orig_height x orig_width map
  void PaddingZero(int32 orig_height, int32 orig_width, int32 orig_channel,
                   int32 kernel_height, int32 kernel_width,
                   CuMatrix<Real> *padmat) const;
  void TpBlock(int32 in_channel, int32 block_size, CuMatrix<Real> *out) const;
  void TpInsideBlock(int32 group, int32 block_size, CuMatrix<Real> *out) const;
  void ModPermuteRow(int32 in_channel, int32 block_size,
                     CuMatrix<Real> *out) const;
  void Maxpool_prop(int32 in_height, int32 in_width, int32 pool_height_dim,
                    int32 pool_width_dim, int32 pool_channel_dim, bool overlap,
                    bool overlap2D, CuMatrixBase<Real> *out) const;
  void Maxpool_backprop(const CuMatrixBase<Real> &out_value,
                        const CuMatrixBase<Real> &out_deriv,
                        CuMatrix<Real> *in_deriv, int32 in_height,
                        int32 in_width, int32 pool_height_dim,
                        int32 pool_width_dim, int32 pool_channel_dim,
                        bool overlap, bool overlap2D) const;
  // (used by the reference's unregistered ConvolutionComponentContainer)
  void ModPermuteChannel(int32 comp_idx, int32 num_component, int32 in_height,
                         int32 in_width, CuMatrixBase<Real> *container,
                         bool fromCompToContainer);

 protected:
  bool GemmF16x3(Real alpha, const CuMatrixBase<Real> &A, const CuMatrixBase<Real> &Ap,
                 MatrixTransposeType transA, const CuMatrixBase<Real> &B,
                 const CuMatrixBase<Real> &Bp, MatrixTransposeType transB, Real beta,
                 const Real *bias);
  CuMatrixBase() : data_(nullptr), num_cols_(0), num_rows_(0), stride_(0) {}
  CuMatrixBase(Real *data, MatrixIndexT num_rows, MatrixIndexT num_cols,
               MatrixIndexT stride)
      : data_(data), num_cols_(num_cols), num_rows_(num_rows), stride_(stride) {}

  Real *data_;
  MatrixIndexT num_cols_;
  MatrixIndexT num_rows_;
  MatrixIndexT stride_;

 private:
  KALDI_DISALLOW_COPY_AND_ASSIGN(CuMatrixBase);
};

template <typename Real>
class CuMatrix : public CuMatrixBase<Real> {
 public:
  CuMatrix() {}
  CuMatrix(MatrixIndexT rows, MatrixIndexT cols,
           MatrixResizeType resize_type = kSetZero) {
    Resize(rows, cols, resize_type);
  }
  CuMatrix(const CuMatrix<Real> &other) { *this = other; }
  explicit CuMatrix(const CuMatrixBase<Real> &other) {
    Resize(other.NumRows(), other.NumCols(), kUndefined);
    this->CopyFromMat(other);
  }
  ~CuMatrix() { Destroy(); }

  CuMatrix<Real> &operator=(const CuMatrixBase<Real> &other);
  CuMatrix<Real> &operator=(const CuMatrix<Real> &other);
  CuMatrix<Real> &operator=(const MatrixBase<Real> &other);

  /// Same semantics as Kaldi: if the size already matches, only kSetZero
  /// acts (zeroes); otherwise reallocate.  A matrix bound to external memory
  /// (Borrow) cannot change size.
  void Resize(MatrixIndexT rows, MatrixIndexT cols,
              MatrixResizeType resize_type = kSetZero);
  void Swap(CuMatrix<Real> *other);
  void Read(std::istream &is, bool binary);

  /// Binds to caller-owned device memory (no ownership).  Used by the
  /// extern "C" layer to hand host-framework buffers to methods that take a
  /// CuMatrix<Real>* output.
  void Borrow(Real *data, MatrixIndexT rows, MatrixIndexT cols,
              MatrixIndexT stride);

 private:
  void Destroy();
  bool borrowed_ = false;
};

template <typename Real>
class CuSubMatrix : public CuMatrixBase<Real> {
 public:
  CuSubMatrix(Real *data, MatrixIndexT num_rows, MatrixIndexT num_cols,
              MatrixIndexT stride)
      : CuMatrixBase<Real>(data, num_rows, num_cols, stride) {}
  CuSubMatrix(const CuSubMatrix<Real> &o)
      : CuMatrixBase<Real>(o.data_, o.num_rows_, o.num_cols_, o.stride_) {}
};

// ---- device vectors -------------------------------------------------------
template <typename Real>
class CuVectorBase {
 public:
  MatrixIndexT Dim() const { return dim_; }
  Real *Data() { return data_; }
  const Real *Data() const { return data_; }
  void SetZero();
  void Set(Real v);
  void Add(Real v);
  void Scale(Real v);
  void SetRandn();
  void CopyFromVec(const CuVectorBase<Real> &v);
  void CopyFromVec(const VectorBase<Real> &v);
  void CopyToVec(VectorBase<Real> *v) const;
  /// *this += alpha * v
  void AddVec(Real alpha, const CuVectorBase<Real> &v, Real beta = 1.0);
  /// *this = beta * *this + alpha * (sum over the rows of M)
  void AddRowSumMat(Real alpha, const CuMatrixBase<Real> &M, Real beta = 1.0);
  /// this = column `col` of M
  void CopyColFromMat(const CuMatrixBase<Real> &M, MatrixIndexT col);
  CuSubVector<Real> Range(MatrixIndexT o, MatrixIndexT l) const;
  void Write(std::ostream &os, bool binary) const;

 protected:
  CuVectorBase() : data_(nullptr), dim_(0) {}
  CuVectorBase(Real *d, MatrixIndexT n) : data_(d), dim_(n) {}
  Real *data_;
  MatrixIndexT dim_;

 private:
  KALDI_DISALLOW_COPY_AND_ASSIGN(CuVectorBase);
};

template <typename Real>
class CuVector : public CuVectorBase<Real> {
 public:
  CuVector() {}
  explicit CuVector(MatrixIndexT d, MatrixResizeType t = kSetZero) { Resize(d, t); }
  CuVector(const CuVector<Real> &o) { *this = o; }
  ~CuVector() { Destroy(); }
  CuVector<Real> &operator=(const CuVectorBase<Real> &o);
  CuVector<Real> &operator=(const CuVector<Real> &o);
  CuVector<Real> &operator=(const VectorBase<Real> &o);
  void Resize(MatrixIndexT d, MatrixResizeType t = kSetZero);
  void Read(std::istream &is, bool binary);
  void Borrow(Real *data, MatrixIndexT dim);

 private:
  void Destroy();
  bool borrowed_ = false;
};

template <typename Real>
class CuSubVector : public CuVectorBase<Real> {
 public:
  CuSubVector(Real *d, MatrixIndexT n) : CuVectorBase<Real>(d, n) {}
  CuSubVector(const CuSubVector<Real> &o) : CuVectorBase<Real>(o.data_, o.dim_) {}
};

/// tr(A B^T) for kTrans (= sum_ij A_ij B_ij), tr(A B) for kNoTrans.
template <typename Real>
Real TraceMatMat(const CuMatrixBase<Real> &A, const CuMatrixBase<Real> &B,
                 MatrixTransposeType trans = kNoTrans);
template <typename Real>
Real VecVec(const CuVectorBase<Real> &a, const CuVectorBase<Real> &b);

/// Statistics a producer computed for a matrix's contents -- max |x| bit
/// patterns per row and per column (device arrays, either nullable) -- offered
/// to AddMatMat while the object is in scope on this thread.  AddMatMat's
/// f16x3 engine scales each operand row / column by them
/// (kaldi-lite/cu-gemm-f16x3.hip) and would otherwise read the operand once
/// more to compute them.  The owner keeps the matrix unmodified in scope.
}  // namespace kaldi
struct PoolColDeferred;  // cnslmat/pool-stats.h
namespace kaldi {
class CuGemmStatsHint {
 public:
  CuGemmStatsHint(const float *data, MatrixIndexT rows, MatrixIndexT cols, MatrixIndexT stride,
                  const uint32_t *rowmax, const uint32_t *colmax);
  ~CuGemmStatsHint();
  CuGemmStatsHint(const CuGemmStatsHint &) = delete;
  CuGemmStatsHint &operator=(const CuGemmStatsHint &) = delete;
  /// the innermost hint for exactly this matrix, or NULL
  static const CuGemmStatsHint *Find(const float *data, MatrixIndexT rows, MatrixIndexT cols,
                                     MatrixIndexT stride);
  const uint32_t *rowmax, *colmax;
  /// colmax's work left pending by its producer (nullable): run by the
  /// reader (CuGemmBackpropStats merges it into its launches; AddMatMat
  /// runs it first) before colmax is read
  PoolColDeferred *pending = nullptr;

 private:
  const float *data_;
  MatrixIndexT rows_, cols_, stride_;
  const CuGemmStatsHint *prev_;
};

/// The statistics of an affine layer's backward GEMMs in one launch set
/// (kl_gemm_stats3) -- out_deriv's rows (the data gradient's op(A)),
/// linear_params' columns (its op(B)) and, with `cols`, out_deriv's columns
/// (the weight gradient's op(A) = out_deriv^T) -- offered to those AddMatMat
/// calls as CuGemmStatsHint while in scope; without it each GEMM takes its
/// own statistics pass, two for the pair (three kernels each).  Does nothing
/// unless AddMatMat runs the f16x3 engine on these operands.  The caller
/// keeps out_deriv and linear_params unmodified while it is in scope (the
/// weight update itself is fine: the weight-gradient GEMM reads neither).
class CuGemmBackpropStats {
 public:
  /// in_value (nullable): the layer's input, whose pending column
  /// statistics (a fused pool's, CuGemmStatsHint::pending) join the launches
  CuGemmBackpropStats(const CuMatrixBase<float> &out_deriv, const CuMatrixBase<float> &linear,
                      bool cols, const CuMatrixBase<float> *in_value = NULL);
  ~CuGemmBackpropStats();
  CuGemmBackpropStats(const CuGemmBackpropStats &) = delete;
  CuGemmBackpropStats &operator=(const CuGemmBackpropStats &) = delete;

 private:
  void *ws_ = nullptr;
  CuGemmStatsHint *hint_d_ = nullptr, *hint_w_ = nullptr;  // destroyed in reverse order
};

/// Host N(0,1) generator shared by SetRandn (splitmix64 -> Box-Muller).
void RandnFill(float *dst, size_t n);
void SetRandnSeed(uint64_t seed);

}  // namespace kaldi

#endif  // KCNN_KALDI_LITE_CU_MATRIX_H_
