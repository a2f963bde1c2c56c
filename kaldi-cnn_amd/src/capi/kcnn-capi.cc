// capi/kcnn-capi.cc -- extern "C" layer of libkcnn.so (include/kcnn.h).
// Converts C++ exceptions (KALDI_ASSERT / KALDI_ERR / HIP errors) into error
// codes + kcnn_last_error(), and wraps caller device buffers as CuSubMatrix /
// borrowed CuMatrix views.
#include "kcnn.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../cnslmat/hip-util.h"
#include "../kaldi-lite/cu-device.h"
#include "../kaldi-lite/cu-kernels-lite.h"
#include "../kaldi-lite/cu-matrix.h"
#include "../kaldi-lite/kaldi-io.h"
#include "../nnet0/nnet-component-nnet0.h"
#include "../nnet2/nnet-component.h"

using namespace kaldi;
using namespace kaldi::nnet2;

struct kcnn_component {
  Component *c;
};

struct kcnn_nnet {
  std::vector<Component *> comps;
  std::vector<kcnn_component> handles;
  std::vector<CuMatrix<BaseFloat>> fwd;    // fwd[0] borrowed input, fwd[i+1] = out_i
  std::vector<CuMatrix<BaseFloat>> deriv;  // deriv[i] = d input_i
  int num_chunks = 0;
  // chunk offsets (upstream Nnet::ComputeChunkInfo): offs[i] are the frame
  // offsets of component i's input chunk, offs[i + 1] of its output, in
  // ascending order.  The last output is one frame per chunk; walking back,
  // a component's input offsets are the set of output offset + Context();
  // the network input is made contiguous; shifted so the first offset is 0.
  // Gapped contexts (SpliceComponent context=-3:0:3) make a middle layer's
  // offsets non-contiguous.
  std::vector<std::vector<int32>> offs;
  // Conv -> channel-only Maxpool pairs run fused: routing mask of pool i
  // ([rows x OutputDim] bytes), valid for the minibatch of the last Propagate
  std::vector<unsigned char *> mask;
  std::vector<size_t> mask_bytes;
  std::vector<char> mask_valid;
  // fwd[i] not stored by the fused pass (fusion mode 1; nothing in training
  // reads it): 1 = kcnn_nnet_output recomputes it on request, 2 = no longer
  // possible (the producing component's backprop may have changed its
  // parameters)
  std::vector<char> out_stale;
  // deriv[i] of a mask-fused pool not computed (fusion mode 1): the conv
  // below consumes the pool's out_deriv and mask directly; materialised by
  // kcnn_nnet_input_deriv on request, or when that conv's pass declines
  std::vector<char> deriv_deferred;
  // fwd[i]'s max |value| per row and per column from the fused forward that
  // wrote it (pool-stats.h; fstat_valid[i]), offered to the next component's
  // GEMMs (CuGemmStatsHint) for the minibatch of the last Propagate
  std::vector<uint32_t *> fstat;
  std::vector<size_t> fstat_words;
  std::vector<char> fstat_valid;
  // fwd[i]'s column statistics left pending by the fused forward (the next
  // component's FC backward runs them, pool-stats.h PoolColDeferred) and the
  // forward's per-workgroup column partials they read, kept until then
  std::vector<PoolColDeferred> fdefer;
  std::vector<void *> fpart;
  std::vector<size_t> fpart_bytes;
  ~kcnn_nnet() {
    for (auto *m : mask)
      if (m) CuDevice::Instantiate().Free(m);
    for (auto *f : fstat)
      if (f) CuDevice::Instantiate().Free(f);
    for (auto *f : fpart)
      if (f) CuDevice::Instantiate().Free(f);
    for (auto *c : comps) delete c;
  }
};

namespace {
thread_local std::string g_err;

// Runtime fusion of Conv -> Maxpool (kcnn_set_fusion; env KCNN_FUSE): 0 off,
// 1 on without storing the conv output, 2 on and the conv output stored.
int g_fusion = [] {
  const char *e = getenv("KCNN_FUSE");
  return e && *e ? atoi(e) : 1;
}();

int fail(const char *what) {
  g_err = what;
  return -1;
}

template <typename F>
int guard(F f) {
  try {
    f();
    return 0;
  } catch (const std::exception &e) {
    return fail(e.what());
  } catch (...) {
    return fail("unknown C++ exception");
  }
}

CuSubMatrix<BaseFloat> view(const float *p, MatrixDim d) {
  return CuSubMatrix<BaseFloat>(const_cast<float *>(p), d.rows, d.cols, d.stride);
}

void borrow(CuMatrix<BaseFloat> *m, const float *p, MatrixDim d) {
  m->Borrow(const_cast<float *>(p), d.rows, d.cols, d.stride);
}

ChunkInfo chunk_info(int cols, int rows, int num_chunks) {
  if (num_chunks <= 0) num_chunks = rows;
  KALDI_ASSERT(rows > 0 && rows % num_chunks == 0);
  return ChunkInfo(cols, num_chunks, 0, rows / num_chunks - 1);
}

// In/out ChunkInfos of one component call: the output chunk holds frames
// [0, out_rows/num_chunks - 1]; the input chunk is widened by the component's
// Context() (SpliceComponent; {0} for every other component).
void component_chunks(const Component *c, MatrixDim in_dim, MatrixDim out_dim,
                      int num_chunks, ChunkInfo *ii, ChunkInfo *oi) {
  const std::vector<int32> ctx = c->Context();
  if (num_chunks <= 0) num_chunks = out_dim.rows;
  KALDI_ASSERT(out_dim.rows > 0 && out_dim.rows % num_chunks == 0 &&
               in_dim.rows % num_chunks == 0);
  const int ocs = out_dim.rows / num_chunks;
  KALDI_ASSERT(in_dim.rows / num_chunks == ocs + ctx.back() - ctx.front());
  *oi = ChunkInfo(out_dim.cols, num_chunks, 0, ocs - 1);
  if (ctx.front() == 0 && ctx.back() == 0) {
    *ii = ChunkInfo(in_dim.cols, num_chunks, 0, ocs - 1);
  } else {
    // ChunkInfo offsets are >= 0 (Check): shift both by -ctx.front()
    *oi = ChunkInfo(out_dim.cols, num_chunks, -ctx.front(), ocs - 1 - ctx.front());
    *ii = ChunkInfo(in_dim.cols, num_chunks, 0, ocs - 1 + ctx.back() - ctx.front());
  }
}

void copy_out(std::string s, char *buf, size_t len) {
  if (!buf || !len) return;
  strncpy(buf, s.c_str(), len - 1);
  buf[len - 1] = '\0';
}

UpdatableComponent *updatable(const kcnn_component *c) {
  KALDI_ASSERT(c && c->c);
  UpdatableComponent *u = dynamic_cast<UpdatableComponent *>(c->c);
  if (!u) KALDI_ERR << c->c->Type() << " has no parameters";
  return u;
}

// Parameter storage of a component: linear (0), bias (1), prev_grad (2).
void param_ref(const kcnn_component *c, int which, float **data, MatrixDim *dim) {
  using cnsl::nnet0::ConvolutionComponent;
  using cnsl::nnet0::FullyConnectedComponent;
  CuMatrixBase<BaseFloat> *m = nullptr;
  CuVectorBase<BaseFloat> *v = nullptr;
  if (auto *cc = dynamic_cast<ConvolutionComponent *>(c->c)) {
    if (which == 0) m = &cc->LinearParamsMutable();
    else if (which == 1) v = &cc->BiasParamsMutable();
    else if (which == 2) m = &cc->PrevGradMutable();
  } else if (auto *fc = dynamic_cast<FullyConnectedComponent *>(c->c)) {
    if (which == 0) m = &fc->LinearParamsMutable();
    else if (which == 1) v = &fc->BiasParamsMutable();
    else if (which == 2) m = &fc->PrevGradMutable();
  } else if (auto *af = dynamic_cast<AffineComponent *>(c->c)) {
    if (which == 0) m = &af->LinearParamsMutable();
    else if (which == 1) v = &af->BiasParamsMutable();
  }
  if (m) {
    *data = m->Data();
    *dim = m->Dim();
  } else if (v) {
    *data = v->Data();
    dim->rows = 1; dim->cols = v->Dim(); dim->stride = v->Dim();
  } else {
    KALDI_ERR << c->c->Type() << " has no parameter #" << which;
  }
}

void copy2d(float *dst, MatrixDim dd, const float *src, MatrixDim sd) {
  KALDI_ASSERT(dd.rows == sd.rows && dd.cols == sd.cols);
  if (dd.rows == 0 || dd.cols == 0) return;
  CU_SAFE_CALL(hipMemcpy2DAsync(dst, sizeof(float) * dd.stride, src,
                                sizeof(float) * sd.stride,
                                sizeof(float) * dd.cols, dd.rows,
                                hipMemcpyDeviceToDevice,
                                CuDevice::Instantiate().Stream()));
}
}  // namespace

extern "C" {

const char *kcnn_last_error(void) { return g_err.c_str(); }
const char *kcnn_version(void) { return "kcnn-mi355x 0.1 (gfx950)"; }
unsigned long long kcnn_device_malloc_calls(void) {
  return (unsigned long long)CuDevice::Instantiate().MallocCalls();
}

int kcnn_init(int device) {
  return guard([&] { CuDevice::Instantiate().SelectGpuId("yes", device); });
}
int kcnn_set_stream(kcnn_stream_t stream) {
  return guard([&] {
    CuDevice::Instantiate().SetStream(reinterpret_cast<hipStream_t>(stream));
  });
}
int kcnn_synchronize(void) {
  return guard([&] { CuDevice::Instantiate().Synchronize(); });
}
int kcnn_set_literal_path(int literal) {
  cnsl::nnet0::SetLiteralPath(literal != 0);
  return 0;
}
int kcnn_set_fusion(int on) {
  if (on < 0 || on > 2) return fail("kcnn_set_fusion: mode is 0, 1 or 2");
  g_fusion = on;
  return 0;
}
int kcnn_set_gemm_mode(int mode) {
  if (mode < 0 || mode > 2) return fail("kcnn_set_gemm_mode: mode is 0, 1 or 2");
  CuDevice::Instantiate().SetGemmMode(mode);
  return 0;
}
int kcnn_set_kernel_family(const char *name, int value) {
  const int f = kcnn::family_by_name(name);
  if (f < 0) return fail("kcnn_set_kernel_family: unknown family");
  if (kcnn::set_family(static_cast<kcnn::Family>(f), value) != 0)
    return fail("kcnn_set_kernel_family: value out of range");
  return 0;
}
int kcnn_get_kernel_family(const char *name) {
  const int f = kcnn::family_by_name(name);
  return f < 0 ? -1 : kcnn::family(static_cast<kcnn::Family>(f));
}
int kcnn_gemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
              const float *a, int lda, const float *b, int ldb, float beta,
              float *c, int ldc) {
  return guard([&] {
    if (m < 0 || n < 0 || k < 0) KALDI_ERR << "kcnn_gemm: negative dimension";
    const int ar = trans_a ? k : m, ac = trans_a ? m : k;
    const int br = trans_b ? n : k, bc = trans_b ? k : n;
    if (lda < ac || ldb < bc || ldc < n) KALDI_ERR << "kcnn_gemm: leading dimension too small";
    CuSubMatrix<BaseFloat> A(const_cast<float *>(a), ar, ac, lda);
    CuSubMatrix<BaseFloat> B(const_cast<float *>(b), br, bc, ldb);
    CuSubMatrix<BaseFloat> C(c, m, n, ldc);
    C.AddMatMat(alpha, A, trans_a ? kTrans : kNoTrans, B, trans_b ? kTrans : kNoTrans, beta);
  });
}
int kcnn_split_planes(const float *src, int rows, int cols, int ld, uint16_t *dst, int ldp,
                      int64_t ps) {
  return guard([&] {
    CuDevice &d = CuDevice::Instantiate();
    const int rc = kl_split_planes(src, rows, cols, ld, dst, ldp, ps,
                                   reinterpret_cast<kcnn_stream_t>(d.Stream()));
    if (rc) KALDI_ERR << "kcnn_split_planes: " << hipGetErrorString((hipError_t)rc);
  });
}
int kcnn_gemm_planes(int trans_a, int trans_b, int m, int n, int k, float alpha,
                     const uint16_t *a, int lda, int64_t aps, const uint16_t *b, int ldb,
                     int64_t bps, float beta, float *c, int ldc) {
  return guard([&] {
    CuDevice &d = CuDevice::Instantiate();
    const size_t wsb = kl_gemm_planes_workspace_bytes(m, n, k);
    CuScratch ws_s(wsb);
    void *ws = ws_s.p;
    const int rc = kl_gemm_planes(trans_a, trans_b, m, n, k, alpha, a, lda, aps, b, ldb, bps,
                                  beta, c, ldc, ws, wsb,
                                  reinterpret_cast<kcnn_stream_t>(d.Stream()));
    if (rc) KALDI_ERR << "kcnn_gemm_planes: " << hipGetErrorString((hipError_t)rc);
  });
}
int kcnn_set_profiling(int on) {
  CuDevice::Instantiate().SetProfiling(on != 0);
  return 0;
}
int kcnn_profile_string(char *buf, size_t len) {
  return guard([&] { copy_out(CuDevice::Instantiate().ProfileString(), buf, len); });
}
int kcnn_reset_profile(void) {
  return guard([&] {
    CuDevice &d = CuDevice::Instantiate();
    (void)d.ProfileString();  // resolves and recycles the pending events
    d.ResetProfile();
  });
}
void kcnn_set_randn_seed(uint64_t seed) { SetRandnSeed(seed); }

int kcnn_selftest_fastdiv(void) {
  const uint32_t divs[] = {1, 2, 3, 5, 7, 8, 11, 24, 33, 40, 128, 363, 440,
                           1320, 11616, 46464, 65535, 1000003, 0x7fffffffu};
  uint64_t state = 12345;
  for (uint32_t d : divs) {
    kcnn::FastDiv f(d);
    for (int t = 0; t < 20000; t++) {
      state = state * 6364136223846793005ull + 1442695040888963407ull;
      uint32_t n = (uint32_t)(state >> 33);  // < 2^31
      if (t < 64) n = (uint32_t)t;
      if (t >= 64 && t < 128) n = 0x7fffffffu - (uint32_t)(t - 64);
      uint32_t q, r;
      f.divmod(n, q, r);
      if (q != n / d || r != n % d) {
        std::ostringstream ss;
        ss << "FastDiv(" << d << ") failed at n=" << n << ": " << q << "," << r;
        return fail(ss.str().c_str());
      }
    }
  }
  return 0;
}

// ---- CuMatrixBase methods -----------------------------------------------------
int kcnn_mat_conv2d(const float *in, MatrixDim in_dim, const float *kernel,
                    MatrixDim kernel_dim, int in_height, int in_width,
                    int in_channel, int kernel_height, int kernel_width,
                    int group, float *out, MatrixDim out_dim, int concat) {
  return guard([&] {
    auto x = view(in, in_dim), k = view(kernel, kernel_dim), o = view(out, out_dim);
    x.Conv2D(k, in_height, in_width, in_channel, kernel_height, kernel_width,
             group, &o, concat != 0);
  });
}
int kcnn_mat_add_mat_rep_vec(float *m, MatrixDim dim, const float *vec,
                             int vec_dim, int rep) {
  return guard([&] {
    auto x = view(m, dim);
    CuSubVector<BaseFloat> v(const_cast<float *>(vec), vec_dim);
    x.AddMatRepVec(v, rep);
  });
}
int kcnn_mat_flip_mat(const float *m, MatrixDim dim, int kernel_height,
                      int kernel_width, int in_channel, int group, float *flip,
                      MatrixDim flip_dim) {
  return guard([&] {
    auto x = view(m, dim);
    CuMatrix<BaseFloat> f;
    borrow(&f, flip, flip_dim);
    x.FlipMat(kernel_height, kernel_width, in_channel, group, &f);
  });
}
int kcnn_mat_padding_zero(const float *m, MatrixDim dim, int orig_height,
                          int orig_width, int orig_channel, int kernel_height,
                          int kernel_width, float *padmat, MatrixDim pad_dim) {
  return guard([&] {
    auto x = view(m, dim);
    CuMatrix<BaseFloat> p;
    borrow(&p, padmat, pad_dim);
    x.PaddingZero(orig_height, orig_width, orig_channel, kernel_height,
                  kernel_width, &p);
  });
}
int kcnn_mat_tp_block(const float *m, MatrixDim dim, int in_channel,
                      int block_size, float *out, MatrixDim out_dim) {
  return guard([&] {
    auto x = view(m, dim);
    CuMatrix<BaseFloat> o;
    borrow(&o, out, out_dim);
    x.TpBlock(in_channel, block_size, &o);
  });
}
int kcnn_mat_tp_inside_block(const float *m, MatrixDim dim, int group,
                             int block_size, float *out, MatrixDim out_dim) {
  return guard([&] {
    auto x = view(m, dim);
    CuMatrix<BaseFloat> o;
    borrow(&o, out, out_dim);
    x.TpInsideBlock(group, block_size, &o);
  });
}
int kcnn_mat_mod_permute_channel(float *comp, MatrixDim dim, int comp_idx,
                                 int num_component, int in_height, int in_width,
                                 float *container, MatrixDim container_dim,
                                 int from_comp_to_container) {
  return guard([&] {
    auto c = view(comp, dim);
    auto k = view(container, container_dim);
    c.ModPermuteChannel(comp_idx, num_component, in_height, in_width, &k,
                        from_comp_to_container != 0);
  });
}
int kcnn_mat_mod_permute_row(const float *m, MatrixDim dim, int in_channel,
                             int block_size, float *out, MatrixDim out_dim) {
  return guard([&] {
    auto x = view(m, dim);
    CuMatrix<BaseFloat> o;
    borrow(&o, out, out_dim);
    x.ModPermuteRow(in_channel, block_size, &o);
  });
}
int kcnn_mat_maxpool_prop(const float *in, MatrixDim in_dim, int in_height,
                          int in_width, int pool_height_dim, int pool_width_dim,
                          int pool_channel_dim, int overlap, int overlap2D,
                          float *out, MatrixDim out_dim) {
  return guard([&] {
    auto x = view(in, in_dim), o = view(out, out_dim);
    x.Maxpool_prop(in_height, in_width, pool_height_dim, pool_width_dim,
                   pool_channel_dim, overlap != 0, overlap2D != 0, &o);
  });
}
int kcnn_mat_maxpool_backprop(const float *in_value, MatrixDim in_dim,
                              const float *out_value, MatrixDim ov_dim,
                              const float *out_deriv, MatrixDim od_dim,
                              float *in_deriv, MatrixDim id_dim, int in_height,
                              int in_width, int pool_height_dim,
                              int pool_width_dim, int pool_channel_dim,
                              int overlap, int overlap2D) {
  return guard([&] {
    auto x = view(in_value, in_dim), y = view(out_value, ov_dim),
         dy = view(out_deriv, od_dim);
    CuMatrix<BaseFloat> dx;
    borrow(&dx, in_deriv, id_dim);
    x.Maxpool_backprop(y, dy, &dx, in_height, in_width, pool_height_dim,
                       pool_width_dim, pool_channel_dim, overlap != 0,
                       overlap2D != 0);
  });
}

// ---- components ------------------------------------------------------------------
kcnn_component *kcnn_component_new_from_string(const char *line) {
  kcnn_component *h = nullptr;
  guard([&] { h = new kcnn_component{Component::NewFromString(line)}; });
  return h;
}
kcnn_component *kcnn_component_read(const char *path) {
  kcnn_component *h = nullptr;
  guard([&] {
    std::ifstream is(path, std::ios::binary);
    if (!is) KALDI_ERR << "cannot open " << path;
    bool binary = false;
    if (!InitKaldiInputStream(is, &binary)) KALDI_ERR << "bad Kaldi header in " << path;
    h = new kcnn_component{Component::ReadNew(is, binary)};
  });
  return h;
}
int kcnn_component_write(const kcnn_component *c, const char *path, int binary) {
  return guard([&] {
    std::ofstream os(path, std::ios::binary);
    if (!os) KALDI_ERR << "cannot open " << path << " for writing";
    InitKaldiOutputStream(os, binary != 0);
    c->c->Write(os, binary != 0);
    if (!os) KALDI_ERR << "write failed: " << path;
  });
}
kcnn_component *kcnn_component_copy(const kcnn_component *c) {
  kcnn_component *h = nullptr;
  guard([&] { h = new kcnn_component{c->c->Copy()}; });
  return h;
}
void kcnn_component_free(kcnn_component *c) {
  if (!c) return;
  delete c->c;
  delete c;
}
int kcnn_component_type(const kcnn_component *c, char *buf, size_t len) {
  return guard([&] { copy_out(c->c->Type(), buf, len); });
}
int kcnn_component_info(const kcnn_component *c, char *buf, size_t len) {
  return guard([&] { copy_out(c->c->Info(), buf, len); });
}
int kcnn_component_input_dim(const kcnn_component *c) { return c->c->InputDim(); }
int kcnn_component_output_dim(const kcnn_component *c) { return c->c->OutputDim(); }
int kcnn_component_context(const kcnn_component *c, int *offsets, int max_len) {
  int n = -1;
  guard([&] {
    const std::vector<int32> ctx = c->c->Context();
    n = (int)ctx.size();
    for (int k = 0; k < n && k < max_len; k++) offsets[k] = ctx[k];
  });
  return n;
}
int kcnn_component_nonlinear_stats(const kcnn_component *c, double *value_sum,
                                   double *deriv_sum, int max_len, int *len,
                                   double *count) {
  return guard([&] {
    auto *nl = dynamic_cast<const kaldi::nnet2::NonlinearComponent *>(c->c);
    if (!nl) KALDI_ERR << c->c->Type() << " is not a NonlinearComponent";
    Vector<double> v, d;
    nl->GetValueSum(&v);
    nl->GetDerivSum(&d);
    *len = v.Dim();
    for (int k = 0; k < v.Dim() && k < max_len; k++) {
      value_sum[k] = v(k);
      deriv_sum[k] = d(k);
    }
    *count = nl->Count();
  });
}
int kcnn_component_backprop_needs_input(const kcnn_component *c) {
  return c->c->BackpropNeedsInput();
}
int kcnn_component_backprop_needs_output(const kcnn_component *c) {
  return c->c->BackpropNeedsOutput();
}

int kcnn_component_propagate(const kcnn_component *c, const float *in,
                             MatrixDim in_dim, float *out, MatrixDim out_dim,
                             int num_chunks) {
  return guard([&] {
    auto x = view(in, in_dim), y = view(out, out_dim);
    ChunkInfo ii, oi;
    component_chunks(c->c, in_dim, out_dim, num_chunks, &ii, &oi);
    c->c->Propagate(ii, oi, x, &y);
  });
}

int kcnn_component_backprop(kcnn_component *c, const float *in_value,
                            MatrixDim in_dim, const float *out_value,
                            MatrixDim ov_dim, const float *out_deriv,
                            MatrixDim od_dim, float *in_deriv,
                            MatrixDim id_dim, int num_chunks, int update) {
  return guard([&] {
    auto x = view(in_value, in_dim), y = view(out_value, ov_dim),
         dy = view(out_deriv, od_dim);
    ChunkInfo ii, oi;
    component_chunks(c->c, in_dim, od_dim, num_chunks, &ii, &oi);
    CuMatrix<BaseFloat> dx;
    if (in_deriv) borrow(&dx, in_deriv, id_dim);
    // the component itself, as NnetUpdater passes it: parameters for
    // updatable components, diagnostic stats for NonlinearComponents
    Component *to_update = update ? c->c : nullptr;
    c->c->Backprop(ii, oi, x, y, dy, to_update, in_deriv ? &dx : nullptr);
  });
}

int kcnn_component_param_dim(const kcnn_component *c, int which, int *rows,
                             int *cols) {
  return guard([&] {
    float *p;
    MatrixDim d;
    param_ref(c, which, &p, &d);
    *rows = d.rows;
    *cols = d.cols;
  });
}
int kcnn_component_get_param(const kcnn_component *c, int which, float *dst,
                             MatrixDim dst_dim) {
  return guard([&] {
    float *p;
    MatrixDim d;
    param_ref(c, which, &p, &d);
    copy2d(dst, dst_dim, p, d);
  });
}
int kcnn_component_set_param(kcnn_component *c, int which, const float *src,
                             MatrixDim src_dim) {
  return guard([&] {
    float *p;
    MatrixDim d;
    param_ref(c, which, &p, &d);
    copy2d(p, d, src, src_dim);
  });
}
float kcnn_component_learning_rate(const kcnn_component *c) {
  float lr = -1.0f;
  guard([&] { lr = updatable(c)->LearningRate(); });
  return lr;
}
int kcnn_component_set_learning_rate(kcnn_component *c, float lr) {
  return guard([&] { updatable(c)->SetLearningRate(lr); });
}
int kcnn_component_dot_product(const kcnn_component *a, const kcnn_component *b,
                               float *out) {
  return guard([&] { *out = updatable(a)->DotProduct(*updatable(b)); });
}
int kcnn_component_set_zero(kcnn_component *c, int treat_as_gradient) {
  return guard([&] { updatable(c)->SetZero(treat_as_gradient != 0); });
}
int kcnn_component_scale(kcnn_component *c, float scale) {
  return guard([&] { updatable(c)->Scale(scale); });
}
int kcnn_component_add(kcnn_component *c, float alpha, const kcnn_component *other) {
  return guard([&] { updatable(c)->Add(alpha, *updatable(other)); });
}
int kcnn_component_perturb_params(kcnn_component *c, float stddev) {
  return guard([&] { updatable(c)->PerturbParams(stddev); });
}
int kcnn_component_num_gradient_params(const kcnn_component *c) {
  auto *u = dynamic_cast<UpdatableComponent *>(c->c);
  return u ? u->NumGradientParams() : 0;
}
int kcnn_component_compute_gradient(const kcnn_component *c,
                                    const float *in_value, MatrixDim in_dim,
                                    const float *out_deriv, MatrixDim od_dim,
                                    float *grad) {
  return guard([&] {
    updatable(c)->ComputeGradient(view(in_value, in_dim), view(out_deriv, od_dim),
                                  grad);
  });
}
int kcnn_component_apply_gradient(kcnn_component *c, const float *grad,
                                  int num_sample) {
  return guard([&] { updatable(c)->ApplyGradient(grad, num_sample); });
}
int kcnn_component_backprop_gradient(const kcnn_component *c,
                                     const float *in_value, MatrixDim in_dim,
                                     const float *out_deriv, MatrixDim od_dim,
                                     float *in_deriv, MatrixDim id_dim,
                                     float *grad) {
  return guard([&] {
    const UpdatableComponent *u = updatable(c);
    ChunkInfo ii = chunk_info(in_dim.cols, in_dim.rows, 0);
    ChunkInfo oi = chunk_info(od_dim.cols, od_dim.rows, 0);
    auto x = view(in_value, in_dim);
    CuMatrix<BaseFloat> dx;
    if (in_deriv) borrow(&dx, in_deriv, id_dim);
    u->BackpropGradient(ii, oi, x, x, view(out_deriv, od_dim),
                        in_deriv ? &dx : nullptr, grad);
  });
}
int kcnn_component_conv_flip_branch(const kcnn_component *c) {
  auto *cc = dynamic_cast<cnsl::nnet0::ConvolutionComponent *>(c->c);
  if (!cc) return fail("not a ConvolutionComponent");
  return cc->FlipKernelBranch() ? 1 : 0;
}

// ---- component stack ---------------------------------------------------------------
kcnn_nnet *kcnn_nnet_new(const char *config) {
  std::unique_ptr<kcnn_nnet> n(new kcnn_nnet());
  int rc = guard([&] {
    std::istringstream is(config);
    std::string line;
    while (std::getline(is, line)) {
      const size_t b = line.find_first_not_of(" \t\r");
      if (b == std::string::npos || line[b] == '#') continue;
      n->comps.push_back(Component::NewFromString(line.substr(b)));
    }
    if (n->comps.empty()) KALDI_ERR << "empty nnet config";
    for (size_t i = 0; i + 1 < n->comps.size(); i++)
      if (n->comps[i]->OutputDim() != n->comps[i + 1]->InputDim())
        KALDI_ERR << "dimension mismatch between component " << i << " ("
                  << n->comps[i]->OutputDim() << ") and " << i + 1 << " ("
                  << n->comps[i + 1]->InputDim() << ")";
    const size_t nc = n->comps.size();
    n->offs.assign(nc + 1, std::vector<int32>());
    n->offs[nc].assign(1, 0);
    for (size_t k = nc; k-- > 0;) {
      const std::vector<int32> ctx = n->comps[k]->Context();
      std::set<int32> in;
      for (int32 o : n->offs[k + 1])
        for (int32 c : ctx) in.insert(o + c);
      n->offs[k].assign(in.begin(), in.end());
    }
    {  // MakeOffsetsContiguous on the network input
      const int32 lo = n->offs[0].front(), hi = n->offs[0].back();
      n->offs[0].clear();
      for (int32 o = lo; o <= hi; o++) n->offs[0].push_back(o);
    }
    // ChunkInfo offsets must be >= 0: shift everything by -first input offset
    const int32 shift = -n->offs[0].front();
    for (auto &v : n->offs)
      for (auto &o : v) o += shift;
    for (auto *c : n->comps) n->handles.push_back(kcnn_component{c});
    n->fwd.resize(n->comps.size() + 1);
    n->deriv.resize(n->comps.size());
    n->mask.assign(n->comps.size(), nullptr);
    n->mask_bytes.assign(n->comps.size(), 0);
    n->mask_valid.assign(n->comps.size(), 0);
    n->out_stale.assign(n->comps.size() + 1, 0);
    n->fstat.assign(n->comps.size() + 1, nullptr);
    n->fstat_words.assign(n->comps.size() + 1, 0);
    n->fstat_valid.assign(n->comps.size() + 1, 0);
    n->fdefer.assign(n->comps.size() + 1, PoolColDeferred{});
    n->fpart.assign(n->comps.size() + 1, nullptr);
    n->fpart_bytes.assign(n->comps.size() + 1, 0);
    n->deriv_deferred.assign(n->comps.size(), 0);
  });
  return rc ? nullptr : n.release();
}
void kcnn_nnet_free(kcnn_nnet *n) { delete n; }
int kcnn_nnet_num_components(const kcnn_nnet *n) { return (int)n->comps.size(); }
kcnn_component *kcnn_nnet_component(kcnn_nnet *n, int i) {
  if (i < 0 || i >= (int)n->handles.size()) return nullptr;
  return &n->handles[i];
}

static ChunkInfo nnet_in_info(const kcnn_nnet *n, size_t i) {
  return ChunkInfo(n->comps[i]->InputDim(), n->num_chunks, n->offs[i]);
}
static ChunkInfo nnet_out_info(const kcnn_nnet *n, size_t i) {
  return ChunkInfo(n->comps[i]->OutputDim(), n->num_chunks, n->offs[i + 1]);
}

// The non-virtual Component::Propagate's sizing (nnet-component.h:203-215):
// resize (zero-filled) only when the size differs.
static void size_output(CuMatrix<BaseFloat> *m, int rows, int cols) {
  if (m->NumRows() != rows || m->NumCols() != cols) m->Resize(rows, cols);
}

// The statistics of component i's input (fwd[i]) while its Propagate /
// Backprop runs, when the fused forward that wrote it gave them.
static std::unique_ptr<CuGemmStatsHint> input_stats(const kcnn_nnet *n, size_t i) {
  if (i >= n->fstat_valid.size() || !n->fstat_valid[i]) return nullptr;
  const CuMatrix<BaseFloat> &x = n->fwd[i];
  std::unique_ptr<CuGemmStatsHint> h(new CuGemmStatsHint(
      x.Data(), x.NumRows(), x.NumCols(), x.Stride(), n->fstat[i],
      n->fstat[i] + 3 * (size_t)x.NumRows()));
  if (n->fdefer[i].pending) h->pending = const_cast<PoolColDeferred *>(&n->fdefer[i]);
  return h;
}

// Component i (Conv) and i+1 (channel-only Maxpool) in one fused pass;
// false when the pair does not qualify.
static bool propagate_pair(kcnn_nnet *n, size_t i) {
  using cnsl::nnet0::ConvolutionComponent;
  using cnsl::nnet0::MaxpoolComponent;
  if (!g_fusion || i + 1 >= n->comps.size()) return false;
  auto *conv = dynamic_cast<ConvolutionComponent *>(n->comps[i]);
  auto *pool = dynamic_cast<MaxpoolComponent *>(n->comps[i + 1]);
  if (!conv || !pool) return false;
  const int mask_bytes = pool->FusedMaskBytes();  // 1: channel-only, 2: 3-D window
  if (mask_bytes == 0) return false;
  const int rows = n->fwd[i].NumRows();
  const size_t need = (size_t)rows * pool->OutputDim() * mask_bytes;
  if (n->mask_bytes[i + 1] < need) {
    if (n->mask[i + 1]) CuDevice::Instantiate().Free(n->mask[i + 1]);
    n->mask[i + 1] = static_cast<unsigned char *>(CuDevice::Instantiate().Malloc(need));
    n->mask_bytes[i + 1] = need;
  }
  size_output(&n->fwd[i + 1], rows, conv->OutputDim());
  size_output(&n->fwd[i + 2], rows, pool->OutputDim());
  const bool store = g_fusion == 2;
  // room for the pooled output's statistics (the row block [max, min, cnt]
  // and the column block [max, min, cnt], kept) and the kernel's column
  // partials (this call only)
  PoolStatsOut ps;
  const size_t pw = mask_bytes == 1 && conv->In_pad_height() == 0 && conv->In_pad_width() == 0
                        ? kcnn_conv2d_maxpool_stats_words(
                              rows, conv->In_height(), conv->In_width(), conv->In_channels(),
                              conv->Kernel_height(), conv->Kernel_width(), conv->Group(),
                              pool->FusableChannelPool())
                        : 0;
  if (pw && n->fpart_bytes[i + 2] < pw * 4) {  // kept: the column work may run in the backward
    if (n->fpart[i + 2]) CuDevice::Instantiate().Free(n->fpart[i + 2]);
    n->fpart[i + 2] = CuDevice::Instantiate().Malloc(pw * 4);
    n->fpart_bytes[i + 2] = pw * 4;
  }
  n->fdefer[i + 2].pending = 0;
  if (pw) {
    const size_t need = 3 * ((size_t)rows + pool->OutputDim());
    if (n->fstat_words[i + 2] < need) {
      if (n->fstat[i + 2]) CuDevice::Instantiate().Free(n->fstat[i + 2]);
      n->fstat[i + 2] = static_cast<uint32_t *>(CuDevice::Instantiate().Malloc(need * 4));
      n->fstat_words[i + 2] = need;
    }
    ps.rowmax = n->fstat[i + 2];
    ps.colmax = n->fstat[i + 2] + 3 * (size_t)rows;
    ps.partials = static_cast<uint32_t *>(n->fpart[i + 2]);
    ps.partial_words = pw;
  }
  {
    PoolColDeferScope defer(pw ? &n->fdefer[i + 2] : nullptr);
    if (!conv->PropagateMaxpool(n->fwd[i], &n->fwd[i + 1], *pool, &n->fwd[i + 2],
                                n->mask[i + 1], pool->OutputDim(), store, pw ? &ps : nullptr))
      return false;
  }
  n->fstat_valid[i + 2] = ps.produced;
  n->mask_valid[i + 1] = 1;
  n->out_stale[i + 1] = !store;
  return true;
}

// Component i (Conv) and i+1 (RectifiedLinearComponent) in one pass, fusion
// mode 1 only: the conv output (the ReLU's in_value, which its Backprop does
// not read) is left unstored; false when the pair does not qualify.
static bool propagate_relu_pair(kcnn_nnet *n, size_t i) {
  if (g_fusion != 1 || i + 1 >= n->comps.size()) return false;
  auto *conv = dynamic_cast<cnsl::nnet0::ConvolutionComponent *>(n->comps[i]);
  auto *relu = dynamic_cast<kaldi::nnet2::RectifiedLinearComponent *>(n->comps[i + 1]);
  if (!conv || !relu || relu->InputDim() != conv->OutputDim()) return false;
  const int rows = n->fwd[i].NumRows();
  size_output(&n->fwd[i + 1], rows, conv->OutputDim());
  size_output(&n->fwd[i + 2], rows, relu->OutputDim());
  if (!conv->PropagateRelu(n->fwd[i], &n->fwd[i + 2])) return false;
  n->out_stale[i + 1] = 1;
  return true;
}

int kcnn_nnet_propagate(kcnn_nnet *n, const float *in, MatrixDim in_dim) {
  return guard([&] {
    KALDI_ASSERT(in_dim.cols == n->comps[0]->InputDim());
    const int in_cs = (int)n->offs[0].size();
    if (in_dim.rows % in_cs != 0)
      KALDI_ERR << "input rows " << in_dim.rows << " are not a multiple of the "
                << in_cs << "-frame input chunk";
    borrow(&n->fwd[0], in, in_dim);
    n->num_chunks = in_dim.rows / in_cs;
    std::fill(n->mask_valid.begin(), n->mask_valid.end(), 0);
    std::fill(n->out_stale.begin(), n->out_stale.end(), 0);
    std::fill(n->deriv_deferred.begin(), n->deriv_deferred.end(), 0);
    std::fill(n->fstat_valid.begin(), n->fstat_valid.end(), 0);
    for (auto &d : n->fdefer) d.pending = 0;
    for (size_t i = 0; i < n->comps.size(); i++) {
      if (propagate_pair(n, i) || propagate_relu_pair(n, i)) { i++; continue; }
      ChunkInfo ii = nnet_in_info(n, i), oi = nnet_out_info(n, i);
      auto hint = input_stats(n, i);
      n->comps[i]->Propagate(ii, oi, n->fwd[i], &n->fwd[i + 1]);
    }
  });
}

int kcnn_nnet_output(const kcnn_nnet *n, int i, const float **data,
                     MatrixDim *dim) {
  return guard([&] {
    KALDI_ASSERT(i >= -1 && i < (int)n->comps.size());
    if (n->out_stale[i + 1] == 2)
      KALDI_ERR << "output of component " << i << " was not stored (fused with the "
                << "next Maxpool, kcnn_set_fusion(1)) and its backprop has run; "
                << "use kcnn_set_fusion(2) to keep it";
    if (n->out_stale[i + 1]) {  // a fused conv's output: run its Propagate now
      kcnn_nnet *nm = const_cast<kcnn_nnet *>(n);
      nm->comps[i]->Propagate(nnet_in_info(nm, i), nnet_out_info(nm, i), nm->fwd[i],
                              &nm->fwd[i + 1]);
      nm->out_stale[i + 1] = 0;
    }
    const CuMatrix<BaseFloat> &m = n->fwd[i + 1];
    *data = m.Data();
    *dim = m.Dim();
  });
}

// A deferred pool Backprop (see kcnn_nnet::deriv_deferred), run now.
static void materialise_pool_deriv(kcnn_nnet *n, int i) {
  auto *pool = dynamic_cast<cnsl::nnet0::MaxpoolComponent *>(n->comps[i]);
  KALDI_ASSERT(pool != NULL && n->mask_valid[i] && i + 1 < (int)n->comps.size());
  CuMatrix<BaseFloat> &od = n->deriv[i + 1];
  pool->BackpropFromMask(n->mask[i], pool->OutputDim(),
                         CuSubMatrix<BaseFloat>(od.Data(), od.NumRows(), od.NumCols(),
                                                od.Stride()),
                         &n->deriv[i]);
  n->deriv_deferred[i] = 0;
}

int kcnn_nnet_input_deriv(const kcnn_nnet *n, int i, const float **data,
                          MatrixDim *dim) {
  return guard([&] {
    KALDI_ASSERT(i >= 0 && i < (int)n->comps.size());
    if (n->deriv_deferred[i]) materialise_pool_deriv(const_cast<kcnn_nnet *>(n), i);
    const CuMatrix<BaseFloat> &m = n->deriv[i];
    *data = m.Data();
    *dim = m.Dim();
  });
}

int kcnn_nnet_backprop_component(kcnn_nnet *n, int i, const float *out_deriv,
                                 MatrixDim od_dim, int mode, float *grad,
                                 int skip_first_dx) {
  return guard([&] {
    const int nc = (int)n->comps.size();
    KALDI_ASSERT(i >= 0 && i < nc);
    Component *c = n->comps[i];
    auto hint = input_stats(n, i);
    if (n->out_stale[i + 1]) n->out_stale[i + 1] = 2;
    auto *u = dynamic_cast<UpdatableComponent *>(c);
    CuMatrix<BaseFloat> *dx = &n->deriv[i];
    if (i == 0 && skip_first_dx && u) dx = nullptr;
    if (mode == 3) {  // the parameter gradient alone (a later mode 2 call adds dX)
      KALDI_ASSERT(u != NULL && grad != NULL &&
                   !(i + 1 < nc && n->deriv_deferred[i + 1]) && !n->mask_valid[i]);
      CuSubMatrix<BaseFloat> od = (i == nc - 1)
          ? view(out_deriv, od_dim)
          : CuSubMatrix<BaseFloat>(n->deriv[i + 1].Data(), n->deriv[i + 1].NumRows(),
                                   n->deriv[i + 1].NumCols(), n->deriv[i + 1].Stride());
      u->BackpropGradient(nnet_in_info(n, i), nnet_out_info(n, i), n->fwd[i], n->fwd[i + 1],
                          od, nullptr, grad);
      return;
    }
    if (i + 1 < nc && n->deriv_deferred[i + 1]) {  // pool above left its Backprop here
      auto *conv = dynamic_cast<cnsl::nnet0::ConvolutionComponent *>(c);
      auto *pool = dynamic_cast<cnsl::nnet0::MaxpoolComponent *>(n->comps[i + 1]);
      CuMatrix<BaseFloat> &pd = n->deriv[i + 2];
      CuSubMatrix<BaseFloat> pod(pd.Data(), pd.NumRows(), pd.NumCols(), pd.Stride());
      if (conv && pool &&
          conv->BackpropPooled(n->fwd[i], *pool, n->mask[i + 1], pool->OutputDim(), pod,
                               mode == 0 ? c : nullptr, dx, mode == 1 ? grad : nullptr))
        return;
      materialise_pool_deriv(n, i + 1);
    }
    CuSubMatrix<BaseFloat> od = (i == nc - 1)
        ? view(out_deriv, od_dim)
        : CuSubMatrix<BaseFloat>(n->deriv[i + 1].Data(), n->deriv[i + 1].NumRows(),
                                 n->deriv[i + 1].NumCols(), n->deriv[i + 1].Stride());
    ChunkInfo ii = nnet_in_info(n, i), oi = nnet_out_info(n, i);
    if (mode == 1 && u) {
      u->BackpropGradient(ii, oi, n->fwd[i], n->fwd[i + 1], od, dx, grad);
      return;
    }
    if (n->mask_valid[i]) {  // pool of a fused pair: route through its mask
      auto *pool = dynamic_cast<cnsl::nnet0::MaxpoolComponent *>(c);
      KALDI_ASSERT(pool != NULL);
      // mode 1, not the last component: left to the conv below, which
      // builds its out_deriv from od and the mask slab by slab
      if (g_fusion == 1 && i < nc - 1 && pool->FoldsIntoConvBackprop()) {
        n->deriv_deferred[i] = 1;
        return;
      }
      pool->BackpropFromMask(n->mask[i], pool->OutputDim(), od, dx);
      return;
    }
    // NnetUpdater passes every component as to_update: updatable ones only
    // update in mode 0; NonlinearComponent stats (per replica) always
    Component *to_update = (mode == 0 || !u) ? c : nullptr;
    c->Backprop(ii, oi, n->fwd[i], n->fwd[i + 1], od, to_update, dx);
  });
}

// An affine layer's parameter gradient, then between(ctx) (the caller starts
// its all-reduce there), then the layer's data gradient: mode 3 and mode 2 in
// one call, so both GEMMs' operand statistics come from one launch set that
// lives across the callback (the pair of calls computed them twice).
int kcnn_nnet_backprop_split(kcnn_nnet *n, int i, const float *out_deriv, MatrixDim od_dim,
                             float *grad, int skip_first_dx, void (*between)(void *),
                             void *ctx) {
  return guard([&] {
    const int nc = (int)n->comps.size();
    KALDI_ASSERT(i >= 0 && i < nc && grad != NULL);
    Component *c = n->comps[i];
    auto *af = dynamic_cast<kaldi::nnet2::AffineComponent *>(c);
    if (af == NULL) KALDI_ERR << "kcnn_nnet_backprop_split: component " << i << " is not affine";
    KALDI_ASSERT(!(i + 1 < nc && n->deriv_deferred[i + 1]) && !n->mask_valid[i]);
    auto hint = input_stats(n, i);
    if (n->out_stale[i + 1]) n->out_stale[i + 1] = 2;
    CuSubMatrix<BaseFloat> od = (i == nc - 1)
        ? view(out_deriv, od_dim)
        : CuSubMatrix<BaseFloat>(n->deriv[i + 1].Data(), n->deriv[i + 1].NumRows(),
                                 n->deriv[i + 1].NumCols(), n->deriv[i + 1].Stride());
    CuMatrix<BaseFloat> *dx = (i == 0 && skip_first_dx) ? nullptr : &n->deriv[i];
    ChunkInfo ii = nnet_in_info(n, i), oi = nnet_out_info(n, i);
    CuGemmBackpropStats stats(od, af->LinearParams(), true, &n->fwd[i]);
    af->BackpropGradient(ii, oi, n->fwd[i], n->fwd[i + 1], od, nullptr, grad);
    if (between) between(ctx);
    if (dx) c->Backprop(ii, oi, n->fwd[i], n->fwd[i + 1], od, nullptr, dx);
  });
}

int kcnn_nnet_backprop(kcnn_nnet *n, const float *out_deriv, MatrixDim od_dim) {
  for (int i = (int)n->comps.size() - 1; i >= 0; i--) {
    int rc = kcnn_nnet_backprop_component(n, i, out_deriv, od_dim, 0, nullptr, 0);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
