// kaldi-lite/cu-device.h -- device singleton of the MI355X build.
//
// Upstream Kaldi's CuDevice (cudamatrix/cu-device.h) selects the GPU, owns
// the cuBLAS handle and a caching allocator and accumulates per-function
// profile times (AccuProfile, used around every launch in conv2D.cc:110 ff.).
// This one does the same for HIP/ROCm, with three MI355X-first changes:
//   - one explicit hipStream_t that every kernel of the library is launched
//     on (settable, so a host framework can hand its own stream in);
//   - a caching allocator whose blocks are reused in stream order (no
//     hipMalloc / hipFree in steady state, which would serialise the device);
//   - profiling through hipEvents around the launches (the reference's Timer
//     measured launch latency only).
// There is no CPU mode: Enabled() is always true once a device is selected,
// and selecting "no" throws -- the product path has no CPU fallback.
#ifndef KCNN_KALDI_LITE_CU_DEVICE_H_
#define KCNN_KALDI_LITE_CU_DEVICE_H_

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "kaldi-common.h"
#include "kcnn-knobs.h"

namespace kaldi {

#define CU_SAFE_CALL(expr)                                               \
  do {                                                                   \
    hipError_t e__ = (expr);                                             \
    if (e__ != hipSuccess)                                               \
      KALDI_ERR << "HIP error " << (int)e__ << " (" << hipGetErrorString(e__) \
                << ") in " << #expr;                                     \
  } while (0)

#define CNSL_SAFE_CALL(expr)                                            \
  do {                                                                  \
    int e__ = (expr);                                                   \
    if (e__ != 0)                                                       \
      KALDI_ERR << "kernel launch failed: " << #expr << " -> HIP error " \
                << e__ << " (" << hipGetErrorString((hipError_t)e__) << ")"; \
  } while (0)

class CuDevice {
 public:
  static CuDevice &Instantiate();

  // "yes"/"optional"/"wait": use device `device_id` (or the current one if
  // < 0); "no": throws (no CPU path in this build).
  void SelectGpuId(const std::string &use_gpu, int device_id = -1);
  bool Enabled() const { return active_device_ >= 0; }
  int ActiveDevice() const { return active_device_; }

  hipStream_t Stream() { EnsureInit(); return stream_; }
  void SetStream(hipStream_t s);
  rocblas_handle GetBlasHandle() { EnsureInit(); return blas_; }

  // Caching allocator (stream-ordered reuse on Stream()).
  void *Malloc(size_t bytes);
  void Free(void *ptr);
  // Malloc calls so far (a HIP graph captured over cached blocks is replayed
  // safely only while none is made: bench.py --graph checks it)
  uint64_t MallocCalls();
  void ReleaseCache();
  size_t BytesInUse() const { return bytes_in_use_; }
  size_t BytesCached() const { return bytes_cached_; }


  // Profiling: per-function accumulated kernel milliseconds, measured with
  // hipEvents when enabled (KCNN_PROFILE=1 or SetProfiling(true)).
  void SetProfiling(bool on) { profiling_ = on; }
  bool Profiling() const { return profiling_; }
  void AccuProfile(const std::string &key, double ms);
  void AccuProfileLocked(const std::string &key, double ms);  // caller holds the profile lock
  std::string ProfileString() const;
  void ResetProfile() { profile_.clear(); }

  // AddMatMat's fp32 product: 0 = rocBLAS sgemm, 1 = bf16x6 split kernel,
  // 2 = f16x3 split kernel (the "gemm" kernel family, kcnn-knobs.h)
  void SetGemmMode(int m) { kcnn::set_family(kcnn::kFamGemm, m); }
  int GemmMode() const { return kcnn::family(kcnn::kFamGemm); }

  void Synchronize();

 private:
  CuDevice();
  ~CuDevice();
  void EnsureInit();

  int active_device_ = -1;
  hipStream_t stream_ = nullptr;
  rocblas_handle blas_ = nullptr;
  bool profiling_ = false;
  std::map<std::string, std::pair<double, long>> profile_;

  std::mutex mu_;
  std::multimap<size_t, void *> free_blocks_;
  std::map<void *, size_t> live_blocks_;
  size_t bytes_in_use_ = 0, bytes_cached_ = 0;
  uint64_t malloc_calls_ = 0;
};

// Per-call scratch (split-K partials, GEMM workspaces) from the caching
// allocator, freed at scope exit.  Every call owns its block, so concurrent
// const Propagate / Backprop calls from several host threads never share one
// (SURVEY 8(b) Threading: nnet-train-parallel runs them multi-threaded); the
// allocator's stream-ordered reuse keeps a freed block away from kernels
// still to run on Stream().
struct CuScratch {
  void *p = nullptr;
  explicit CuScratch(size_t bytes) {
    if (bytes) p = CuDevice::Instantiate().Malloc(bytes);
  }
  ~CuScratch() { if (p) CuDevice::Instantiate().Free(p); }
  CuScratch(const CuScratch &) = delete;
  CuScratch &operator=(const CuScratch &) = delete;
  float *f() { return static_cast<float *>(p); }
};

// Times a scope with hipEvents on the device stream when profiling is on.
class CuProfileScope {
 public:
  explicit CuProfileScope(const char *key);
  ~CuProfileScope();
  // nothing launched after all (e.g. a fused path declined): record nothing
  void Cancel();

 private:
  const char *key_;
  hipEvent_t beg_ = nullptr, end_ = nullptr;
};

}  // namespace kaldi

#endif  // KCNN_KALDI_LITE_CU_DEVICE_H_
